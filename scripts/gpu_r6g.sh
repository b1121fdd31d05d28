# Round-6 GPU session g: fused classifier tail (xent + fc1 backward + the last block's BN reduction
# in one launch) -- same-box A/B at 32 / 64 / 256 images, then the 32-image kernel profile.
set -o pipefail
mkdir -p gpurun_out/r6g
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fused_tail_gpu.py > gpurun_out/r6g/t.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r6g/t.log | head -20; tail -30 gpurun_out/r6g/t.log; exit 1; }
tail -2 gpurun_out/r6g/t.log
for lb in 32 64 256; do
  for rep in 1 2 3; do
    for f in 0 1; do
      CDP_FUSED_CLASSIFIER=$f timeout -k 10 150 python bench.py --local-batch $lb --steps 100 --warmup 10 --no-extra > gpurun_out/r6g/b.log 2>&1 || { tail -20 gpurun_out/r6g/b.log; exit 1; }
      python -c "import json; r=json.loads([l for l in open('gpurun_out/r6g/b.log') if l.startswith('{')][-1]); print($lb, 'fused_classifier=$f', r['ms_per_step'])"
    done
  done
done
bash scripts/prof_bench.sh r6g_b32 10 --local-batch 32
