# Round-6 GPU session f: fused tail / split-K BN tests, model tests, then the 32/64/256-image step
# A/B of the split-K + BN one-launch path and a 32-image kernel profile.
set -o pipefail
mkdir -p gpurun_out/r6f
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fused_tail_gpu.py tests/test_model_gpu.py tests/test_accuracy_gpu.py -k "not loss_curve" > gpurun_out/r6f/t.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r6f/t.log | head -20; tail -30 gpurun_out/r6f/t.log; exit 1; }
tail -3 gpurun_out/r6f/t.log
for lb in 32 64 256; do
  for rep in 1 2; do
    for f in 0 1; do
      CDP_SPLITK_FIN=$f timeout -k 10 150 python bench.py --local-batch $lb --steps 100 --warmup 10 --no-extra > gpurun_out/r6f/b.log 2>&1 || { tail -20 gpurun_out/r6f/b.log; exit 1; }
      python -c "import json; r=json.loads([l for l in open('gpurun_out/r6f/b.log') if l.startswith('{')][-1]); print($lb, 'splitk_fin=$f', r['ms_per_step'])"
    done
  done
done
bash scripts/prof_bench.sh r6f_b32 10 --local-batch 32
