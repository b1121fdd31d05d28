# Round-6 GPU session m: early buffer broadcast (DistributedDataParallel.early_buffer_broadcast):
# bitwise tests (overlap / early / both, eager + replay), the comm and multi-rank tests, then a
# same-box A/B at 32 and 256 images with the modelled 8-rank xGMI collectives (one rank standing in
# for W = 8: every all-reduce alpha + 2(W-1)/W S/B, every broadcast alpha + S/B on the comm stream).
set -o pipefail
mkdir -p gpurun_out/r6m
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_step_overlap_gpu.py tests/test_comm_gpu.py tests/test_multirank_gpu.py > gpurun_out/r6m/t.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r6m/t.log | head -20; tail -40 gpurun_out/r6m/t.log; exit 1; }
tail -2 gpurun_out/r6m/t.log
export CDP_BENCH_DDP_W1=1 CDP_REDUCER_TEST_POSTOP=xgmi:20:100:8
for lb in 32 256; do
for rep in 1 2 3; do
  for fl in "" "--early-bcast" "--early-bcast --overlap-step"; do
    timeout -k 10 150 python bench.py --local-batch $lb --steps 60 --warmup 10 --no-extra --bucket-cap-mb 10 $fl > gpurun_out/r6m/b.log 2>&1 || { tail -20 gpurun_out/r6m/b.log; exit 1; }
    python -c "import json; r=json.loads([l for l in open('gpurun_out/r6m/b.log') if l.startswith('{')][-1]); c=r['config']; print($lb, 'early' if c['early_buffer_broadcast'] else 'fwd-start', 'overlap' if c['optimizer_overlap'] else '', r['ms_per_step'])"
  done
done
done
