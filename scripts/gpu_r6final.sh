# Final-tree rehearsal of the driver's N > 1 bench on the one GPU: 2 ranks over gloo on cuda:0 through the
# per-rank supervisor (headline first, then each extra in fresh workers), one JSON line from rank 0.
set -o pipefail
mkdir -p gpurun_out/r6final
timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --local-batch 64 > gpurun_out/r6final/b2g.log 2>&1 || { tail -30 gpurun_out/r6final/b2g.log; exit 1; }
grep -c '^{' gpurun_out/r6final/b2g.log
tail -1 gpurun_out/r6final/b2g.log | cut -c1-1500
