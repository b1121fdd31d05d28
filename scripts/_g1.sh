set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bdef.log 2>&1 || { tail -30 gpurun_out/bdef.log; exit 1; }
tail -1 gpurun_out/bdef.log
bash scripts/prof_bench.sh b32 10 --local-batch 32 || exit 1
for lb in 32 256; do bash scripts/ab_env.sh CDP_BWD_PAIR "0 1" 2 --local-batch $lb || exit 1; done
timeout -k 10 600 python scripts/sweep_gemm.py --batches 32,256 > gpurun_out/sweep.log 2>&1 || { tail -20 gpurun_out/sweep.log; exit 1; }
tail -3 gpurun_out/sweep.log
