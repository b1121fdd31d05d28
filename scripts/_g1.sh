set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { tail -60 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bdef.log 2>&1 || { tail -30 gpurun_out/bdef.log; exit 1; }
tail -1 gpurun_out/bdef.log
for lb in 256 32; do bash scripts/ab_env.sh CDP_BWD_PAIR "0 1" 2 --local-batch $lb || exit 1; done
bash scripts/prof_bench.sh b32 10 --local-batch 32 || exit 1
