set -o pipefail
mkdir -p gpurun_out
for lb in 32 64 128 256; do bash scripts/ab_env.sh CDP_PLANNER "legacy model" 2 --local-batch $lb || exit 1; done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bdef.log 2>&1 || { tail -30 gpurun_out/bdef.log; exit 1; }
tail -1 gpurun_out/bdef.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { tail -60 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
