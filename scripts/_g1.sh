set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_a.log 2>&1 || { tail -60 gpurun_out/gputest_a.log; exit 1; }
tail -2 gpurun_out/gputest_a.log
for lb in 32 64 128 256; do bash scripts/ab_env.sh CDP_PLANNER "legacy model" 2 --local-batch $lb || exit 1; done
CDP_PLANNER=legacy bash scripts/prof_bench.sh p128L 6 --local-batch 128 || exit 1
CDP_PLANNER=model bash scripts/prof_bench.sh p128M 6 --local-batch 128 || exit 1
bash scripts/pmc_layers.sh pl256 256 || exit 1
bash scripts/pmc_layers.sh pl32 32 || exit 1
