set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_a.log 2>&1 || { tail -60 gpurun_out/gputest_a.log; exit 1; }
tail -2 gpurun_out/gputest_a.log
for lb in 256 32; do bash scripts/ab_env.sh CDP_STAGGER "0 1" 3 --local-batch $lb || exit 1; done
