set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 180 python bench.py > gpurun_out/b1.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/b1.log; exit 1; }
tail -1 gpurun_out/b1.log
bash scripts/prof_bench.sh r3d_b256 6 || exit 1
bash scripts/prof_bench.sh r3d_b32 10 --local-batch 32 || exit 1
