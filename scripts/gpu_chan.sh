set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_model.log 2>&1 || { echo "model tests failed"; tail -40 gpurun_out/t_model.log; exit 1; }
tail -3 gpurun_out/t_model.log
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/b_chan.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/b_chan.log; exit 1; }
tail -1 gpurun_out/b_chan.log
CDP_CHAN=0 timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/b_nochan.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/b_nochan.log; exit 1; }
tail -1 gpurun_out/b_nochan.log
