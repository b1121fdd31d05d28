set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_accuracy_gpu.py -x -q -k "256x256 or headline" --timeout 200 --timeout-method thread > gpurun_out/gputest_b.log 2>&1 || { tail -60 gpurun_out/gputest_b.log; exit 1; }
tail -2 gpurun_out/gputest_b.log
timeout -k 10 600 python scripts/sweep_gemm.py --batches 256,128,64 --layers 2,3,4,5 --ops fwd,dgrad --tiles 256x256,256x128,128x128 --out gpurun_out/sweep256.json > gpurun_out/sweep256.log 2>&1 || { tail -20 gpurun_out/sweep256.log; exit 1; }
cat gpurun_out/sweep256.log
