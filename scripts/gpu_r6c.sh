# Round-6 GPU session c: ResNet-50 numerics at the bench's shapes (fp64-bound per GEMM + 20-step loss trajectory).
set -o pipefail
mkdir -p gpurun_out/r6c
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_resnet_accuracy_gpu.py > gpurun_out/r6c/t.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r6c/t.log | head -20; tail -30 gpurun_out/r6c/t.log; exit 1; }
grep -E "worst|resnet50:" gpurun_out/r6c/t.log | tail -60
tail -3 gpurun_out/r6c/t.log
