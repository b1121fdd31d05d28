# Round-6 GPU session d: fused classifier tail tests + the model-level GPU tests that run through it.
set -o pipefail
mkdir -p gpurun_out/r6d
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fused_tail_gpu.py tests/test_model_gpu.py > gpurun_out/r6d/t.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r6d/t.log | head -20; tail -30 gpurun_out/r6d/t.log; exit 1; }
tail -3 gpurun_out/r6d/t.log
