# Round-6 GPU session h: tap-less sub-pixel classes of stride-2 data gradients (zero fill / skip vs
# K-less GEMM launches): ResNet tests, then a same-box ResNet-50 A/B and the per-GEMM table.
set -o pipefail
mkdir -p gpurun_out/r6h
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_resnet_accuracy_gpu.py tests/test_model_gpu.py tests/test_kernels_gpu.py > gpurun_out/r6h/t.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r6h/t.log | head -20; tail -30 gpurun_out/r6h/t.log; exit 1; }
tail -2 gpurun_out/r6h/t.log
for rep in 1 2 3; do
  for f in 0 1; do
    CDP_SUBPIXEL_ZERO=$f timeout -k 10 200 python bench.py --model resnet50 --local-batch 64 --steps 20 --warmup 5 --no-extra > gpurun_out/r6h/b.log 2>&1 || { tail -20 gpurun_out/r6h/b.log; exit 1; }
    python -c "import json; r=json.loads([l for l in open('gpurun_out/r6h/b.log') if l.startswith('{')][-1]); print('resnet50 subpixel_zero=$f', r['ms_per_step'], r['value'])"
  done
done
