# Round-6 GPU session i: LDS-staged 16-B epilogue stores of the conv GEMMs (conv_epilogue.h):
# conv / pair / ResNet numerics, the small-K micro-benchmark both ways, then same-box A/B of the
# ResNet-50 step and the headline VGG-11 step (CDP_WIDE_STORES=0 = the four-byte stores).
set -o pipefail
mkdir -p gpurun_out/r6i
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_pair_gpu.py tests/test_accuracy_gpu.py tests/test_resnet_accuracy_gpu.py > gpurun_out/r6i/t.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r6i/t.log | head -20; tail -30 gpurun_out/r6i/t.log; exit 1; }
tail -2 gpurun_out/r6i/t.log
for f in 0 1; do
  echo "wide=$f"; CDP_WIDE_STORES=$f PYTHONPATH=. timeout -k 10 120 python scripts/diag/small_k_gemm.py || exit 1
done
for rep in 1 2; do
  for f in 0 1; do
    CDP_WIDE_STORES=$f timeout -k 10 200 python bench.py --model resnet50 --local-batch 64 --steps 20 --warmup 5 --no-extra > gpurun_out/r6i/b.log 2>&1 || { tail -20 gpurun_out/r6i/b.log; exit 1; }
    python -c "import json; r=json.loads([l for l in open('gpurun_out/r6i/b.log') if l.startswith('{')][-1]); print('resnet50 wide=$f', r['ms_per_step'], r['value'])"
    CDP_WIDE_STORES=$f timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-extra > gpurun_out/r6i/v.log 2>&1 || { tail -20 gpurun_out/r6i/v.log; exit 1; }
    python -c "import json; r=json.loads([l for l in open('gpurun_out/r6i/v.log') if l.startswith('{')][-1]); print('vgg wide=$f', r['ms_per_step'], r['value'])"
  done
done
