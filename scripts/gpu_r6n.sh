# Round-6 GPU session n: BN tile statistics with one barrier (per-wave exact two-pass, Chan merge of
# the wave rows) vs the block-wide two-pass version (CDP_TILE_STATS=2pass): numerics, the small-K
# micro-benchmark both ways, same-box A/B of VGG-11 at 256 / 32 images and ResNet-50.
set -o pipefail
mkdir -p gpurun_out/r6n
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_accuracy_gpu.py tests/test_resnet_accuracy_gpu.py tests/test_model_gpu.py tests/test_deferred_bn_gpu.py > gpurun_out/r6n/t.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r6n/t.log | head -20; tail -30 gpurun_out/r6n/t.log; exit 1; }
tail -2 gpurun_out/r6n/t.log
for v in 2pass wave; do
  echo "stats=$v"; CDP_TILE_STATS=$v PYTHONPATH=. timeout -k 10 120 python scripts/diag/small_k_gemm.py 2>&1 | grep -v sweep || exit 1
done
for rep in 1 2 3; do
  for v in 2pass wave; do
    CDP_TILE_STATS=$v timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-extra > gpurun_out/r6n/v.log 2>&1 || { tail -20 gpurun_out/r6n/v.log; exit 1; }
    python -c "import json; r=json.loads([l for l in open('gpurun_out/r6n/v.log') if l.startswith('{')][-1]); print('vgg256 $v', r['ms_per_step'])"
    CDP_TILE_STATS=$v timeout -k 10 200 python bench.py --local-batch 32 --steps 200 --warmup 30 --no-extra > gpurun_out/r6n/v.log 2>&1 || { tail -20 gpurun_out/r6n/v.log; exit 1; }
    python -c "import json; r=json.loads([l for l in open('gpurun_out/r6n/v.log') if l.startswith('{')][-1]); print('vgg32 $v', r['ms_per_step'])"
    CDP_TILE_STATS=$v timeout -k 10 200 python bench.py --model resnet50 --local-batch 64 --steps 20 --warmup 5 --no-extra > gpurun_out/r6n/b.log 2>&1 || { tail -20 gpurun_out/r6n/b.log; exit 1; }
    python -c "import json; r=json.loads([l for l in open('gpurun_out/r6n/b.log') if l.startswith('{')][-1]); print('resnet50 $v', r['ms_per_step'])"
  done
done
