# Round-6 GPU session k: three-way same-box A/B of the conv epilogue's memory widths on ResNet-50
# (CDP_WIDE_STORES 0 = four-byte loads and stores, 2 = wide stores only, 1 = wide stores and
# addend loads) and two-way on VGG-11 (no addend there).
set -o pipefail
mkdir -p gpurun_out/r6k
for rep in 1 2 3; do
  for f in 0 2 1; do
    CDP_WIDE_STORES=$f timeout -k 10 200 python bench.py --model resnet50 --local-batch 64 --steps 20 --warmup 5 --no-extra > gpurun_out/r6k/b.log 2>&1 || { tail -20 gpurun_out/r6k/b.log; exit 1; }
    python -c "import json; r=json.loads([l for l in open('gpurun_out/r6k/b.log') if l.startswith('{')][-1]); print('resnet50 wide=$f', r['ms_per_step'], r['value'])"
  done
  for f in 0 1; do
    CDP_WIDE_STORES=$f timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-extra > gpurun_out/r6k/v.log 2>&1 || { tail -20 gpurun_out/r6k/v.log; exit 1; }
    python -c "import json; r=json.loads([l for l in open('gpurun_out/r6k/v.log') if l.startswith('{')][-1]); print('vgg wide=$f', r['ms_per_step'], r['value'])"
  done
done
