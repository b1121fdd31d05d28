#!/bin/bash
# ResNet-50 residual blocks: backward reads a 1-byte-per-float4 ReLU mask (CDP_RES_MASK=1, shipped)
# instead of the block output (=0), interleaved, 64 images.
set -o pipefail
mkdir -p gpurun_out/resmask
for rep in 1 2 3; do
  for v in 0 1; do
    CDP_RES_MASK=$v timeout -k 10 200 python3 bench.py --model resnet50 --local-batch 64 --steps 20 --warmup 5 --no-extra > gpurun_out/resmask/$v.$rep.log 2>&1 || { echo "v $v failed"; tail -5 gpurun_out/resmask/$v.$rep.log; exit 1; }
    python3 -c "import json; r=json.loads([l for l in open('gpurun_out/resmask/$v.$rep.log') if l.startswith('{')][-1]); print('resnet50 res_mask=$v', r['ms_per_step'], 'ms')"
  done
done
