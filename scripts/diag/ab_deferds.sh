#!/bin/bash
# ResNet-50 downsample branches: BatchNorm applied inside the residual add (CDP_DEFER_DS=1, shipped)
# vs materialized (=0), interleaved, 64 images.
set -o pipefail
mkdir -p gpurun_out/deferds
for rep in 1 2 3; do
  for v in 0 1; do
    CDP_DEFER_DS=$v timeout -k 10 200 python3 bench.py --model resnet50 --local-batch 64 --steps 20 --warmup 5 --no-extra > gpurun_out/deferds/$v.$rep.log 2>&1 || { echo "v $v failed"; tail -5 gpurun_out/deferds/$v.$rep.log; exit 1; }
    python3 -c "import json; r=json.loads([l for l in open('gpurun_out/deferds/$v.$rep.log') if l.startswith('{')][-1]); print('resnet50 defer_ds=$v', r['ms_per_step'], 'ms')"
  done
done
