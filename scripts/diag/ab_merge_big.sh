#!/bin/bash
# BN finalize merge cost at the large batches: shipped step (=0) vs fused finalize+apply kernels
# merging one partial (CDP_EXP_SKIP_BN_APPLY=2, numbers wrong, timing only), interleaved.
set -o pipefail
mkdir -p gpurun_out/mergebig
for rep in 1 2 3; do
  for lb in 256 128; do
    for v in 0 2; do
      CDP_EXP_SKIP_BN_APPLY=$v timeout -k 10 120 python3 bench.py --local-batch $lb --steps 50 --warmup 5 --no-extra > gpurun_out/mergebig/$lb.$v.$rep.log 2>&1 || { echo "lb $lb v $v failed"; tail -5 gpurun_out/mergebig/$lb.$v.$rep.log; exit 1; }
      python3 -c "import json; r=json.loads([l for l in open('gpurun_out/mergebig/$lb.$v.$rep.log') if l.startswith('{')][-1]); print('images $lb skip_bn_apply=$v', r['ms_per_step'], 'ms')"
    done
  done
done
