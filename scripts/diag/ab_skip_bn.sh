#!/bin/bash
# Ceiling of BatchNorm-in-the-consumer-GEMM: the per-GPU strong-scaling
# steps with the small layers' finalize + apply launches skipped (CDP_EXP_SKIP_BN_APPLY=1) and with
# only their statistics merge cut to one partial (=2, the ceiling of a producer-side finalize), vs
# the shipped step (=0), interleaved. Numbers wrong under 1 and 2: timing only.
set -o pipefail
mkdir -p gpurun_out/skipbn
for rep in 1 2 3; do
  for lb in 32 64; do
    for v in 0 1 2; do
      CDP_EXP_SKIP_BN_APPLY=$v timeout -k 10 120 python3 bench.py --local-batch $lb --steps 50 --warmup 5 --no-extra > gpurun_out/skipbn/$lb.$v.$rep.log 2>&1 || { echo "lb $lb skip $v failed"; tail -5 gpurun_out/skipbn/$lb.$v.$rep.log; exit 1; }
      python3 -c "import json; r=json.loads([l for l in open('gpurun_out/skipbn/$lb.$v.$rep.log') if l.startswith('{')][-1]); print('images $lb skip_bn_apply=$v', r['ms_per_step'], 'ms')"
    done
  done
done
