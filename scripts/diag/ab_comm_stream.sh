#!/bin/bash
# A/B of the communicator's stream kind (CDP_COMM_STREAM = pool | own | low | cumask) at one rank,
# 32 images: (1) the eager DDP backward span (scripts/diag/ddp_slowdown.py "ddp" row), (2) the
# captured DDP step with a real RCCL kernel + a scale kernel per bucket (CDP_BENCH_DDP_W1 +
# CDP_REDUCER_TEST_POSTOP), interleaved twice.
set -o pipefail
mkdir -p gpurun_out/abcs
for rep in 1 2; do
  for k in pool own low; do
    CDP_COMM_STREAM=$k timeout -k 10 120 python3 scripts/diag/ddp_slowdown.py ddp > gpurun_out/abcs/eager_$k.$rep.log 2>&1 || { echo "$k eager failed"; tail -5 gpurun_out/abcs/eager_$k.$rep.log; exit 1; }
    echo "$k eager: $(grep -m3 'iter' gpurun_out/abcs/eager_$k.$rep.log | tail -1)"
    CDP_COMM_STREAM=$k CDP_BENCH_DDP_W1=1 CDP_REDUCER_TEST_POSTOP=0:1 timeout -k 10 180 python3 bench.py --local-batch 32 --steps 50 --warmup 5 --no-extra > gpurun_out/abcs/graph_$k.$rep.log 2>&1 || { echo "$k graph failed"; tail -5 gpurun_out/abcs/graph_$k.$rep.log; exit 1; }
    python3 -c "import json,sys; r=json.loads([l for l in open('gpurun_out/abcs/graph_$k.$rep.log') if l.startswith('{')][-1]); print('$k captured DDP step', r['ms_per_step'], 'ms')"
  done
done
