#!/bin/bash
# Diagnostic: the captured (hipGraph) 32-image step on one GPU, plain vs the DDP wrapper at one rank
# (CDP_BENCH_DDP_W1) without and with real RCCL kernels per bucket (CDP_REDUCER_TEST_POSTOP).
set -e
mkdir -p gpurun_out
B=${B:-32}
run() { echo "== $1"; shift; env "$@" timeout -k 10 150 python bench.py --local-batch $B --steps 50 --warmup 10 --no-extra 2>&1 | grep '"metric"' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms/step', 'hipgraph', d.get('hipgraph'))"; }
run plain X=1
run "ddp at one rank (events only)" CDP_BENCH_DDP_W1=1
run "ddp at one rank (RCCL kernel per bucket)" CDP_BENCH_DDP_W1=1 CDP_REDUCER_TEST_POSTOP=0:1.0000002
run plain X=1
