#!/bin/bash
# HBM bytes per dispatch of one eager bench step (FETCH_SIZE and WRITE_SIZE in separate passes,
# each with the kernel trace for durations) -> gpurun_out/bnbw/{fetch,write}/
# usage: scripts/diag/bn_bw.sh [bench args]
set -o pipefail
ROOT=$PWD
mkdir -p gpurun_out/bnbw
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  d=$ROOT/gpurun_out/bnbw/$c
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $d -o run -- \
    python3 $ROOT/bench.py --steps 1 --warmup 1 --no-graph --no-extra "$@" > $d.log 2>&1 || { echo "$c pass failed"; tail -5 $d.log; exit 1; }
  echo "$c done"
done
