#!/bin/bash
# Per-kernel kernel-trace stats of staged builds (ab_so/<tag>/_C.so) on one box.
# usage: [MODEL=resnet50] [LB=64] scripts/diag/ab_prof.sh TAG...
set -o pipefail
PKG=cs744_distributed_data_parallel_amd
SO=$(ls $PKG/_C*.so)
MODEL=${MODEL:-resnet50}
LB=${LB:-64}
ROOT=$PWD
for tag in "$@"; do
  cp ab_so/$tag/_C.so "$SO"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/abprof/$tag -o run -- python3 $ROOT/bench.py --model $MODEL --local-batch $LB --steps 20 --warmup 5 --no-extra --no-graph > $ROOT/gpurun_out/abprof_$tag.log 2>&1) || { echo "$tag failed"; tail -5 gpurun_out/abprof_$tag.log; exit 1; }
  echo "$tag done"
done
