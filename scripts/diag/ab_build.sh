#!/bin/bash
# Two builds of the extension on one box, interleaved: the .so under ab_so/<tag>/ (git-ignored, but
# sent with the tree) are swapped into the package before each run.
# usage: [MODEL=resnet50] [LBS="256 32"] scripts/diag/ab_build.sh TAG_A TAG_B
set -o pipefail
PKG=cs744_distributed_data_parallel_amd
SO=$(ls $PKG/_C*.so)
MODEL=${MODEL:-vgg11}
LBS=${LBS:-"256 32"}
for rep in 1 2 3; do
  for tag in "$@"; do
    cp ab_so/$tag/_C.so "$SO"
    for lb in $LBS; do
      timeout -k 10 150 python3 bench.py --model $MODEL --local-batch $lb --steps 50 --warmup 5 --no-extra > gpurun_out/ab_$tag.$lb.$rep.log 2>&1 || { echo "$tag $lb failed"; tail -5 gpurun_out/ab_$tag.$lb.$rep.log; exit 1; }
      python3 -c "import json; r=json.loads([l for l in open('gpurun_out/ab_$tag.$lb.$rep.log') if l.startswith('{')][-1]); print('$tag images $lb', r['ms_per_step'], 'ms')"
    done
  done
done
