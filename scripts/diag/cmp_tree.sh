#!/bin/bash
# Same-box comparison of staged source trees (abbuild/<tag>/: package + built .so + bench.py) and
# the current tree ("now"), interleaved. usage: scripts/diag/cmp_tree.sh LOCAL_BATCH TAG...
set -o pipefail
LB=$1; shift
mkdir -p gpurun_out/cmp
for rep in 1 2 3; do
  for tag in "$@" now; do
    if [ "$tag" = now ]; then dir=.; else dir=abbuild/$tag; fi
    (cd $dir && timeout -k 10 150 python3 bench.py --local-batch $LB --steps 50 --warmup 5 --no-extra > $GRAFT_REPO_ROOT/gpurun_out/cmp/$tag.$LB.$rep.log 2>&1) || { echo "$tag failed"; tail -5 gpurun_out/cmp/$tag.$LB.$rep.log; exit 1; }
    python3 -c "import json; r=json.loads([l for l in open('gpurun_out/cmp/$tag.$LB.$rep.log') if l.startswith('{')][-1]); print('$tag images $LB', r['ms_per_step'], 'ms')"
  done
done
