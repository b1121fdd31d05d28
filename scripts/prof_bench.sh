#!/bin/bash
# rocprofv3 kernel-trace + stats of a short eager bench run; summary -> gpurun_out/<tag>/summary.md,
# last step's dispatch timeline -> gpurun_out/<tag>/sequence.md
set -o pipefail
TAG=${1:-prof}
STEPS=${2:-10}
shift 2
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG -o run -- \
  python bench.py --steps $STEPS --warmup 3 --no-graph --no-extra "$@" > gpurun_out/$TAG/bench.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/$TAG/run_kernel_stats.csv $((STEPS + 3)) gpurun_out/$TAG/summary.md > /dev/null
python scripts/prof_sequence.py gpurun_out/$TAG/run_kernel_trace.csv augment_kernel gpurun_out/$TAG/sequence.md > /dev/null || true
rm -f gpurun_out/$TAG/run_kernel_trace.csv
tail -1 gpurun_out/$TAG/bench.log
