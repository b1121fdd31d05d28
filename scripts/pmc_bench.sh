#!/bin/bash
# rocprofv3 PMC counters (no trace domains) of a short eager bench run -> gpurun_out/<tag>/
# usage: scripts/pmc_bench.sh TAG "COUNTERS" [bench args]
set -o pipefail
TAG=${1:-pmc}
COUNTERS=${2:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM"}
shift 2
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --pmc $COUNTERS --output-format csv -d gpurun_out/$TAG -o run -- \
  python bench.py --steps 3 --warmup 1 --no-graph "$@" > gpurun_out/$TAG/bench.log 2>&1 || exit $?
python scripts/pmc_summary.py gpurun_out/$TAG/run_counter_collection.csv > gpurun_out/$TAG/summary.md
