#!/bin/bash
# Hardware-queue placement of side streams vs the compute stream (scripts/diag/comm_queue.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cq
for k in none pool own own_low cumask own_first; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cq/$k -o run -- python3 scripts/diag/comm_queue.py $k > gpurun_out/cq/$k.log 2>&1 || { echo "$k failed"; tail -20 gpurun_out/cq/$k.log; exit 1; }
  grep "iter\|range" gpurun_out/cq/$k.log
  f=$(find gpurun_out/cq/$k -name "*kernel_trace.csv" | head -1)
  python3 scripts/diag/comm_queue.py summary "$f" | tee gpurun_out/cq/$k.md
done
