# Stability of the two-rank one-GPU strategy-equivalence test on the tree without the stem-deferred
# slot zeroing: three solo runs, then the driver's steps.
set -o pipefail
mkdir -p gpurun_out/r6mr
for i in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests/test_multirank_gpu.py -q --timeout 250 --timeout-method thread -k strategy_equivalence > gpurun_out/r6mr/m$i.log 2>&1; echo "multirank run $i rc=$?"; grep -E "passed|failed|AssertionError: \(" gpurun_out/r6mr/m$i.log | tail -2
done
bash scripts/diag/driver_flow.sh
