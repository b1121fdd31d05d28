#!/bin/bash
# Round-5 GPU session: whole GPU suite, bench, then diagnostics (HW queues, comm stream A/B, ResNet copies).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?
tail -15 gpurun_out/gputest.log | grep -E "passed|failed|FAILED|ERROR"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc (not a plain test failure): stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b1.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/b1.log; exit 1; }
tail -1 gpurun_out/b1.log
timeout -k 10 120 python scripts/diag/resnet_copies.py > gpurun_out/rn_copies.md 2>&1 || { echo "resnet copies failed"; tail -20 gpurun_out/rn_copies.md; exit 1; }
bash scripts/diag/comm_queue.sh
