#!/bin/bash
# Round-5 GPU session f: whole GPU suite, smoke, bench, ResNet-50 kernel profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?
tail -15 gpurun_out/gputest.log | grep -E "passed|failed|FAILED|ERROR"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc (not a plain test failure): stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b1.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/b1.log; exit 1; }
tail -1 gpurun_out/b1.log
bash scripts/prof_bench.sh profrn50_r5b 5 --model resnet50 --local-batch 64 || { echo "profrn50 failed"; exit 1; }
exit $rc
