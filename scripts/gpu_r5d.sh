#!/bin/bash
# Round-5 GPU session d: whole GPU suite, bench, BN-apply ceiling A/B, rocprofv3 profiles at 256 / 32
# images and ResNet-50.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?
tail -15 gpurun_out/gputest.log | grep -E "passed|failed|FAILED|ERROR"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc (not a plain test failure): stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b1.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/b1.log; exit 1; }
tail -1 gpurun_out/b1.log
bash scripts/diag/ab_skip_bn.sh || exit 1
bash scripts/prof_bench.sh prof256_r5 10 || { echo "prof256 failed"; exit 1; }
bash scripts/prof_bench.sh prof32_r5 20 --local-batch 32 || { echo "prof32 failed"; exit 1; }
bash scripts/prof_bench.sh profrn50_r5 5 --model resnet50 --local-batch 64 || { echo "profrn50 failed"; exit 1; }
timeout -k 10 120 python scripts/diag/resnet_copies.py > gpurun_out/rn_copies.md 2>&1 || { echo "resnet copies failed"; tail -20 gpurun_out/rn_copies.md; exit 1; }
