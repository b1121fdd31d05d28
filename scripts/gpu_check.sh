#!/bin/bash
# GPU check used during development: gpu tests, 1-GPU bench, optional extra command.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/b1.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/b1.log; exit 1; }
tail -1 gpurun_out/b1.log
