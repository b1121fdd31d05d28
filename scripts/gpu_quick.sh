# Targeted GPU tests (PYTEST_FILES) then the default 1-GPU bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${PYTEST_FILES} -x -v --timeout 200 --timeout-method thread > gpurun_out/gpuquick.log 2>&1 || { tail -60 gpurun_out/gpuquick.log; exit 1; }
tail -3 gpurun_out/gpuquick.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || { tail -20 gpurun_out/bench_driver.log; exit 1; }
tail -1 gpurun_out/bench_driver.log
