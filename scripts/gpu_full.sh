# Full GPU check + profiles: smoke, GPU test suite, default bench, eager kernel profiles at 256 / 32
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r4}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || { tail -20 gpurun_out/bench_driver.log; exit 1; }
tail -1 gpurun_out/bench_driver.log
bash scripts/prof_bench.sh b256_$TAG 6 || exit 1
bash scripts/prof_bench.sh b32_$TAG 10 --local-batch 32 || exit 1
