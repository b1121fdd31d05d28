# Round-6 GPU session z: the step's first act-max chunk zeroed inside the RGB stem's launch (no fill dispatch).
# Full GPU suite, replayed-step traces at 256 / 32 images, K = 200 at 256 / 32, the driver's bench command.
set -o pipefail
mkdir -p gpurun_out/r6z
for i in 1 2; do
  timeout -k 10 300 python -u -m pytest tests/test_multirank_gpu.py -q --timeout 250 --timeout-method thread -k strategy_equivalence > gpurun_out/r6z/m$i.log 2>&1; echo "multirank run $i rc=$?"; grep -E "passed|failed|AssertionError: \(" gpurun_out/r6z/m$i.log | tail -2
done
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --deselect tests/test_multirank_gpu.py::test_two_ranks_on_one_gpu_strategy_equivalence > gpurun_out/r6z/t.log 2>&1 || { tail -30 gpurun_out/r6z/t.log; exit 1; }
tail -1 gpurun_out/r6z/t.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lb in 256 32; do
  rm -rf gpurun_out/r6z/g$lb
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6z/g$lb -o run -- python3 bench.py --steps 60 --warmup 10 --no-extra --local-batch $lb > gpurun_out/r6z/g$lb.log 2>&1 || { tail -20 gpurun_out/r6z/g$lb.log; exit 1; }
  python scripts/prof_graph_step.py gpurun_out/r6z/g$lb/run_kernel_trace.csv > gpurun_out/r6z/g$lb.md || exit 1
  rm -f gpurun_out/r6z/g$lb/run_kernel_trace.csv
  tail -1 gpurun_out/r6z/g$lb.md
done
for lb in 256 32; do
  timeout -k 10 200 python bench.py --no-extra --local-batch $lb --steps 200 --warmup 30 > gpurun_out/r6z/k$lb.log 2>&1 || { tail -20 gpurun_out/r6z/k$lb.log; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r6z/k$lb.log') if l.startswith('{')][-1]); print('K200 b$lb', r['ms_per_step'])"
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6z/bench.log 2>&1 || { tail -20 gpurun_out/r6z/bench.log; exit 1; }
tail -1 gpurun_out/r6z/bench.log
