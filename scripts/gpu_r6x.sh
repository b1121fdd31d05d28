# Round-6 GPU session x: the final tree (fill-kernel slot zeroing, kernel root copies): comm tests, eager kernel
# tables at 256 and 32 images, and the replayed hipGraph step at 256 and 32 images under a kernel trace.
set -o pipefail
mkdir -p gpurun_out/r6x
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_comm_gpu.py tests/test_model_gpu.py > gpurun_out/r6x/t.log 2>&1 || { tail -30 gpurun_out/r6x/t.log; exit 1; }
tail -1 gpurun_out/r6x/t.log
bash scripts/prof_bench.sh r6x_b256 10 || exit $?
bash scripts/prof_bench.sh r6x_b32 10 --local-batch 32 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lb in 256 32; do
  rm -rf gpurun_out/r6x/g$lb
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6x/g$lb -o run -- python3 bench.py --steps 60 --warmup 10 --no-extra --local-batch $lb > gpurun_out/r6x/g$lb.log 2>&1 || { tail -20 gpurun_out/r6x/g$lb.log; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r6x/g$lb.log') if l.startswith('{')][-1]); print('graph $lb', r['ms_per_step'])"
  python scripts/prof_graph_step.py gpurun_out/r6x/g$lb/run_kernel_trace.csv > gpurun_out/r6x/g$lb.md || exit 1
  rm -f gpurun_out/r6x/g$lb/run_kernel_trace.csv
  tail -1 gpurun_out/r6x/g$lb.md
done
