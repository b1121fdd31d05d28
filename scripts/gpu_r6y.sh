# Round-6 GPU session y: 16-B fill kernel for the act-max chunks. Full GPU suite, replayed-step kernel traces at
# 256 and 32 images, the default bench.
set -o pipefail
mkdir -p gpurun_out/r6y
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6y/t.log 2>&1 || { tail -30 gpurun_out/r6y/t.log; exit 1; }
tail -1 gpurun_out/r6y/t.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lb in 256 32; do
  rm -rf gpurun_out/r6y/g$lb
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6y/g$lb -o run -- python3 bench.py --steps 60 --warmup 10 --no-extra --local-batch $lb > gpurun_out/r6y/g$lb.log 2>&1 || { tail -20 gpurun_out/r6y/g$lb.log; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r6y/g$lb.log') if l.startswith('{')][-1]); print('graph $lb', r['ms_per_step'])"
  python scripts/prof_graph_step.py gpurun_out/r6y/g$lb/run_kernel_trace.csv > gpurun_out/r6y/g$lb.md || exit 1
  rm -f gpurun_out/r6y/g$lb/run_kernel_trace.csv
  tail -1 gpurun_out/r6y/g$lb.md
done
timeout -k 10 300 python bench.py > gpurun_out/r6y/bench.log 2>&1 || { tail -20 gpurun_out/r6y/bench.log; exit 1; }
tail -1 gpurun_out/r6y/bench.log
