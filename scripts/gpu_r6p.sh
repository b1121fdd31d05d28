# Round-6 GPU session p: the 256-image step replayed from its hipGraph under a kernel trace, both
# tile-statistics variants (the eager tables of session o are equal; the replayed bench is not).
set -o pipefail
mkdir -p gpurun_out/r6p
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 2pass wave 2pass wave; do
  rm -rf gpurun_out/r6p/$v
  CDP_TILE_STATS=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6p/$v -o run -- python3 bench.py --steps 30 --warmup 5 --no-extra > gpurun_out/r6p/$v.log 2>&1 || { tail -20 gpurun_out/r6p/$v.log; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r6p/$v.log') if l.startswith('{')][-1]); print('$v', r['ms_per_step'])"
  python scripts/prof_graph_step.py gpurun_out/r6p/$v/run_kernel_trace.csv > gpurun_out/r6p/$v.md || exit 1
done
