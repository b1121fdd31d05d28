# Round-6 GPU session b: the overlapped optimizer step -- bitwise test, then a same-box A/B of the
# DDP step at 32 images with a modelled 8-rank xGMI all-reduce behind every bucket, and one kernel
# trace of each mode for the overlap timeline.
set -o pipefail
mkdir -p gpurun_out/r6b
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_step_overlap_gpu.py tests/test_comm_gpu.py > gpurun_out/r6b/t.log 2>&1 || { tail -40 gpurun_out/r6b/t.log; exit 1; }
tail -3 gpurun_out/r6b/t.log
export CDP_BENCH_DDP_W1=1 CDP_REDUCER_TEST_POSTOP=xgmi:20:100:8
for rep in 1 2 3; do
  for ov in "" "--overlap-step"; do
    timeout -k 10 150 python bench.py --local-batch 32 --steps 100 --warmup 10 --no-extra $ov > gpurun_out/r6b/b.log 2>&1 || { tail -20 gpurun_out/r6b/b.log; exit 1; }
    python -c "import json; r=json.loads([l for l in open('gpurun_out/r6b/b.log') if l.startswith('{')][-1]); print('overlap' if '$ov' else 'end-step', r['ms_per_step'], r['config']['hipgraph'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for ov in "" "--overlap-step"; do
  tag=$([ -n "$ov" ] && echo ov || echo base)
  timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6b/prof_$tag -o run -- python3 bench.py --local-batch 32 --steps 5 --warmup 3 --no-extra $ov > gpurun_out/r6b/prof_$tag.log 2>&1 || { tail -20 gpurun_out/r6b/prof_$tag.log; exit 1; }
done
echo done
