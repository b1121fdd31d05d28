# Overlapped step at a fixed bucket plan (--bucket-cap-mb: no calibration, so rocprof cannot distort
# the plan): same-box A/B at 32 and 256 images with the modelled 8-rank xGMI all-reduce, then one
# kernel trace per mode at 32 images for the timeline.
set -o pipefail
mkdir -p gpurun_out/r6e
export CDP_BENCH_DDP_W1=1 CDP_REDUCER_TEST_POSTOP=xgmi:20:100:8
for lb in 32 256; do
for rep in 1 2 3; do
  for ov in "" "--overlap-step"; do
    timeout -k 10 150 python bench.py --local-batch $lb --steps 60 --warmup 10 --no-extra --bucket-cap-mb 10 $ov > gpurun_out/r6e/b.log 2>&1 || { tail -20 gpurun_out/r6e/b.log; exit 1; }
    python -c "import json; r=json.loads([l for l in open('gpurun_out/r6e/b.log') if l.startswith('{')][-1]); print($lb, 'overlap' if '$ov' else 'end-step', r['ms_per_step'], [x['bytes'] for x in r['buckets']['launch_order']])"
  done
done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for ov in "" "--overlap-step"; do
  tag=$([ -n "$ov" ] && echo ov || echo base)
  timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6e/prof_$tag -o run -- python3 bench.py --local-batch 32 --steps 5 --warmup 3 --no-extra --bucket-cap-mb 10 $ov > gpurun_out/r6e/prof_$tag.log 2>&1 || { tail -20 gpurun_out/r6e/prof_$tag.log; exit 1; }
done
echo done
