# Does the measured step depend on the timed-step count? Two builds x K = 20 / 60 / 200 / 600
# (warmup 5 / 10 / 30 / 30), headline step at 256 images, interleaved.
set -o pipefail
SO=cs744_distributed_data_parallel_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/_C_keep.so
mkdir -p gpurun_out/abs
for i in 1 2; do for v in $1; do
  cp ab/_C_$v.so $SO
  for kw in 20:5 60:10 200:30 600:30; do
    k=${kw%:*}; w=${kw#*:}
    timeout -k 10 200 python bench.py --steps $k --warmup $w --no-extra > gpurun_out/abs/b.log 2>&1 || { tail -20 gpurun_out/abs/b.log; cp /tmp/_C_keep.so $SO; exit 1; }
    python -c "import json; r=json.loads([l for l in open('gpurun_out/abs/b.log') if l.startswith('{')][-1]); print('$i $v K=$k', r['ms_per_step'])"
  done
done; done
cp /tmp/_C_keep.so $SO
