# Same-box A/B of three builds of the extension (ab/_C_<name>.so copied in turn over the in-tree
# one), hipGraph headline step at 256 and 32 images, 200 timed steps, interleaved repetitions.
# usage: bash scripts/diag/ab_so3.sh "name1 name2 name3" [reps]
set -o pipefail
SO=cs744_distributed_data_parallel_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/_C_keep.so
mkdir -p gpurun_out/ab3
for i in $(seq 1 ${2:-3}); do for v in $1; do
  cp ab/_C_$v.so $SO
  for b in 256 32; do
    timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-extra --local-batch $b > gpurun_out/ab3/b.log 2>&1 || { tail -20 gpurun_out/ab3/b.log; cp /tmp/_C_keep.so $SO; exit 1; }
    python -c "import json; r=json.loads([l for l in open('gpurun_out/ab3/b.log') if l.startswith('{')][-1]); print('$i $v $b', r['ms_per_step'])"
  done
done; done
cp /tmp/_C_keep.so $SO
