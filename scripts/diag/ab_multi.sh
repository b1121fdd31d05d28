#!/bin/bash
# A/B several builds of the extension on one box: ab/_C_<v>.so for v in $VARIANTS (copied in turn
# over the in-tree _C); the GPU kernel tests run first on $TESTED
set -o pipefail
mkdir -p gpurun_out
SO=cs744_distributed_data_parallel_amd/_C.cpython-310-x86_64-linux-gnu.so
cp ab/_C_${TESTED}.so $SO
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_pair_gpu.py tests/test_accuracy_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ab.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_ab.log; exit 1; }
tail -1 gpurun_out/t_ab.log
for i in $(seq ${ROUNDS:-2}); do for v in $VARIANTS; do
  cp ab/_C_$v.so $SO
  timeout -k 10 180 python bench.py --steps 60 --warmup 10 --no-extra > gpurun_out/b_$v.log 2>&1 || { tail -20 gpurun_out/b_$v.log; exit 1; }
  for b in 64 32; do timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-extra --local-batch $b > gpurun_out/b_${v}_$b.log 2>&1 || { tail -20 gpurun_out/b_${v}_$b.log; exit 1; }; done
  python -c "
import json
def ms(f): return json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step']
print('$v', ms('gpurun_out/b_$v.log'), [ms('gpurun_out/b_${v}_%d.log' % b) for b in (64, 32)])"
done; done
