set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extra > gpurun_out/b20.log 2>&1 || { tail -20 gpurun_out/b20.log; exit 1; }
  timeout -k 10 300 python bench.py --gpus 1 --steps 50 --warmup 10 --no-extra > gpurun_out/b50.log 2>&1 || { tail -20 gpurun_out/b50.log; exit 1; }
  python -c "
import json
def ms(f): return json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step']
print('steps20', ms('gpurun_out/b20.log'), 'steps50', ms('gpurun_out/b50.log'))"
done
