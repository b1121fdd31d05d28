set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_model.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_model.log; exit 1; }
tail -2 gpurun_out/t_model.log
for cfg in "1 4" "0 0" "2 2" "1 2" "1 1"; do
  set -- $cfg
  CDP_CHAN_FWD_RT=$1 CDP_CHAN_BWD_RT=$2 timeout -k 10 180 python bench.py --steps 30 --warmup 5 > gpurun_out/b_rt$1_$2.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/b_rt$1_$2.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/b_rt$1_$2.log').read().strip().splitlines()[-1]); print('fwd_rt $1 bwd_rt $2', d['ms_per_step'], d['strict_fp32']['ms_per_step'], [s['ms_per_step'] for s in d['per_gpu_strong']], d['resnet50']['ms_per_step'])"
done
