set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py tests/test_accuracy_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_model.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_model.log; exit 1; }
tail -2 gpurun_out/t_model.log
for i in 1 2; do
for f in 1 0; do
  CDP_BN_BWD_FIN=$f timeout -k 10 180 python bench.py --steps 30 --warmup 5 > gpurun_out/b_bf$f.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/b_bf$f.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/b_bf$f.log').read().strip().splitlines()[-1]); print('bwd_fin $f', d['ms_per_step'], d['strict_fp32']['ms_per_step'], [s['ms_per_step'] for s in d['per_gpu_strong']], d['resnet50']['ms_per_step'])"
done
done
