set -o pipefail
timeout -k 10 120 python scripts/diag/arena_steal.py || exit 1
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_model.log 2>&1 || { tail -30 gpurun_out/t_model.log; exit 1; }
tail -1 gpurun_out/t_model.log
for i in 1 2; do for c in 1 0; do
CDP_CHAN=$c timeout -k 10 180 python bench.py --steps 30 --warmup 5 > gpurun_out/b_c$c.log 2>&1 || { tail -20 gpurun_out/b_c$c.log; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/b_c$c.log').read().strip().splitlines()[-1]); print('chan $c', d['ms_per_step'], d['strict_fp32']['ms_per_step'], [s['ms_per_step'] for s in d['per_gpu_strong']], d['resnet50']['ms_per_step'])"
done; done
