set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
for pr in 0 1; do
  CDP_GEMM_PRIO=$pr timeout -k 10 180 python bench.py --steps 30 --warmup 5 > gpurun_out/b_prio$pr.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/b_prio$pr.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/b_prio$pr.log').read().strip().splitlines()[-1]); print('prio $pr', d['ms_per_step'], d['strict_fp32']['ms_per_step'], [s['ms_per_step'] for s in d['per_gpu_strong']], d['resnet50']['ms_per_step'])"
done
done
