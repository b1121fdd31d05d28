set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
for mb in 128 256 512; do
  CDP_FIN_MAXBLK=$mb timeout -k 10 180 python bench.py --steps 30 --warmup 5 > gpurun_out/b_fin$mb.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/b_fin$mb.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/b_fin$mb.log').read().strip().splitlines()[-1]); print('finblk $mb', d['ms_per_step'], d['strict_fp32']['ms_per_step'], [s['ms_per_step'] for s in d['per_gpu_strong']], d['resnet50']['ms_per_step'])"
done
done
