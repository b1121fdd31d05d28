set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bdef.log 2>&1 || { tail -30 gpurun_out/bdef.log; exit 1; }
tail -1 gpurun_out/bdef.log
bash scripts/prof_bench.sh b32 10 --local-batch 32
