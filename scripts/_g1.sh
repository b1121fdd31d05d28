set -o pipefail
mkdir -p gpurun_out
PMC_MEM=1 bash scripts/pmc_layers.sh pmem256 256 > /dev/null || exit 1
python scripts/pmc_layers_summary.py gpurun_out/pmem256 256 | tail -20
bash scripts/prof_bench.sh b32f 10 --local-batch 32 || exit 1
bash scripts/prof_bench.sh b256f 6 || exit 1
