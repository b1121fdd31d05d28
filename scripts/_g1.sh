set -o pipefail
mkdir -p gpurun_out
for lb in 32 256; do bash scripts/ab_env.sh CDP_BN_BWD_FIN "0 1" 2 --local-batch $lb || exit 1; done
PMC_MIX=1 bash scripts/pmc_layers.sh pm256 256 || exit 1
bash scripts/prof_bench.sh b32m 10 --local-batch 32 || exit 1
