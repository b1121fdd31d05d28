# Same-box A/B: optimizer step fused with the next forward's weight preparation (default) vs the
# separate weight_prep launch (CDP_BENCH_NO_FUSED_PREP=1), hipGraph bench at 256 and 32 images
set -o pipefail
mkdir -p gpurun_out
for lb in 256 32; do
  bash scripts/ab_env.sh CDP_BENCH_NO_FUSED_PREP "0 1" 3 --local-batch $lb || exit 1
done
