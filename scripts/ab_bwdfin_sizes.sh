# Same-box A/B of the fused backward BN finalize + apply (CDP_BN_BWD_FIN=1, bn_bwd_fin_apply) against
# chan_finalize + bn_bwd_apply (=0) at 256 / 128 / 64 / 32 images per GPU (hipGraph bench)
set -o pipefail
for lb in 256 128 64 32; do
  bash scripts/ab_env.sh CDP_BN_BWD_FIN "1 0" 3 --local-batch $lb || exit 1
done
