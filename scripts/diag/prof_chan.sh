set -o pipefail
bash scripts/prof_bench.sh pchan32 6 --local-batch 32 || exit 1
grep -E "chan_|bwd_reduce|splitk|bn_fin|bn_bwd" gpurun_out/pchan32/summary.md | head -20
CDP_CHAN=0 bash scripts/prof_bench.sh pnochan32 6 --local-batch 32 || exit 1
grep -E "chan_|bwd_reduce|splitk|bn_fin|bn_bwd" gpurun_out/pnochan32/summary.md | head -20
