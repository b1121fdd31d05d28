# Round-6 GPU session o: which kernels the one-barrier tile statistics sped up (kernel tables of
# the 256-image step with CDP_TILE_STATS=2pass and the default).
set -o pipefail
CDP_TILE_STATS=2pass bash scripts/prof_bench.sh r6o_2pass 10 || exit $?
bash scripts/prof_bench.sh r6o_wave 10 || exit $?
