set -o pipefail
mkdir -p gpurun_out
for lb in 32 64 128 256; do bash scripts/ab_env.sh CDP_PLANNER_GAIN "0.8 0.87 0.95" 2 --local-batch $lb || exit 1; done
