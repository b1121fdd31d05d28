# Round-6 GPU session l: the kept profiles of the round-6 tree -- VGG-11 kernel tables at 256 and
# 32 images, the ResNet-50 per-GEMM table (scripts/pmc_resnet_layers.sh), one 1-GPU bench run.
set -o pipefail
bash scripts/prof_bench.sh r6l_b256 10 || exit $?
bash scripts/prof_bench.sh r6l_b32 10 --local-batch 32 || exit $?
bash scripts/pmc_resnet_layers.sh r6l_rn50 64 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r6l_bench.log 2>&1 || { tail -20 gpurun_out/r6l_bench.log; exit 1; }
tail -1 gpurun_out/r6l_bench.log
