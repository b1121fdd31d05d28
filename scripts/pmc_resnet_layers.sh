#!/bin/bash
# Per-GEMM table of one eager ResNet-50 training step (64 x 224^2 by default): kernel trace
# (durations), one counter pass for MFMA busy / waits, one each for FETCH_SIZE and WRITE_SIZE (TCC
# limits), GEMM shapes from the engine's own launch log (CDP_GEMM_LOG) -> gpurun_out/<tag>/layers.md
# usage: scripts/pmc_resnet_layers.sh TAG [LOCAL_BATCH]
set -o pipefail
TAG=${1:-rn50l}
LB=${2:-64}
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
ARGS="--model resnet50 --local-batch $LB --no-graph --no-extra --steps 1 --warmup 1"
export CDP_GEMM_LOG=1
CDP_GEMM_LOG_OUT=gpurun_out/$TAG/gemm_log.json timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/$TAG/kt -o run -- python bench.py $ARGS > gpurun_out/$TAG/kt.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY \
  SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/$TAG/pmc -o run -- \
  python bench.py $ARGS > gpurun_out/$TAG/pmc.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$TAG/fetch -o run -- \
  python bench.py $ARGS > gpurun_out/$TAG/fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/$TAG/write -o run -- \
  python bench.py $ARGS > gpurun_out/$TAG/write.log 2>&1 || exit $?
python scripts/pmc_resnet_layers.py gpurun_out/$TAG > gpurun_out/$TAG/layers.md
tail -12 gpurun_out/$TAG/layers.md
