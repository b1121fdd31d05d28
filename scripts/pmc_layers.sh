#!/bin/bash
# Per-layer GEMM efficiency of the VGG-11 training step: one kernel-trace pass (durations) and one
# PMC pass (MFMA busy, wave stalls, LDS bank conflicts) over a short eager bench run; the last
# step's GEMM dispatches are labelled by layer -> gpurun_out/<tag>/layers.md
# usage: scripts/pmc_layers.sh TAG LOCAL_BATCH
set -o pipefail
TAG=${1:-pmcl}
LB=${2:-256}
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$TAG/kt -o run -- \
  python bench.py --no-graph --no-extra --steps 2 --warmup 1 --local-batch $LB > gpurun_out/$TAG/kt.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY \
  SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT \
  --output-format csv -d gpurun_out/$TAG/pmc -o run -- \
  python bench.py --no-graph --no-extra --steps 2 --warmup 1 --local-batch $LB > gpurun_out/$TAG/pmc.log 2>&1 || exit $?
# optional second pass: instruction mix (per wave) of the same dispatches
if [ -n "$PMC_MIX" ]; then
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVES \
    SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d gpurun_out/$TAG/mix -o run -- \
    python bench.py --no-graph --no-extra --steps 2 --warmup 1 --local-batch $LB > gpurun_out/$TAG/mix.log 2>&1 || exit $?
fi
# optional third pass: L2 hits / misses and memory-side requests of the same dispatches
if [ -n "$PMC_MEM" ]; then
  timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE \
    --output-format csv -d gpurun_out/$TAG/mem -o run -- \
    python bench.py --no-graph --no-extra --steps 2 --warmup 1 --local-batch $LB > gpurun_out/$TAG/mem.log 2>&1 || exit $?
fi
python scripts/pmc_layers_summary.py gpurun_out/$TAG $LB > gpurun_out/$TAG/layers.md
cat gpurun_out/$TAG/layers.md
