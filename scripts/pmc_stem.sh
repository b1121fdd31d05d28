#!/bin/bash
# PMC passes over scripts/stem_micro.py (one rocprofv3 run per counter set, kernel trace only)
set -o pipefail
mkdir -p gpurun_out/pmc_stem
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_INSTS_MFMA" \
           "TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $SET --output-format csv -d gpurun_out/pmc_stem/p$i -o run -- python scripts/stem_micro.py > gpurun_out/pmc_stem/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_stem/p$i.log; }
  f=$(ls gpurun_out/pmc_stem/p$i/*counter_collection.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python scripts/pmc_summary.py $f > gpurun_out/pmc_stem/p$i.md
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_stem/kt -o run -- python scripts/stem_micro.py > gpurun_out/pmc_stem/kt.log 2>&1
python scripts/prof_summary.py gpurun_out/pmc_stem/kt/run_kernel_stats.csv 5 gpurun_out/pmc_stem/kt.md > /dev/null
