set -o pipefail
mkdir -p gpurun_out/r6v
CDP_SLOT_TRACE=1 PYTHONPATH=. timeout -k 10 120 python scripts/diag/replay_vs_eager.py one > gpurun_out/r6v/trace.log 2>&1 || { tail -30 gpurun_out/r6v/trace.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6v/trace.log | grep -n "===\|step\|cap=" | head -400 > gpurun_out/r6v/trace_head.txt
wc -l gpurun_out/r6v/trace.log
