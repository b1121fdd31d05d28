set -o pipefail
mkdir -p gpurun_out/r6v
for z in kernel memset kernel; do
  CDP_SLOT_ZERO=$z PYTHONPATH=. timeout -k 10 120 python scripts/diag/replay_vs_eager.py one > gpurun_out/r6v/d.log 2>&1 || { tail -30 gpurun_out/r6v/d.log; exit 1; }
  echo "== zero by $z"; grep "^step" gpurun_out/r6v/d.log | head -6
done
