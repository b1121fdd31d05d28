set -o pipefail
mkdir -p gpurun_out/r6v
PYTHONPATH=. timeout -k 10 120 python scripts/diag/capture_frees.py > gpurun_out/r6v/cf.log 2>&1 || { tail -30 gpurun_out/r6v/cf.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6v/cf.log | head -60 | cut -c1-600
