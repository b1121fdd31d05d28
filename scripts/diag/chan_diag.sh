set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python scripts/diag/chan_grad_diff.py 32 > gpurun_out/diag32.txt 2>&1 || { tail -20 gpurun_out/diag32.txt; exit 1; }
timeout -k 10 200 python scripts/diag/chan_grad_diff.py 64 > gpurun_out/diag64.txt 2>&1 || { tail -20 gpurun_out/diag64.txt; exit 1; }
cat gpurun_out/diag32.txt gpurun_out/diag64.txt
