# Round-6 GPU session sw: VGG-11 block-level plan re-sweep (f16x2, 256 and 32 images) on the final tree
# (after the round-6 epilogue changes), scripts/sweep_pair.py.
set -o pipefail
mkdir -p gpurun_out/r6sw
timeout -k 10 1000 python -u scripts/sweep_pair.py --batches 256,32 --out gpurun_out/r6sw/sweep.json > gpurun_out/r6sw/sweep.log 2>&1 || { tail -20 gpurun_out/r6sw/sweep.log; exit 1; }
grep -E "^B=|^total" gpurun_out/r6sw/sweep.log
