# One-GPU rehearsal of the driver's multi-GPU bench (2 ranks on cuda:0 over gloo: the strategies
# block, the timed bucket planner, replica digests) and the bucket-plan profile at 32 images
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 3 > gpurun_out/rehearsal2.log 2>&1 || { tail -30 gpurun_out/rehearsal2.log; exit 1; }
tail -1 gpurun_out/rehearsal2.log | cut -c1-600
timeout -k 10 200 python scripts/bucket_plan.py 32 > gpurun_out/bucket_plan_b32.md 2> gpurun_out/bucket_plan.err || { tail -20 gpurun_out/bucket_plan.err; exit 1; }
timeout -k 10 200 python scripts/bucket_plan.py 256 > gpurun_out/bucket_plan_b256.md 2>> gpurun_out/bucket_plan.err || { tail -20 gpurun_out/bucket_plan.err; exit 1; }
tail -5 gpurun_out/bucket_plan_b32.md
