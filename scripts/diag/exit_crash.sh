# Which feature makes the bench process crash at interpreter exit? (overlap-step x fused classifier)
set -o pipefail
mkdir -p gpurun_out/exitcrash
export CDP_BENCH_DDP_W1=1 CDP_REDUCER_TEST_POSTOP=xgmi:20:100:8
for fc in 0 1; do
  for ov in "" "--overlap-step"; do
    CDP_FUSED_CLASSIFIER=$fc timeout -k 10 120 python bench.py --local-batch 32 --steps 20 --warmup 5 --no-extra $ov > gpurun_out/exitcrash/fc$fc$ov.log 2>&1
    echo "fused_classifier=$fc overlap='$ov' rc=$?"
  done
done
CDP_FUSED_CLASSIFIER=1 timeout -k 10 120 python bench.py --local-batch 32 --steps 20 --warmup 5 --no-extra --no-graph --overlap-step > gpurun_out/exitcrash/eager.log 2>&1
echo "eager overlap rc=$?"
unset CDP_BENCH_DDP_W1 CDP_REDUCER_TEST_POSTOP
timeout -k 10 120 python bench.py --local-batch 32 --steps 20 --warmup 5 --no-extra > gpurun_out/exitcrash/plain.log 2>&1
echo "plain 1-GPU rc=$?"
