# Native backtrace of the overlap-step bench's exit crash (CDP_SEGV_BT=1: in-process SIGSEGV handler).
set -o pipefail
mkdir -p gpurun_out/exitcrash
export CDP_BENCH_DDP_W1=1 CDP_REDUCER_TEST_POSTOP=xgmi:20:100:8 CDP_SEGV_BT=1
timeout -k 10 120 python -X faulthandler bench.py --local-batch 32 --steps 5 --warmup 3 --no-extra --no-graph --overlap-step > gpurun_out/exitcrash/bt.log 2>&1
echo "rc=$?"
grep -A40 "native backtrace" gpurun_out/exitcrash/bt.log | c++filt | head -60
