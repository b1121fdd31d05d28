set -o pipefail
mkdir -p gpurun_out/ovl
timeout -k 10 600 python -u -m pytest tests/test_accuracy_gpu.py -q -s --timeout 300 --timeout-method thread > gpurun_out/acc.log 2>&1; echo acc_rc=$?; tail -3 gpurun_out/acc.log
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/b1.log 2>&1 && tail -1 gpurun_out/b1.log || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --marker-trace --output-format csv -d gpurun_out/ovl -o run -- python scripts/overlap_timeline.py > gpurun_out/ovl/log.txt 2>&1 || { echo prof failed; tail -20 gpurun_out/ovl/log.txt; exit 1; }
ls gpurun_out/ovl
python scripts/overlap_summary.py gpurun_out/ovl/run_kernel_trace.csv gpurun_out/ovl/run_marker_api_trace.csv gpurun_out/ovl/summary.md > /dev/null; echo sum_rc=$?
