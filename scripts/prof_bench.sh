set -o pipefail
mkdir -p gpurun_out/prof1
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python bench.py --steps 10 --warmup 3 --no-graph > gpurun_out/prof1/bench.log 2>&1
echo "prof rc=$?"
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --backend torch > gpurun_out/bench_torch.log 2>&1
echo "torch rc=$?"
tail -2 gpurun_out/bench_torch.log
find gpurun_out/prof1 -name "*stats*"
