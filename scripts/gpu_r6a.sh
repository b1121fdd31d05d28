# Round-6 first GPU check: smoke, 1-GPU bench (driver default), two-rank gloo rehearsal of the
# phase supervisor with every extra on the one GPU, and the multi-rank GPU tests.
set -o pipefail
mkdir -p gpurun_out/r6a
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/r6a/smoke.log 2>&1 || { tail -20 gpurun_out/r6a/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6a/b1.log 2>&1 || { tail -30 gpurun_out/r6a/b1.log; exit 1; }
tail -1 gpurun_out/r6a/b1.log
timeout -k 10 500 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --local-batch 64 > gpurun_out/r6a/b2g.log 2>&1 || { tail -30 gpurun_out/r6a/b2g.log; exit 1; }
tail -1 gpurun_out/r6a/b2g.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['phases'])"
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multirank_gpu.py > gpurun_out/r6a/mr.log 2>&1 || { tail -30 gpurun_out/r6a/mr.log; exit 1; }
tail -3 gpurun_out/r6a/mr.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_accuracy_gpu.py -k "act_max" > gpurun_out/r6a/am.log 2>&1 || { tail -30 gpurun_out/r6a/am.log; exit 1; }
tail -3 gpurun_out/r6a/am.log
