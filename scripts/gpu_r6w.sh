# Round-6 GPU session w: act-max chunks zeroed by a fill kernel. The new replay-vs-eager test, the driver's
# own steps (smoke, GPU tests, bench), then a steady-state K = 200 headline and ResNet-50.
set -o pipefail
mkdir -p gpurun_out/r6w
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_model_gpu.py -k "replayed_step_matches_eager" > gpurun_out/r6w/t1.log 2>&1 || { tail -30 gpurun_out/r6w/t1.log; exit 1; }
tail -1 gpurun_out/r6w/t1.log
bash scripts/diag/driver_flow.sh || exit 1
timeout -k 10 200 python bench.py --no-extra --steps 200 --warmup 30 > gpurun_out/r6w/b200.log 2>&1 || { tail -20 gpurun_out/r6w/b200.log; exit 1; }
python -c "import json; r=json.loads([l for l in open('gpurun_out/r6w/b200.log') if l.startswith('{')][-1]); print('K200', r['ms_per_step'])"
timeout -k 10 200 python bench.py --no-extra --local-batch 32 --steps 200 --warmup 30 > gpurun_out/r6w/b32.log 2>&1 || { tail -20 gpurun_out/r6w/b32.log; exit 1; }
python -c "import json; r=json.loads([l for l in open('gpurun_out/r6w/b32.log') if l.startswith('{')][-1]); print('b32 K200', r['ms_per_step'])"
