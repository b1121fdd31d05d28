# Round-6 GPU session j: wide addend loads in the conv epilogue + the re-swept ResNet-50 plans:
# conv / pair / ResNet numerics, same-box A/B of ResNet-50 (CDP_WIDE_STORES=0 = four-byte epilogue
# loads and stores), then the per-GEMM ResNet-50 table (scripts/pmc_resnet_layers.sh).
set -o pipefail
mkdir -p gpurun_out/r6j
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_pair_gpu.py tests/test_resnet_accuracy_gpu.py tests/test_model_gpu.py > gpurun_out/r6j/t.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r6j/t.log | head -20; tail -30 gpurun_out/r6j/t.log; exit 1; }
tail -2 gpurun_out/r6j/t.log
for rep in 1 2; do
  for f in 0 1; do
    CDP_WIDE_STORES=$f timeout -k 10 200 python bench.py --model resnet50 --local-batch 64 --steps 20 --warmup 5 --no-extra > gpurun_out/r6j/b.log 2>&1 || { tail -20 gpurun_out/r6j/b.log; exit 1; }
    python -c "import json; r=json.loads([l for l in open('gpurun_out/r6j/b.log') if l.startswith('{')][-1]); print('resnet50 wide=$f', r['ms_per_step'], r['value'])"
  done
done
bash scripts/pmc_resnet_layers.sh rn50w 64
