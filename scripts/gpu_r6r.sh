# Round-6 GPU session r (run twice: with and without the wide slab stores): weight-gradient epilogue -- reciprocal scales in their own LDS slots (two
# barriers fewer) and 16-B slab stores through LDS. Tests on the new build, then same-box A/B of
# ab/_C_old.so vs ab/_C_new.so: VGG-11 256 / 32 images (K = 200), ResNet-50.
set -o pipefail
mkdir -p gpurun_out/r6r
SO=cs744_distributed_data_parallel_amd/_C.cpython-310-x86_64-linux-gnu.so
cp ab/_C_new.so $SO
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_pair_gpu.py tests/test_accuracy_gpu.py tests/test_resnet_accuracy_gpu.py tests/test_model_gpu.py tests/test_fused_tail_gpu.py > gpurun_out/r6r/t.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r6r/t.log | head -20; tail -30 gpurun_out/r6r/t.log; exit 1; }
tail -1 gpurun_out/r6r/t.log
bash scripts/diag/ab_so3.sh "old new" 3 || exit 1
for i in 1 2; do for v in old new; do
  cp ab/_C_$v.so $SO
  timeout -k 10 200 python bench.py --model resnet50 --local-batch 64 --steps 20 --warmup 5 --no-extra > gpurun_out/r6r/b.log 2>&1 || { tail -20 gpurun_out/r6r/b.log; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r6r/b.log') if l.startswith('{')][-1]); print('resnet50 $v', r['ms_per_step'])"
done; done
cp ab/_C_new.so $SO
