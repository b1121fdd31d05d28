# Round-6 GPU session s: split-K reduction kernel (splitk_reduce4) BN partials with one barrier (per-thread
# exact triples + Chan merge of the row lanes). Tests on the new build, then same-box A/B of
# ab/_C_old.so vs ab/_C_new.so: VGG-11 256 / 32 images (K = 200), ResNet-50.
set -o pipefail
mkdir -p gpurun_out/r6s
SO=cs744_distributed_data_parallel_amd/_C.cpython-310-x86_64-linux-gnu.so
cp ab/_C_new.so $SO
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_pair_gpu.py tests/test_accuracy_gpu.py tests/test_resnet_accuracy_gpu.py tests/test_model_gpu.py tests/test_fused_tail_gpu.py > gpurun_out/r6s/t.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r6s/t.log | head -20; tail -30 gpurun_out/r6s/t.log; exit 1; }
tail -1 gpurun_out/r6s/t.log
bash scripts/diag/ab_so3.sh "old new" 3 || exit 1
for i in 1 2; do for v in old new; do
  cp ab/_C_$v.so $SO
  timeout -k 10 200 python bench.py --model resnet50 --local-batch 64 --steps 20 --warmup 5 --no-extra > gpurun_out/r6s/b.log 2>&1 || { tail -20 gpurun_out/r6s/b.log; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r6s/b.log') if l.startswith('{')][-1]); print('resnet50 $v', r['ms_per_step'])"
done; done
cp ab/_C_new.so $SO
