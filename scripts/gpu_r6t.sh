# Round-6 GPU session t: single-device overlapped SGD (parallel.overlapped_step, bench --overlap-step at
# one GPU) vs the end-of-step SGD: VGG-11 at 256 and 32 images (K = 200 and K = 20), ResNet-50 (20 steps),
# bucket caps 2 MB (default) and 1 MB, interleaved.
set -o pipefail
mkdir -p gpurun_out/r6t
run() {  # label, bench args...
  local lab=$1; shift
  timeout -k 10 200 python bench.py --no-extra "$@" > gpurun_out/r6t/b.log 2>&1 || { tail -20 gpurun_out/r6t/b.log; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r6t/b.log') if l.startswith('{')][-1]); print('$lab', r['ms_per_step'], r['config'].get('optimizer_overlap'))"
}
for i in 1 2; do
  for lb in 256 32; do
    run "b$lb K200 base" --local-batch $lb --steps 200 --warmup 30
    run "b$lb K200 ovl2" --local-batch $lb --steps 200 --warmup 30 --overlap-step
    run "b$lb K200 ovl1" --local-batch $lb --steps 200 --warmup 30 --overlap-step --bucket-cap-mb 1
    run "b$lb K20 base" --local-batch $lb --steps 20 --warmup 5
    run "b$lb K20 ovl2" --local-batch $lb --steps 20 --warmup 5 --overlap-step
  done
done
for i in 1 2; do
  run "rn50 base" --model resnet50 --local-batch 64 --steps 20 --warmup 5
  run "rn50 ovl2" --model resnet50 --local-batch 64 --steps 20 --warmup 5 --overlap-step
done
