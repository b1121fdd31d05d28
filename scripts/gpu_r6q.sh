# Round-6 GPU session q: the tile-statistics A/B again, order alternating (wave first in odd reps).
set -o pipefail
mkdir -p gpurun_out/r6q
for rep in 1 2 3 4; do
  if [ $((rep % 2)) = 1 ]; then order="wave 2pass"; else order="2pass wave"; fi
  for v in $order; do
    CDP_TILE_STATS=$v timeout -k 10 200 python bench.py --steps 200 --warmup 30 --no-extra > gpurun_out/r6q/v.log 2>&1 || { tail -20 gpurun_out/r6q/v.log; exit 1; }
    python -c "import json; r=json.loads([l for l in open('gpurun_out/r6q/v.log') if l.startswith('{')][-1]); print('vgg256 $rep $v', r['ms_per_step'])"
  done
done
