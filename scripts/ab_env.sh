#!/bin/bash
# Same-box A/B of an environment toggle on the 1-GPU bench: ab_env.sh VAR "VAL_A VAL_B" [reps] [bench args]
# Prints one line per run: VAR=value ms_per_step img/s
set -o pipefail
var=$1; vals=$2; reps=${3:-2}; shift 3
mkdir -p gpurun_out
for r in $(seq "$reps"); do
  for v in $vals; do
    env "$var=$v" timeout -k 10 180 python bench.py --steps 30 --warmup 10 --no-extra "$@" > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    python - "$var=$v" <<'PY'
import json, sys
line = [l for l in open("gpurun_out/ab.log") if l.startswith("{")][-1]
d = json.loads(line)
print(sys.argv[1], d["ms_per_step"], d["value"], flush=True)
PY
  done
done
