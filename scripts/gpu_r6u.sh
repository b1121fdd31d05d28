set -o pipefail
mkdir -p gpurun_out/r6u
for a in "1 x bo" "1 x bo" "1 x bo" "1 x bo" "1 x bb" "1 x bb"; do
  PYTHONPATH=. timeout -k 10 120 python scripts/diag/single_overlap_debug.py $a > gpurun_out/r6u/d.log 2>&1 || { tail -30 gpurun_out/r6u/d.log; exit 1; }
  echo "== $a"; grep "^replay" gpurun_out/r6u/d.log | cut -c1-150 | head -8
done
