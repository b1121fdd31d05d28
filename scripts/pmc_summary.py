"""Aggregate a rocprofv3 --pmc counter_collection.csv: per kernel name, mean of each counter."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
names = sorted({c for k in acc.values() for c in k})
print("| kernel | n | " + " | ".join(names) + " |")
print("|---|---|" + "---|" * len(names))
for k, d in sorted(acc.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    n = max(len(v) for v in d.values())
    vals = [f"{sum(d[c]) / len(d[c]):.4g}" if d.get(c) else "-" for c in names]
    print(f"| `{k[:70]}` | {n} | " + " | ".join(vals) + " |")
