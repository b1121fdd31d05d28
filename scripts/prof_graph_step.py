"""Per-kernel table of the last complete training step in a rocprofv3 kernel trace of a
hipGraph-replayed bench run (steps delimited by augment_kernel): duration of each dispatch and the
idle gap before it, so replayed steps can be compared dispatch by dispatch.
usage: python scripts/prof_graph_step.py run_kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "augment_kernel" in r["Kernel_Name"]]
step = rows[starts[-2]:starts[-1]]
t0 = int(step[0]["Start_Timestamp"])
prev_end = t0
busy = 0
print("| # | kernel | us | gap us |\n|---|---|---|---|")
for i, r in enumerate(step):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    nm = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace("cdp::", "")
    nm = nm.split("(")[0][:60]
    print(f"| {i} | `{nm}` | {(e - s) / 1e3:.1f} | {(s - prev_end) / 1e3:.1f} |")
    busy += e - s
    prev_end = max(prev_end, e)
print(f"\n{len(step)} dispatches; busy {busy / 1e3:.1f} us; step {(int(rows[starts[-1]]['Start_Timestamp']) - t0) / 1e3:.1f} us")
