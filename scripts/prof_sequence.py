"""Per-dispatch timeline of the last profiled step from a rocprofv3 kernel-trace CSV.

usage: python scripts/prof_sequence.py run_kernel_trace.csv FIRST_KERNEL_SUBSTRING [out.md]

The step boundary is the last dispatch whose name contains FIRST_KERNEL_SUBSTRING (e.g.
``augment_kernel`` for bench.py). Prints every dispatch of that step with its grid, duration and
the idle gap before it, so a layer-by-layer cost and the launch gaps are visible.
"""
import csv
import sys


def main(path, marker, out=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(starts) < 2:
        raise SystemExit(f"need >= 2 occurrences of {marker!r}")
    lo, hi = starts[-2], starts[-1]
    step = rows[lo:hi]
    t0 = int(step[0]["Start_Timestamp"])
    lines = ["| # | kernel | grid | wg | us | gap us |", "|---|---|---|---|---|---|"]
    busy = 0
    prev_end = t0
    for i, r in enumerate(step):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("cdp::(anonymous namespace)::", "")
        name = name.split("(")[0] if "(" in name and "<" not in name.split("(")[0][-3:] else name
        name = name if len(name) < 70 else name[:67] + "..."
        grid = f"{r.get('Grid_Size_X', r.get('Grid_Size', '?'))}"
        wg = f"{r.get('Workgroup_Size_X', r.get('Workgroup_Size', '?'))}"
        lines.append(f"| {i} | `{name}` | {grid} | {wg} | {(e - s) / 1e3:.1f} | {max(0, s - prev_end) / 1e3:.1f} |")
        busy += e - s
        prev_end = max(prev_end, e)
    wall = prev_end - t0
    lines.append(f"\n{len(step)} dispatches; busy {busy / 1e3:.1f} us, wall {wall / 1e3:.1f} us")
    text = "\n".join(lines)
    if out:
        open(out, "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[1], a[2] if len(a) > 2 else None)
