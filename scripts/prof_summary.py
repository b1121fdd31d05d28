"""Summarise a rocprofv3 --kernel-trace --stats CSV run into a markdown table (per-step kernel time)."""
import csv
import sys
from collections import defaultdict

def main(stats_csv, trace_csv=None, steps=1, top=40, out=None):
    rows = list(csv.DictReader(open(stats_csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        name = r["Name"].replace("cdp::(anonymous namespace)::", "")
        name = name if len(name) < 90 else name[:87] + "..."
        lines.append(f"| `{name}` | {int(r['Calls'])} | {float(r['TotalDurationNs'])/1e6:.3f} | "
                     f"{float(r['AverageNs'])/1e3:.1f} | {float(r['Percentage']):.1f} |")
    lines.append(f"\nTotal GPU kernel time: {tot/1e6:.3f} ms over {steps} profiled steps "
                 f"= {tot/1e6/steps:.3f} ms/step")
    text = "\n".join(lines)
    if out:
        open(out, "w").write(text + "\n")
    print(text)

if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], steps=int(a[1]) if len(a) > 1 else 1, out=a[2] if len(a) > 2 else None)
