"""HBM traffic per kernel of the last profiled step (scripts/diag/bn_bw.sh): FETCH_SIZE and
WRITE_SIZE (KB, TCC counters, separate passes) against each pass's own kernel durations."""
import collections
import csv
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bnbw"


def last_step(counter):
    rows = list(csv.DictReader(open(f"{root}/{counter}/run_counter_collection.csv")))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    start = max(i for i, r in enumerate(rows) if "augment_kernel" in r["Kernel_Name"])
    out = []
    for r in rows[start:]:
        name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
        name = re.sub(r"\(.*", "", name).replace("cdp::", "").replace("void ", "")
        out.append((name, float(r["Counter_Value"]) * 1024,
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9))
    return out


f, w = last_step("FETCH_SIZE"), last_step("WRITE_SIZE")
assert [a[0] for a in f] == [b[0] for b in w], "the two passes dispatched different sequences"
agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
for (name, fb, ft), (_, wb, wt) in zip(f, w):
    a = agg[name]
    a[0] += 1
    a[1] += fb
    a[2] += wb
    a[3] += (ft + wt) / 2
print("| kernel | calls | read MB | written MB | time us | TB/s |")
print("|---|---|---|---|---|---|")
tot = [0.0, 0.0, 0.0]
for name, (n, fb, wb, t) in sorted(agg.items(), key=lambda kv: -kv[1][3])[: int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    print(f"| `{name[:60]}` | {n} | {fb / 1e6:.1f} | {wb / 1e6:.1f} | {t * 1e6:.0f} | {(fb + wb) / t / 1e12:.2f} |")
for n, fb, wb, t in agg.values():
    tot[0] += fb
    tot[1] += wb
    tot[2] += t
print(f"\nStep total: {tot[0] / 1e9:.2f} GB read, {tot[1] / 1e9:.2f} GB written, {tot[2] * 1e3:.2f} ms of kernels "
      f"(PMC passes serialize dispatches: durations are those of the counter runs)")
