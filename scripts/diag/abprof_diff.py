"""Per-kernel totals of two rocprofv3 rocpd databases (scripts/diag/ab_prof.sh), largest change first."""
import collections
import re
import sqlite3
import sys


def load(tag):
    c = sqlite3.connect(f"gpurun_out/abprof/{tag}/run_results.db")
    d = collections.defaultdict(lambda: [0, 0.0])
    for name, s, e in c.execute("select name, start, end from kernels"):
        n = re.sub(r"\(anonymous namespace\)::", "", name)
        n = re.sub(r"\(.*", "", n)[:72]
        d[n][0] += 1
        d[n][1] += (e - s) / 1e3
    return d


a, b = load(sys.argv[1]), load(sys.argv[2])
keys = sorted(set(a) | set(b), key=lambda k: -abs(b.get(k, [0, 0])[1] - a.get(k, [0, 0])[1]))
print("%-72s %6s %10s %6s %10s %8s" % ("kernel", "n_a", "us_a", "n_b", "us_b", "b-a"))
for k in keys[: int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    x, y = a.get(k, [0, 0]), b.get(k, [0, 0])
    print("%-72s %6d %10.0f %6d %10.0f %8.0f" % (k, x[0], x[1], y[0], y[1], y[1] - x[1]))
print("total us", round(sum(v[1] for v in a.values())), round(sum(v[1] for v in b.values())))
