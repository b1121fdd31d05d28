"""Run the two-rank strategy-equivalence training twice per strategy (gloo, one GPU) and report
(a) whether a strategy's repeated runs are bitwise identical and (b) each strategy's step-1 max abs
and step-3 relative L2 difference to allreduce_blocking (diagnostic for tests/test_multirank_gpu.py)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from _dist_util import run_ranks  # noqa: E402
from test_multirank_gpu import _train_gpu  # noqa: E402

if __name__ == "__main__":
    runs = {}
    for s in ["allreduce_blocking", "gather_scatter", "bucketed_overlap", "ddp"]:
        runs[s] = [run_ranks(_train_gpu, 2, (s,), timeout=300) for _ in range(2)]
    (ref1, ref), _, _ = runs["allreduce_blocking"][0][0]
    for s, rr in runs.items():
        (a1, a3), la, _ = rr[0][0]
        (b1, b3), lb, _ = rr[1][0]
        same = np.array_equal(a1, b1) and np.array_equal(a3, b3)
        d1 = float(np.abs(a1 - ref1).max())
        rel = float(np.linalg.norm(a3 - ref) / np.linalg.norm(ref))
        rel_rep = float(np.linalg.norm(a3 - b3) / np.linalg.norm(b3))
        print(f"{s:20s} repeat-identical={same} rep-rel={rel_rep:.2e} step1-maxabs={d1:.2e} step3-rel={rel:.2e} losses={la}")
