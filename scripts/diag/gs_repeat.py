"""Repeat the two-rank gather/scatter training and compare every run bitwise with the first
(diagnostic: run-to-run determinism of the gloo-on-device gather/scatter path)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from _dist_util import run_ranks  # noqa: E402
from test_multirank_gpu import _train_gpu  # noqa: E402

if __name__ == "__main__":
    strat = sys.argv[1] if len(sys.argv) > 1 else "gather_scatter"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    first = None
    for k in range(n):
        (a1, a3), la, _ = run_ranks(_train_gpu, 2, (strat,), timeout=300)[0]
        if first is None:
            first = (a1, a3)
            print(k, "reference", la, flush=True)
            continue
        d1 = float(np.abs(a1 - first[0]).max())
        rel = float(np.linalg.norm(a3 - first[1]) / np.linalg.norm(first[1]))
        print(k, f"step1-maxabs={d1:.2e} step3-rel={rel:.2e}", la, flush=True)
