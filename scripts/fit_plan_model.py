"""Fit the GEMM planner's cost model (csrc/runtime/ops.cpp plan_gemm / plan_wgrad) to a tile /
split-K sweep (scripts/sweep_gemm.py output) and report how close its choices come to the measured
best configuration.

    python scripts/fit_plan_model.py profiles/tuning/vgg11_gemm_sweep_r3.json

Model of one GEMM + its split-K reduction, for a tile (bm, bn) and s splits over a P x Q output with
reduction length R (conv: P = M rows, Q = N, R = K; weight gradient: P = Cout, Q = Kdim, R = M):
  tiles = ceil(P/bm) ceil(Q/bn), blocks = tiles s, kps = ceil(ceil(R/32) / s) K-tiles per block
  a CU runs nb = ceil(blocks / CUs) blocks, k = min(nb, residency) at a time, in ceil(nb / residency)
  rounds; a round takes a0 + kps * max(l0 + l1 (bm + bn), k bm bn / rho, k (bm + bn) / beta)
  (per-K-tile latency floor vs the CU's MAC rate vs its operand-load rate, both shared by the k
  co-resident blocks)
  + a reduction launch when s > 1: r0 + r1 * s * P * Q * 4 bytes
"""
from __future__ import annotations

import json
import math
import sys

import numpy as np
from scipy.optimize import least_squares

CUS = 256


def residency(kind, bm, bn):
    if kind == "conv":
        return 1 if bm + bn >= 384 else 2 if bm + bn >= 256 else 3
    return 1 if bm >= 256 else 2 if bm + bn >= 192 else 3


def dims(r):
    if r["op"] == "wgrad":
        return r["N"], r["K"], r["M"]  # Cout, Kdim, reduction rows
    return r["M"], r["N"], r["K"]


def features(kind, P, Q, R, bm, bn, s):
    tiles = math.ceil(P / bm) * math.ceil(Q / bn)
    blocks = tiles * s
    kt = math.ceil(R / 32)
    kps = math.ceil(kt / s)
    res = residency(kind, bm, bn)
    nb = math.ceil(blocks / CUS)
    k = min(nb, res)
    rounds = math.ceil(nb / res)
    return rounds, kps, bm + bn, k * bm * bn, (s > 1), s * P * Q * 4e-6, k * (bm + bn)


def predict(theta, f):
    t0, a0, l0, l1, rho, r0, r1, beta = theta
    rounds, kps, bmn, kw, red, sbytes, kb = f
    per_round = a0 + kps * np.maximum(np.maximum(l0 + l1 * bmn, kw / rho), kb / beta)
    return t0 + rounds * per_round + red * (r0 + r1 * sbytes)


def fit(records, kind):
    rows = []
    for r in records:
        if (r["op"] == "wgrad") != (kind == "wgrad"):
            continue
        P, Q, R = dims(r)
        for bm, bn, s, t in r["all"]:
            rows.append((features(kind, P, Q, R, bm, bn, s), t))
    F = [np.array([f[i] for f, _ in rows], dtype=float) for i in range(7)]
    T = np.array([t for _, t in rows])

    def res(th):
        return np.log(predict(np.abs(th), F)) - np.log(T)

    th0 = np.array([5.0, 1.0, 0.3, 0.003, 20000.0, 3.0, 0.5, 400.0])
    sol = least_squares(res, th0, x_scale="jac")
    return np.abs(sol.x)


def regret(records, kind, theta):
    tot_choice = tot_best = 0.0
    for r in records:
        if (r["op"] == "wgrad") != (kind == "wgrad"):
            continue
        P, Q, R = dims(r)
        meas = {(bm, bn, s): t for bm, bn, s, t in r["all"]}
        pred = {c: predict(theta, features(kind, P, Q, R, *c)) for c in meas}
        choice = min(pred, key=pred.get)
        best = min(meas, key=meas.get)
        tot_choice += meas[choice]
        tot_best += meas[best]
        print(f"  B={r['B']:3d} L{r['layer']} {r['op']:5s} model {choice} {meas[choice]:6.2f} us | "
              f"best {best} {meas[best]:6.2f} us")
    return tot_choice, tot_best


def main(path):
    records = json.load(open(path))
    for kind in ("conv", "wgrad"):
        th = fit(records, kind)
        print(kind, "theta (t0, a0, l0, l1, rho, r0, r1, beta) =", ", ".join(f"{v:.4g}" for v in th))
        c, b = regret(records, kind, th)
        print(f"{kind}: model choices {c:.1f} us, measured best {b:.1f} us ({100 * (c / b - 1):.1f} % over)")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "profiles/tuning/vgg11_gemm_sweep_r3.json")
