"""Tile / split-K sweep of VGG-11's conv GEMMs on the GPU (tuning data for plan_gemm / plan_wgrad).

For every VGG-11 conv layer 1-7, every per-GPU batch of the reference's strong-scaling rule
(256 / 128 / 64 / 32 images: W = 1, 2, 4, 8, /root/reference/src/Part 2a/main.py:22) and each of the
three GEMMs (forward with BN partials, data gradient, weight gradient -- each with its split-K
reduction), time the planner's choice and every candidate (tile, splits) forced through
``set_gemm_override``. Timing: 20 launches captured in one hipGraph, replayed 5 times, median
per launch (so per-launch host overhead is excluded the way the bench's captured step excludes it).

    python scripts/sweep_gemm.py [--batches 32,64] [--layers 1,2] [--out gpurun_out/sweep.json]

Prints one line per (batch, layer, op): planner config / time, best config / time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

VGG = [(3, 64, 32), (64, 128, 16), (128, 256, 8), (256, 256, 8), (256, 512, 4), (512, 512, 4), (512, 512, 2),
       (512, 512, 2)]
CONV_TILES = [(256, 128), (128, 128), (128, 64), (64, 128), (64, 64)]
WGRAD_TILES = [(256, 128), (128, 128), (128, 64), (64, 128), (64, 64)]
SPLITS = [1, 2, 3, 4, 5, 6, 8, 10, 12, 16, 20, 24, 32, 48, 64]


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def time_graph(fn, reps=20, rounds=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    ts = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / reps)
    g.reset()
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="32,64,128,256")
    ap.add_argument("--layers", default="1,2,3,4,5,6,7")
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    ap.add_argument("--out", default="gpurun_out/sweep_gemm.json")
    args = ap.parse_args()
    import cs744_distributed_data_parallel_amd as cdp

    C = cdp._native.lib()
    torch.manual_seed(0)
    results = []
    for B in [int(b) for b in args.batches.split(",")]:
        for li in [int(v) for v in args.layers.split(",")]:
            Ci, Co, HW = VGG[li]
            x = cl(torch.randn(B, Ci, HW, HW, device="cuda"))
            w = cl(torch.randn(Co, Ci, 3, 3, device="cuda") * (1.0 / (Ci * 9) ** 0.5))
            gy = cl(torch.randn(B, Co, HW, HW, device="cuda"))
            b = torch.zeros(Co, device="cuda")
            xa, ga, wa = C.act_max(x), C.act_max(gy), C.weight_prep([w], [False])[0][0]
            wt = C.weight_prep([w], [True])[1][0]
            M = B * HW * HW
            for op in args.ops.split(","):
                if op == "fwd":
                    kind, shape = "conv", (M, Co, 9 * Ci)
                    fn = lambda: C.conv2d_fwd(x, w, b, 1, 1, True, xa, wa)  # noqa: E731
                    tiles = CONV_TILES
                elif op == "dgrad":
                    kind, shape = "conv", (M, Ci, 9 * Co)
                    fn = lambda: C.conv2d_dgrad(gy, w, list(x.shape), 1, 1, None, ga, wa, wt)  # noqa: E731
                    tiles = CONV_TILES
                else:
                    kind, shape = "wgrad", (M, Co, 9 * Ci)
                    fn = lambda: C.conv2d_wgrad(gy, x, list(w.shape), 1, 1, None, False, ga, xa)  # noqa: E731
                    tiles = WGRAD_TILES
                plan = list(C.plan_info(kind, *shape))
                C.set_gemm_override(kind, 0, 0, 0)
                t_plan = time_graph(fn)
                kt = (shape[2] + 31) // 32 if kind == "conv" else (M + 31) // 32
                best = (t_plan, plan)
                rows = []
                for bm, bn in tiles:
                    for sp in SPLITS:
                        if sp > max(1, kt // 2):
                            continue
                        C.set_gemm_override(kind, bm, bn, sp)
                        try:
                            t = time_graph(fn)
                        finally:
                            C.set_gemm_override(kind, 0, 0, 0)
                        rows.append((bm, bn, sp, round(t, 2)))
                        if t < best[0]:
                            best = (t, [bm, bn, sp])
                rec = {"B": B, "layer": li, "op": op, "M": shape[0], "N": shape[1], "K": shape[2], "plan": plan,
                       "t_plan_us": round(t_plan, 2), "best": best[1], "t_best_us": round(best[0], 2), "all": rows}
                results.append(rec)
                print(f"B={B:3d} L{li} {op:5s} M={shape[0]:6d} N={shape[1]:3d} K={shape[2]:4d} plan {plan} "
                      f"{t_plan:7.2f} us | best {best[1]} {best[0]:7.2f} us", flush=True)
                with open(args.out, "w") as f:
                    json.dump(results, f)
    tot_p = sum(r["t_plan_us"] for r in results)
    tot_b = sum(r["t_best_us"] for r in results)
    print(f"total planner {tot_p:.1f} us, best {tot_b:.1f} us")


if __name__ == "__main__":
    main()
