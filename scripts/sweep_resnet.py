"""Tile / split-K sweep of ResNet-50's conv GEMMs (224x224, 64 images per GPU: BASELINE config #5)
on the GPU, per op (forward with BN partials, stride-1 data gradient, weight gradient), for the
tuned-plan table of csrc/runtime/ops.cpp. The fitted planner model was fitted to VGG-11's 3x3
shapes only; ResNet's 1x1 / strided / 7x7 shapes are checked here.

Every distinct conv of the model (shapes recorded by forward hooks) is timed at the planner's plan
and at every (tile, splits) candidate through ``set_gemm_override`` (hipGraph, see
scripts/sweep_gemm.py); the planner's plan and the best are then re-timed alternately (3 each,
medians). Stride-2 data gradients run as sub-pixel GEMMs of other shapes and are not swept.

    python scripts/sweep_resnet.py [--batch 64] [--out gpurun_out/sweep_resnet.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sweep_gemm import CONV_TILES, SPLITS, WGRAD_TILES, cl, time_graph  # noqa: E402


def conv_shapes(model, B, hw):
    seen, shapes = set(), []

    def hook(mod, inp, _out):
        x = inp[0]
        key = (x.shape[1], mod.out_channels, mod.kernel_size[0], mod.stride[0], mod.padding[0], x.shape[2], x.shape[3])
        if key not in seen:
            seen.add(key)
            shapes.append(key)

    hs = [m.register_forward_hook(hook) for m in model.modules() if isinstance(m, torch.nn.Conv2d)]
    with torch.no_grad():
        model(torch.randn(2, 3, hw, hw))
    for h in hs:
        h.remove()
    return shapes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--hw", type=int, default=224)
    ap.add_argument("--out", default="gpurun_out/sweep_resnet.json")
    ap.add_argument("--engine", default="f16x2")
    ap.add_argument("--max-shapes", type=int, default=0)
    args = ap.parse_args()
    import cs744_distributed_data_parallel_amd as cdp

    C = cdp._native.lib()
    C.set_conv_gemm(args.engine)
    shapes = conv_shapes(cdp.get_model("resnet50"), 2, args.hw)
    if args.max_shapes:
        shapes = shapes[: args.max_shapes]
    print(f"{len(shapes)} distinct convs", flush=True)
    B = args.batch
    torch.manual_seed(0)
    results = []
    for Ci, Co, k, s, p, H, W in shapes:
        if Ci < 16:
            continue  # the RGB stem (channel-padded path)
        x = cl(torch.randn(B, Ci, H, W, device="cuda"))
        w = cl(torch.randn(Co, Ci, k, k, device="cuda") * (1.0 / (Ci * k * k) ** 0.5))
        P, Q = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        gy = cl(torch.randn(B, Co, P, Q, device="cuda"))
        b = torch.zeros(Co, device="cuda")
        xa, ga, wa = C.act_max(x), C.act_max(gy), C.weight_prep([w], [False])[0][0]
        wt = C.weight_prep([w], [True])[1][0]
        M = B * P * Q
        ops = [("fwd", "conv", (M, Co, k * k * Ci), CONV_TILES,
                lambda: C.conv2d_fwd(x, w, b, s, p, True, xa, wa)),
               ("wgrad", "wgrad", (M, Co, k * k * Ci), WGRAD_TILES,
                lambda: C.conv2d_wgrad(gy, x, list(w.shape), s, p, None, False, ga, xa))]
        if s == 1:
            ops.append(("dgrad", "dgrad", (B * H * W, Ci, k * k * Co), CONV_TILES,
                        lambda: C.conv2d_dgrad(gy, w, list(x.shape), s, p, None, ga, wa, wt)))
        for op, kind, shape, tiles, fn in ops:
            okind = "conv" if kind == "dgrad" else kind
            plan = list(C.plan_info(kind, *shape))
            t_plan = time_graph(fn)
            kt = (shape[2] + 31) // 32 if okind == "conv" else (M + 31) // 32
            best = (t_plan, plan)
            for bm, bn in tiles:
                for sp in SPLITS:
                    if sp > max(1, kt // 2):
                        continue
                    C.set_gemm_override(okind, bm, bn, sp)
                    try:
                        t = time_graph(fn)
                    except RuntimeError:
                        continue
                    finally:
                        C.set_gemm_override(okind, 0, 0, 0)
                    if t < best[0]:
                        best = (t, [bm, bn, sp])
            ta, tb = [], []
            for _ in range(3):
                ta.append(time_graph(fn))
                C.set_gemm_override(okind, *best[1])
                try:
                    tb.append(time_graph(fn))
                finally:
                    C.set_gemm_override(okind, 0, 0, 0)
            ta, tb = sorted(ta)[1], sorted(tb)[1]
            rec = {"conv": [Ci, Co, k, s, p, H, W], "op": op, "kind": kind, "M": shape[0], "N": shape[1],
                   "K": shape[2], "plan": plan, "t_plan_us": round(ta, 2), "best": best[1], "t_best_us": round(tb, 2)}
            results.append(rec)
            print(f"{Ci:4d}->{Co:4d} k{k} s{s} @{H:3d} {op:5s} M={shape[0]:6d} N={shape[1]:4d} K={shape[2]:5d} plan {plan} "
                  f"{ta:7.2f} us | best {best[1]} {tb:7.2f} us ({100 * (ta - tb) / ta:+.1f} %)", flush=True)
            with open(args.out, "w") as f:
                json.dump(results, f)
    tp = sum(r["t_plan_us"] for r in results)
    tb = sum(r["t_best_us"] for r in results)
    print(f"total planner {tp:.1f} us, best {tb:.1f} us")


if __name__ == "__main__":
    main()
