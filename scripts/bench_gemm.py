"""Per-layer timing of the conv GEMMs (forward, data gradient, weight gradient) on VGG-11's B=256
shapes, with the operand maxima passed in as the fused producers would (no standalone amax pass
in the timed region). Prints one line per layer and op: microseconds and fp32-equivalent TFLOP/s.

usage: python scripts/bench_gemm.py [--batch 256] [--iters 20] [--ops fwd,dgrad,wgrad]
(CDP_CONV_GEMM / CDP_TILE_BM select the engine and tile as for bench.py)
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import cs744_distributed_data_parallel_amd as cdp  # noqa: F401
from cs744_distributed_data_parallel_amd import _native

# VGG-11 convs at 32x32 input: (Cin, Cout, H)
VGG11 = [(3, 64, 32), (64, 128, 16), (128, 256, 8), (256, 256, 8), (256, 512, 4), (512, 512, 4), (512, 512, 2),
         (512, 512, 2)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    a = ap.parse_args()
    C = _native.lib()
    dev = torch.device("cuda")
    cl = torch.channels_last
    ops = a.ops.split(",")
    rows = []
    tot = {o: 0.0 for o in ops}
    for li, (ci, co, h) in enumerate(VGG11):
        if ci == 3:
            ci = 4  # the RGB stem runs zero-padded to 4 channels
        x = torch.randn(a.batch, ci, h, h, device=dev).contiguous(memory_format=cl)
        w = (torch.randn(co, ci, 3, 3, device=dev) * 0.05).contiguous(memory_format=cl)
        gy = torch.randn(a.batch, co, h, h, device=dev).contiguous(memory_format=cl) * 1e-3
        xa, ga = C.act_max(x), C.act_max(gy)  # as the producers would pass them (None outside f16x2)
        wl = C.weight_prep([w], [False])[0]
        wa = wl[0] if wl else None
        flop = 2.0 * a.batch * h * h * co * ci * 9
        fns = {
            "fwd": lambda: C.conv2d_fwd(x, w, None, 1, 1, True, xa, wa),
            "dgrad": lambda: C.conv2d_dgrad(gy, w, list(x.shape), 1, 1, None, ga, wa),
            "wgrad": lambda: C.conv2d_wgrad(gy, x, list(w.shape), 1, 1, None, False, ga, xa),
        }
        for o in ops:
            if o == "dgrad" and li == 0:
                continue
            fn = fns[o]
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / a.iters * 1e3
            tot[o] += us
            rows.append({"layer": li, "op": o, "us": round(us, 1), "tflops": round(flop / us * 1e-6, 1)})
            print(f"L{li} {o:6s} {us:8.1f} us {flop / us * 1e-6:7.1f} TF", flush=True)
    print(json.dumps({"engine": C.get_conv_gemm(), "total_us": {k: round(v, 1) for k, v in tot.items()}}))


if __name__ == "__main__":
    main()
