"""Re-time candidate backward plans of VGG-11 blocks against the current planner's, alternately
(the close calls of scripts/sweep_pair.py, before they go into the tuned-plan table).

    python scripts/verify_plans.py "32:2:64,64,4:128,64,6" "256:2:256,128,2:256,128,28" [--rounds 5]

Each argument is images:block:dgrad bm,bn,splits:wgrad bm,bn,splits. Prints the medians.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sweep_pair import POOL_AFTER, VGG, time_graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cands", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    import cs744_distributed_data_parallel_amd as cdp
    from cs744_distributed_data_parallel_amd.ops import functional as CF

    C = cdp._native.lib()
    C.set_conv_gemm("f16x2")
    for cand in args.cands:
        b, li, d, w = cand.split(":")
        B, li = int(b), int(li)
        d = [int(v) for v in d.split(",")]
        w = [int(v) for v in w.split(",")]
        Ci, Co, HW = VGG[li]
        torch.manual_seed(li)
        conv = torch.nn.Conv2d(Ci, Co, 3, padding=1).cuda()
        conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
        bnorm = torch.nn.BatchNorm2d(Co).cuda()
        pool = li in POOL_AFTER
        x = torch.relu(torch.randn(B, Ci, HW, HW, device="cuda")).contiguous(memory_format=torch.channels_last)
        x.requires_grad_()
        oh = HW // 2 if pool else HW
        gy = torch.randn(B, Co, oh, oh, device="cuda").contiguous(memory_format=torch.channels_last)

        def block(dp, wp):
            def fn():
                out = CF.conv_bn_act(x, conv, bnorm, relu=True, pool=pool)
                C.set_gemm_override("conv", *dp)
                C.set_gemm_override("wgrad", *wp)
                try:
                    torch.autograd.grad(out, [x, conv.weight], gy)
                finally:
                    C.set_gemm_override("conv", 0, 0, 0)
                    C.set_gemm_override("wgrad", 0, 0, 0)
            return fn

        base, cand_t = [], []
        for _ in range(args.rounds):
            base.append(time_graph(block([0, 0, 0], [0, 0, 0])))
            cand_t.append(time_graph(block(d, w)))
        mb, mc = sorted(base)[args.rounds // 2], sorted(cand_t)[args.rounds // 2]
        M = B * HW * HW
        print(f"B={B} L{li} planner d{list(C.plan_info('dgrad', M, Ci, 9 * Co))} w{list(C.plan_info('wgrad', M, Co, 9 * Ci))} "
              f"{mb:.2f} us | d{d} w{w} {mc:.2f} us ({100 * (mb - mc) / mb:+.1f} %)", flush=True)


if __name__ == "__main__":
    main()
