"""The planner's GEMM plans on the GPU for every VGG-11 conv layer, and the resulting work balance
of each bwd_pair launch (data-gradient blocks first, then weight-gradient blocks)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import cs744_distributed_data_parallel_amd as cdp  # noqa: E402

C = cdp._native.lib()
torch.zeros(1, device="cuda")
cus = torch.cuda.get_device_properties(0).multi_processor_count
layers = [(64, 128, 16), (128, 256, 8), (256, 256, 8), (256, 512, 4), (512, 512, 4), (512, 512, 2), (512, 512, 2)]
for B in (256, 128, 64, 32):
    print(f"B={B} ({cus} CUs)")
    for ci, co, h in layers:
        M = B * h * h
        f = C.plan_info("conv", M, co, 9 * ci)
        d = C.plan_info("conv", M, ci, 9 * co)
        w = C.plan_info("wgrad", M, co, 9 * ci)
        nd = -(-M // d[0]) * -(-ci // d[1]) * d[2]
        kd = -(-(9 * co) // 32) // d[2]
        nw = -(-co // w[0]) * -(-(9 * ci) // w[1]) * w[2]
        kw = -(-M // 32) // w[2]
        print(f"  {ci:3d}->{co:3d}@{h:2d} fwd {f} dgrad {d} ({nd} blk x {kd} kt) wgrad {w} ({nw} blk x {kw} kt)")
