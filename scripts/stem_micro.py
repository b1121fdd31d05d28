"""Micro-run of the VGG-11 layer-0 block (stem kernels) at B=256 for profiling / PMC passes.

    rocprofv3 --kernel-trace --stats -d OUT -o run -- python scripts/stem_micro.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cs744_distributed_data_parallel_amd.ops import functional as CF  # noqa: E402


def main(reps=5, B=256):
    torch.manual_seed(0)
    conv = torch.nn.Conv2d(3, 64, 3, 1, 1).cuda()
    conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
    bn = torch.nn.BatchNorm2d(64).cuda()
    x = torch.randn(B, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    for _ in range(reps):
        out = CF.conv_bn_act(x, conv, bn, relu=True, pool=True)
        out.backward(torch.ones_like(out))
    torch.cuda.synchronize()
    print("ok", float(conv.weight.grad.abs().sum()))


if __name__ == "__main__":
    main()
