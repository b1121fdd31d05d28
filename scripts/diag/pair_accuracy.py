"""Diagnostic: conv_bn_act backward (VGG layer shapes) of each conv engine vs fp64 torch, and torch
fp32 (MIOpen) vs fp64 for scale."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
import cs744_distributed_data_parallel_amd as cdp  # noqa: E402
from cs744_distributed_data_parallel_amd.ops import functional as CF  # noqa: E402

C = cdp._native.lib()
torch.backends.cudnn.allow_tf32 = False


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm()).item()


for (B, Ci, Co, HW, pool) in [(256, 64, 128, 16, True), (32, 64, 128, 16, True), (32, 256, 256, 8, True),
                               (32, 128, 256, 8, False)]:
    torch.manual_seed(11)
    conv = torch.nn.Conv2d(Ci, Co, 3, padding=1).cuda()
    conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
    bn = torch.nn.BatchNorm2d(Co).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    x = torch.relu(torch.randn(B, Ci, HW, HW, device="cuda")).contiguous(memory_format=torch.channels_last)
    oh = HW // 2 if pool else HW
    gy = torch.randn(B, Co, oh, oh, device="cuda").contiguous(memory_format=torch.channels_last)

    def ref(dt):
        xd = x.to(dt).detach().requires_grad_()
        wd = conv.weight.to(dt).detach().requires_grad_()
        y = F.conv2d(xd, wd, conv.bias.to(dt), 1, 1)
        y = F.batch_norm(y, None, None, bn.weight.to(dt), bn.bias.to(dt), True, 0.0, bn.eps)
        y = F.relu(y)
        if pool:
            y = F.max_pool2d(y, 2, 2)
        y.backward(gy.to(dt))
        return y.detach(), xd.grad, wd.grad

    y64, dx64, dw64 = ref(torch.float64)
    y32, dx32, dw32 = ref(torch.float32)
    print(f"B={B} {Ci}->{Co} {HW} pool={pool}: torch fp32 vs fp64: y {rel(y32, y64):.2e} dx {rel(dx32, dx64):.2e} "
          f"dw {rel(dw32, dw64):.2e}")
    for eng in ["f16x2", "x3", "f32"]:
        C.set_conv_gemm(eng)
        xr = x.detach().clone().requires_grad_()
        conv.weight.grad = None
        out = CF.conv_bn_act(xr, conv, bn, relu=True, pool=pool)
        out.backward(gy)
        torch.cuda.synchronize()
        print(f"   {eng}: y {rel(out, y64):.2e} dx {rel(xr.grad, dx64):.2e} dw {rel(conv.weight.grad, dw64):.2e}")
    C.set_conv_gemm("f16x2")
