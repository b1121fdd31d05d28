"""Where do the small-K 1x1 GEMMs of ResNet-50 layer 1 lose time? Times conv2d_fwd on
200704 x 256 x 64 (and 200704 x 64 x 64, 50176 x 512 x 128) with / without the BN-partials
epilogue, against a plain write (fill) and a read+write (copy) of the same output bytes."""
import torch

import cs744_distributed_data_parallel_amd as cdp

C = cdp._native.lib()


def t(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


for (N, Ci, HW, Co) in [(64, 64, 56, 256), (64, 64, 56, 64), (64, 128, 28, 512), (64, 256, 56, 64)]:
    x = torch.randn(N, Ci, HW, HW, device="cuda").contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Co, Ci, 1, 1, device="cuda") * 0.1).contiguous(memory_format=torch.channels_last)
    xa = C.act_max(x)
    y = torch.empty(N, Co, HW, HW, device="cuda").contiguous(memory_format=torch.channels_last)
    M = N * HW * HW
    out_b = M * Co * 4
    in_b = M * Ci * 4
    t_stats = t(lambda: C.conv2d_fwd(x, w, None, 1, 0, True, xa))
    t_plain = t(lambda: C.conv2d_fwd(x, w, None, 1, 0, False, xa))
    t_fill = t(lambda: y.fill_(1.0))
    y2 = torch.empty_like(y)
    t_copy = t(lambda: y2.copy_(y))
    print(f"M={M} N={Co} K={Ci}: fwd+stats {t_stats:.1f} us ({(in_b + out_b) / t_stats / 1e6:.2f} TB/s), "
          f"fwd {t_plain:.1f} us, fill {t_fill:.1f} us ({out_b / t_fill / 1e6:.2f} TB/s), "
          f"copy {t_copy:.1f} us ({2 * out_b / t_copy / 1e6:.2f} TB/s)", flush=True)

# tile sweep of the forward GEMMs (planner choice first)
for (N, Ci, HW, Co) in [(64, 64, 56, 256), (64, 128, 28, 512), (64, 64, 56, 64), (64, 256, 56, 128)]:
    x = torch.randn(N, Ci, HW, HW, device="cuda").contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Co, Ci, 1, 1, device="cuda") * 0.1).contiguous(memory_format=torch.channels_last)
    xa = C.act_max(x)
    M = N * HW * HW
    res = []
    for bm, bn in [(0, 0), (256, 128), (128, 128), (64, 128), (128, 64), (64, 64)]:
        if bn and Co % bn:
            continue
        C.set_gemm_override("conv", bm, bn, 1 if bm else 0)
        res.append(f"{bm}x{bn}: {t(lambda: C.conv2d_fwd(x, w, None, 1, 0, True, xa)):.1f}")
    C.set_gemm_override("conv")
    print(f"sweep M={M} N={Co} K={Ci}: " + ", ".join(res), flush=True)
