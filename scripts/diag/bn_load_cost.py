"""Consumer-side cost of BatchNorm on the conv operand load.

For each consumer conv of the fused design -- VGG-11's unpooled consumers at 32 / 64 images and
ResNet-50's bottleneck convs at 64 images -- times, in a hipGraph of R replays:
  plain : conv2d_fwd on a materialized activation (what the GEMM costs today)
  bnload: conv2d_fwd on the raw producer output with bn_stats (the same GEMM plus the transform)
  apply : the BatchNorm-apply pass the design removes (torch addcmul + clamp as a stand-in for the
          bandwidth of bn_act_fwd; the real kernel numbers are in profiles/)
Prints a markdown table of us per call.
"""
import sys

import torch

sys.path.insert(0, ".")
import cs744_distributed_data_parallel_amd as cdp  # noqa: E402

C = cdp._native.lib()
C.set_conv_gemm("f16x2")
R = 50
CASES = [
    ("vgg L3 in (32 img)", 32, 256, 8, 8, 256, 3, 1, 1),
    ("vgg L5 in (32 img)", 32, 512, 4, 4, 512, 3, 1, 1),
    ("vgg L7 in (32 img)", 32, 512, 2, 2, 512, 3, 1, 1),
    ("vgg L3 in (64 img)", 64, 256, 8, 8, 256, 3, 1, 1),
    ("vgg L5 in (64 img)", 64, 512, 4, 4, 512, 3, 1, 1),
    ("vgg L3 in (256 img)", 256, 256, 8, 8, 256, 3, 1, 1),
    ("rn50 l1 conv2 (64 img)", 64, 64, 56, 56, 64, 3, 1, 1),
    ("rn50 l1 conv3 (64 img)", 64, 64, 56, 56, 256, 1, 1, 0),
    ("rn50 l2 conv2 s2 (64 img)", 64, 128, 56, 56, 128, 3, 2, 1),
    ("rn50 l3 conv3 (64 img)", 64, 256, 14, 14, 1024, 1, 1, 0),
    ("rn50 l4 conv2 (64 img)", 64, 512, 7, 7, 512, 3, 1, 1),
]


def timed(fn):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g.capture_begin()
        for _ in range(R):
            fn()
        g.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / R)
    return best


print("| consumer conv | plain GEMM us | GEMM + BN on load us | delta us | apply pass (torch) us |")
print("|---|---|---|---|---|")
for name, N, Ci, H, W, Co, k, stride, pad in CASES:
    y = torch.randn(N, Ci, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Co, Ci, k, k, device="cuda") / (Ci * k * k) ** 0.5).contiguous(memory_format=torch.channels_last)
    st = torch.zeros(4, Ci, device="cuda")
    st[2].uniform_(0.5, 1.5)
    st[3].uniform_(-0.2, 0.2)
    act = torch.addcmul(st[3].view(1, Ci, 1, 1), y, st[2].view(1, Ci, 1, 1)).clamp_min(0)
    act = act.contiguous(memory_format=torch.channels_last)
    am = C.act_max(act)
    wm = C.weight_prep([w], [False])[0][0]
    out = torch.empty_like(act)
    t_plain = timed(lambda: C.conv2d_fwd(act, w, None, stride, pad, True, am, wm))
    t_bn = timed(lambda: C.conv2d_fwd(y, w, None, stride, pad, True, am, wm, st, True))
    t_apply = timed(lambda: torch.clamp_min(torch.addcmul(st[3].view(1, Ci, 1, 1), y, st[2].view(1, Ci, 1, 1)), 0,
                                            out=out))
    print(f"| {name} | {t_plain:.2f} | {t_bn:.2f} | {t_bn - t_plain:+.2f} | {t_apply:.2f} |", flush=True)
