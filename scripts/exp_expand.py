import torch, time, sys
sys.path.insert(0, "/root/repo")
import cs744_distributed_data_parallel_amd as cdp
C = cdp._native.lib()
cl = torch.channels_last
def t(fn, it=20):
    fn(); torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3
for (H, Cc) in [(2, 512), (4, 512), (8, 256)]:
    x = torch.randn(256, Cc, H, H, device="cuda").contiguous(memory_format=cl)
    w = (torch.randn(Cc, Cc, 3, 3, device="cuda") * 0.02).contiguous(memory_format=cl)
    xa = C.weight_prep([w], [False])[0]
    K = H * H * Cc
    xe = x.permute(0, 2, 3, 1).reshape(256, K, 1, 1).contiguous(memory_format=cl)
    we = torch.randn(K, K, 1, 1, device="cuda").contiguous(memory_format=cl) * 0.01
    base = t(lambda: C.conv2d_fwd(x, w, None, 1, 1, True))
    exp = t(lambda: C.conv2d_fwd(xe, we, None, 1, 0, True))
    gy = torch.randn(256, Cc, H, H, device="cuda").contiguous(memory_format=cl)
    gye = gy.permute(0, 2, 3, 1).reshape(256, K, 1, 1).contiguous(memory_format=cl)
    bd = t(lambda: C.conv2d_dgrad(gy, w, [256, Cc, H, H], 1, 1))
    ed = t(lambda: C.conv2d_dgrad(gye, we, [256, K, 1, 1], 1, 0))
    bw = t(lambda: C.conv2d_wgrad(gy, x, [Cc, Cc, 3, 3], 1, 1))
    ew = t(lambda: C.conv2d_wgrad(gye, xe, [K, K, 1, 1], 1, 0))
    print(f"H={H} C={Cc}: fwd {base:.1f} -> expanded {exp:.1f} us | dgrad {bd:.1f} -> {ed:.1f} | wgrad {bw:.1f} -> {ew:.1f}")
