"""Experiment: conv GEMM with in-kernel fp32->3xbf16 splitting vs pre-split operand planes, plus
pipeline ablations of the 128x128 kernel (no in-loop global loads / no in-loop LDS stores)."""
import torch

import cs744_distributed_data_parallel_amd as cdp

C = cdp._native.lib()
cases = [  # N, Ci, H, W, Co (VGG-11 layers at B=256)
    (256, 64, 16, 16, 128), (256, 128, 8, 8, 256), (256, 256, 8, 8, 256),
    (256, 256, 4, 4, 512), (256, 512, 4, 4, 512), (256, 512, 2, 2, 512)]
for (n, ci, h, w, co) in cases:
    x = torch.randn(n, ci, h, w, device="cuda").contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(co, ci, 3, 3, device="cuda") * 0.05).contiguous(memory_format=torch.channels_last)
    r = C.bench_presplit(x, wt, 1, 1, 20, False)
    t1, t2, ts, d = r[:4]
    fl = 2.0 * n * h * w * co * ci * 9
    print(f"{(n, ci, h, w, co)}: in-kernel {t1*1e3:.1f}us ({fl/t1/1e9:.0f} TF)  presplit {t2*1e3:.1f}us "
          f"({fl/t2/1e9:.0f} TF)  split3(x) {ts*1e3:.1f}us  maxdiff {d:.2e}", flush=True)
    if len(r) > 4:
        a = [f"{v*1e3:.1f}" for v in r[4:]]
        print(f"    ablations us: in-kernel noload {a[0]} nostore {a[1]} neither {a[2]} | "
              f"presplit noload {a[3]} nostore {a[4]} neither {a[5]}", flush=True)
