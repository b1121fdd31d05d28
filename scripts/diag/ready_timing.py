"""Diagnostic: gradient-ready timing of an eager backward on one GPU (VGG-11), with the host-ahead
sleep: GPU wall-clock stamps from post-accumulate-grad hooks, for a plain model and under DDP at
W = 1 (native RCCL), vs the events around the whole backward and the host's own backward time."""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
import cs744_distributed_data_parallel_amd as cdp  # noqa: E402
from cs744_distributed_data_parallel_amd import distributed as dist  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
dist.init_process_group("rccl", rank=0, world_size=1)
C = cdp._native.lib()
khz = C.gpu_wall_clock_khz()
crit = cdp.CrossEntropyLoss()
x = torch.randn(B, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (B,), device="cuda")

for kind in ("plain", "ddp"):
    torch.manual_seed(0)
    base = cdp.VGG11().cuda()
    model = cdp.DistributedDataParallel(base, bucket_cap_mb=8.0) if kind == "ddp" else base
    opt = cdp.SGD(base.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    params = list(base.parameters())
    ts = torch.zeros(len(params) + 2, dtype=torch.int64, device="cuda")
    hooks = [p.register_post_accumulate_grad_hook(lambda _p, i=i: C.gpu_timestamp(ts, i)) for i, p in enumerate(params)]
    for it in range(5):
        opt.zero_grad()
        out = model(x)
        loss = crit(out, y)
        C.gpu_sleep(5000.0)
        C.gpu_timestamp(ts, len(params))
        C.gpu_timestamp(ts, len(params) + 1)
        h0 = time.perf_counter()
        loss.backward()
        h1 = time.perf_counter()
        opt.step()
        torch.cuda.synchronize()
        r = ts.cpu().tolist()
        st = sorted(r[: len(params)])
        us = lambda t: (t) / (khz * 1e3) * 1e6  # noqa: E731
        print(f"{kind} iter {it}: host backward {1e6 * (h1 - h0):.0f} us; stamps: sleep end -> first grad "
              f"{us(st[0] - r[-1]):.0f} us, first -> last grad {us(st[-1] - st[0]):.0f} us, back-to-back stamp "
              f"{us(r[-1] - r[-2]):.1f} us", flush=True)
    for h in hooks:
        h.remove()
    if kind == "ddp":
        model.reducer.remove()
dist.destroy_process_group()
