"""Diagnostic: which part of the DDP path slows the compute stream's dispatches? Variants of one
training iteration on one GPU (native RCCL at W = 1); for each, two back-to-back stamps after a
host-ahead sleep and the span of the post-accumulate-grad stamps of the backward."""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
import cs744_distributed_data_parallel_amd as cdp  # noqa: E402
from cs744_distributed_data_parallel_amd import distributed as dist  # noqa: E402

B = 32
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29551")
dist.init_process_group("rccl", rank=0, world_size=1)
C = cdp._native.lib()
comm = dist.native_communicator()
hz = C.gpu_wall_clock_khz() * 1e3
crit = cdp.CrossEntropyLoss()
x = torch.randn(B, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (B,), device="cuda")
side = torch.zeros(1024, device="cuda")


def run(name, wrap=None, pre=None, post=None, iters=4):
    torch.manual_seed(0)
    base = cdp.VGG11().cuda()
    model = wrap(base) if wrap else base
    opt = cdp.SGD(base.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    params = list(base.parameters())
    ts = torch.zeros(len(params) + 4, dtype=torch.int64, device="cuda")
    n = len(params)
    hooks = [p.register_post_accumulate_grad_hook(lambda _p, i=i: C.gpu_timestamp(ts, i)) for i, p in enumerate(params)]
    for it in range(iters):
        opt.zero_grad()
        if pre:
            pre()
        out = model(x)
        loss = crit(out, y)
        C.gpu_timestamp(ts, n + 2)
        h0 = time.perf_counter()
        C.gpu_sleep(5000.0)
        C.gpu_timestamp(ts, n)
        C.gpu_timestamp(ts, n + 1)
        h1 = time.perf_counter()
        loss.backward()
        h2 = time.perf_counter()
        C.gpu_timestamp(ts, n + 3)
        if post:
            post()
        opt.step()
        torch.cuda.synchronize()
        r = ts.cpu().tolist()
        st = sorted(r[:n])
        us = lambda a, b: (b - a) / hz * 1e6  # noqa: E731
        print(f"{name} iter {it}: back-to-back stamp {us(r[n], r[n + 1]):.1f} us, backward span "
              f"{us(st[0], st[-1]):.0f} us; sleep+stamp {us(r[n + 2], r[n]):.0f} us on GPU; host: sleep..stamps "
              f"{(h1 - h0) * 1e6:.0f} us, backward call {(h2 - h1) * 1e6:.0f} us; GPU stamps..end of backward "
              f"{us(r[n + 1], r[n + 3]):.0f} us", flush=True)
    for h in hooks:
        h.remove()
    return model


WANT = set(sys.argv[1:]) or {"plain", "ddp", "removed", "bucketed", "never", "armed", "plain2"}
if "ddp" in WANT:
    m = run("ddp", wrap=lambda b: cdp.DistributedDataParallel(b, bucket_cap_mb=8.0))
    m.reducer.remove()
if "plain" in WANT:
    run("plain")


class _NoReducer:
    iterations = 0

    def rebuild_in_ready_order(self):
        return False

    def rebind_if_stream_changed(self):
        return False

    def prepare_for_backward(self, outs):
        return None

    def remove(self):
        return None


def ddp_hooks_removed(b):
    d = cdp.DistributedDataParallel(b, bucket_cap_mb=8.0, rebuild_buckets=False)
    d.reducer.remove()  # the C++ reducer and its autograd hooks are gone
    d.reducer = _NoReducer()
    return d


if "removed" in WANT:
    run("ddp, reducer removed", wrap=ddp_hooks_removed)
holder = {}


def bucketed(b):
    holder["s"] = cdp.parallel.BucketedOverlap(b, bucket_cap_mb=8.0)
    return b


if "bucketed" in WANT:
    run("bucketed_overlap", wrap=bucketed, post=None)
    holder["s"].remove()


def native_reducer_only(b):
    from cs744_distributed_data_parallel_amd.parallel.reducer import GradReducer
    from cs744_distributed_data_parallel_amd.utils.arena import arena_for

    holder["r"] = GradReducer(arena_for([p for p in b.parameters()]), dist.communicator_for(next(b.parameters())), 8.0, 1.0)
    return b


if "never" in WANT:
    run("GradReducer constructed, never armed", wrap=native_reducer_only)
    holder["r"].remove()
if "armed" in WANT:
    run("GradReducer armed by hand", wrap=native_reducer_only, pre=lambda: holder["r"].prepare_for_backward([]))
    holder["r"].remove()
if "armed_nohooks" in WANT:
    # armed, but the backward hooks never fire (removed): only prepare_for_backward's effect
    def _arm():
        holder["r"]._impl.remove_hooks()
        holder["r"].prepare_for_backward([])
        holder["r"].disarm()
    run("GradReducer armed then disarmed, hooks removed", wrap=native_reducer_only, pre=_arm)
if "plain2" in WANT:
    run("plain again")
dist.destroy_process_group()
