"""Bucket plan of the reducer for one batch size (one GPU, DDP over the native RCCL communicator at
W = 1): the measured gradient-ready timeline of an eager backward (GPU stamps per parameter hook,
what the reducer's timed planner records at its ready-order rebuild), and the plan
buckets.plan_buckets_timed designs from it for several xGMI comm models -- the W = 1 fit (no data
moves), and the W = 8 ring (2 (W-1)/W S bytes per GPU) at assumed bus bandwidths / latencies.

    python scripts/bucket_plan.py [local_batch] > profiles/vgg11_b32_ddp_overlap_r4.md
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cs744_distributed_data_parallel_amd as cdp  # noqa: E402
from cs744_distributed_data_parallel_amd import distributed as dist  # noqa: E402
from cs744_distributed_data_parallel_amd.parallel.buckets import plan_buckets, plan_buckets_timed  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dist.init_process_group("rccl", rank=0, world_size=1)
torch.manual_seed(0)
model = cdp.DistributedDataParallel(cdp.VGG11().cuda())
opt = cdp.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
crit = cdp.CrossEntropyLoss()
x = torch.randn(B, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (B,), device="cuda")
red = model.reducer
names = {id(p): n for n, p in model.module.named_parameters()}


def step():
    opt.zero_grad()
    crit(model(x), y).backward()
    opt.step()


for _ in range(3):  # warm kernels / planner caches; the third is timed by the hooks again
    red.start_ready_timing()
    step()
torch.cuda.synchronize()
rt = red._ready_times()
order = sorted(rt, key=lambda k: rt[k])
params = {id(p): p for p in red.arena.params}
nb = [params[k].numel() * 4 for k in order]
ready = [rt[k] for k in order]
alpha1, beta1 = red._measure_comm()
red.stop_ready_timing()

print(f"# VGG-11 bucket plan at {B} images per GPU (round 4, `scripts/bucket_plan.py {B}`)\n")
print("Gradient-ready timeline of the reducer's timed calibration backward on one MI355X (GPU "
      "wall-clock stamps written by the per-parameter hooks; us after the first gradient). A 5 ms GPU "
      "sleep before it lets the host enqueue the whole backward ahead, so the GPU runs it back to back "
      "as in the captured step; its bucket launches wait for its end (Reducer::finalize). The "
      "communicator fit times each all-reduce between two GPU stamps on the compute stream.\n")
print("| # | parameter | bytes | ready us |\n|---|---|---|---|")
for i, k in enumerate(order):
    print(f"| {i} | `{names.get(k, '?')}` | {nb[i]} | {ready[i] * 1e6:.1f} |")


def show(title, alpha, beta):
    g, info = plan_buckets_timed(nb, ready, alpha, beta)
    gr = plan_buckets(nb, 8.0, 1.0)

    def end(groups):
        e = float("-inf")
        for q in groups:
            e = max(e, max(ready[: q[-1] + 1])) + alpha + beta * sum(nb[i] for i in q)
        return e

    print(f"\n## {title}: alpha {alpha * 1e6:.1f} us, {1 / beta / 1e9:.0f} GB/s per GPU (algorithmic)\n")
    print("| bucket | tensors | MB | first | last | ready us |\n|---|---|---|---|---|---|")
    for j, q in enumerate(g):
        print(f"| {j} | {len(q)} | {sum(nb[i] for i in q) / 1e6:.2f} | `{names.get(order[q[0]])}` | "
              f"`{names.get(order[q[-1]])}` | {ready[q[-1]] * 1e6:.1f} |")
    print(f"\nModelled: backward ends {info['backward_end_us']} us, last all-reduce ends {info['comm_end_us']} "
          f"us, exposed {info['exposed_us']} us. The fixed 8 MiB / 1 MiB plan ({len(gr)} buckets) "
          f"would end at {(end(gr) - ready[0]) * 1e6:.1f} us.")


show("Measured W = 1 communicator (no data moves: latency only)", alpha1, max(beta1, 1e-15))
for w, busbw, alpha in ((8, 300e9, 15e-6), (8, 150e9, 15e-6), (4, 300e9, 10e-6), (2, 300e9, 8e-6)):
    show(f"W = {w} ring model, {busbw / 1e9:.0f} GB/s bus bandwidth", alpha, 2 * (w - 1) / w / busbw)
dist.destroy_process_group()
