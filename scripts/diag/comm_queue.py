"""Diagnostic: which hardware queue does each stream land on, and does sharing one with the compute
stream explain the comm-stream stall?

One GPU, VGG-11 backward at 32 images (the reference's 8-rank strong-scaling point). Every 8th
gradient hook records an event on the compute stream, makes the side stream wait on it and runs a
small kernel there (a bucket launch's shape at one rank), so the side stream's kernels appear in a
rocprofv3 kernel trace with their Queue_Id next to the compute kernels'. Run once per side-stream
kind (argv[1]): none | pool (torch.cuda.Stream) | own (hipStreamCreateWithPriority, non-blocking,
normal priority, created after PyTorch's pool) | own_low (least priority) | cumask (full CU mask) |
own_first (created before anything touches PyTorch's stream pool). Prints the backward span per
iteration; `python scripts/diag/comm_queue.py summary <kernel_trace.csv>` tabulates queues.
"""
import csv
import sys

import torch

sys.path.insert(0, ".")


def summary(path):
    rows = list(csv.DictReader(open(path)))
    qcol = next(c for c in ("Queue_Id", "Stream_Id") if c in rows[0])
    by = {}
    for r in rows:
        nm = r["Kernel_Name"].split("(")[0].split("<")[0]
        side = "side" if ("add" in nm.lower() or "elementwise" in nm.lower()) else "compute"
        by.setdefault((side, r[qcol]), 0)
        by[(side, r[qcol])] += 1
    print("| stream role | queue | kernels |\n|---|---|---|")
    for (side, q), n in sorted(by.items()):
        print(f"| {side} | {q} | {n} |")


if len(sys.argv) > 1 and sys.argv[1] == "summary":
    summary(sys.argv[2])
    sys.exit(0)

kind = sys.argv[1] if len(sys.argv) > 1 else "pool"
import cs744_distributed_data_parallel_amd as cdp  # noqa: E402

C = cdp._native.lib()
side = None
raw = []  # raw HIP streams of this run, destroyed before the interpreter (and HIP) tear down


def ext_stream(*a):
    raw.append(C.create_stream(*a))
    return torch.cuda.ExternalStream(raw[-1])


if kind == "own_first":
    side = ext_stream(0, True, False)
B = 32
hz = C.gpu_wall_clock_khz() * 1e3
print("stream priority range (least, greatest):", C.stream_priority_range(), flush=True)
crit = cdp.CrossEntropyLoss()
x = torch.randn(B, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (B,), device="cuda")
torch.cuda.Stream()  # PyTorch's pool is initialised from here on
if kind == "pool":
    side = torch.cuda.Stream()
elif kind == "own":
    side = ext_stream(0, True, False)
elif kind == "own_low":
    side = ext_stream(C.stream_priority_range()[0], True, False)
elif kind == "cumask":
    side = ext_stream(0, True, True)

torch.manual_seed(0)
model = cdp.VGG11().cuda()
opt = cdp.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
params = list(model.parameters())
n = len(params)
ts = torch.zeros(n + 4, dtype=torch.int64, device="cuda")
buf = torch.zeros(1 << 16, device="cuda")
state = {"k": 0, "last": None}


def hook(_p, i):
    C.gpu_timestamp(ts, i)
    if side is None:
        return
    state["k"] += 1
    if state["k"] % 8:
        return
    e1 = torch.cuda.Event()
    e1.record(torch.cuda.current_stream())
    side.wait_event(e1)
    with torch.cuda.stream(side):
        buf.add_(1.0)
    e2 = torch.cuda.Event()
    e2.record(side)
    state["last"] = e2


hooks = [p.register_post_accumulate_grad_hook(lambda _p, i=i: hook(_p, i)) for i, p in enumerate(params)]
for it in range(4):
    opt.zero_grad()
    loss = crit(model(x), y)
    C.gpu_sleep(5000.0)
    loss.backward()
    if state["last"] is not None:
        torch.cuda.current_stream().wait_event(state["last"])
        state["last"] = None
    opt.step()
    torch.cuda.synchronize()
    st = sorted(ts.cpu().tolist()[:n])
    print(f"{kind} iter {it}: backward span {(st[-1] - st[0]) / hz * 1e6:.0f} us", flush=True)
torch.cuda.synchronize()
side = None
for s_ in raw:
    C.destroy_stream(s_)
print("side streams destroyed", flush=True)
