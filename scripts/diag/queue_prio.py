"""Diagnostic: does a side stream that waits on events of the compute stream slow the compute
stream's dispatches, and does its priority matter? Plain VGG-11 training iterations at 32 images on
one GPU; per-parameter hooks (ready order) every `every`-th gradient record an event on the compute
stream, make the side stream wait on it and record a second event there (what the reducer's bucket
launch does at one rank, where no RCCL kernel runs); the end of backward waits on the last one.
Per iteration: two back-to-back stamps after a host-ahead sleep, and the backward span."""
import sys

import torch

sys.path.insert(0, ".")
import cs744_distributed_data_parallel_amd as cdp  # noqa: E402

B = 32
C = cdp._native.lib()
hz = C.gpu_wall_clock_khz() * 1e3
crit = cdp.CrossEntropyLoss()
x = torch.randn(B, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (B,), device="cuda")


def run(name, side=None, every=8, kernel_on_side=False, iters=3, reuse_event=False, poll=False, comm=None):
    torch.manual_seed(0)
    model = cdp.VGG11().cuda()
    opt = cdp.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    params = list(model.parameters())
    n = len(params)
    ts = torch.zeros(n + 4, dtype=torch.int64, device="cuda")
    buf = torch.zeros(1024, device="cuda")
    state = {"k": 0, "last": None, "work": None, "stop": False}
    e_shared = torch.cuda.Event()
    if poll:
        import threading
        import time

        def poller():
            while not state["stop"]:
                time.sleep(0.02)
                e = state["last"]
                if e is not None:
                    e.query()

        th = threading.Thread(target=poller, daemon=True)
        th.start()

    def hook(_p, i):
        C.gpu_timestamp(ts, i)
        if side is None and comm is None:
            return
        state["k"] += 1
        if state["k"] % every:
            return
        if comm is not None:
            state["work"] = comm.all_reduce(buf, "avg", True)
            return
        cur = torch.cuda.current_stream()
        e1 = e_shared if reuse_event else torch.cuda.Event()
        e1.record(cur)
        side.wait_event(e1)
        if kernel_on_side:
            with torch.cuda.stream(side):
                buf.add_(1.0)
        e2 = torch.cuda.Event()
        e2.record(side)
        state["last"] = e2

    hooks = [p.register_post_accumulate_grad_hook(lambda _p, i=i: hook(_p, i)) for i, p in enumerate(params)]
    for it in range(iters):
        opt.zero_grad()
        loss = crit(model(x), y)
        C.gpu_sleep(5000.0)
        C.gpu_timestamp(ts, n)
        C.gpu_timestamp(ts, n + 1)
        loss.backward()
        if state["last"] is not None:
            torch.cuda.current_stream().wait_event(state["last"])
            state["last"] = None
        if state["work"] is not None:
            state["work"].wait()
            state["work"] = None
        opt.step()
        torch.cuda.synchronize()
        r = ts.cpu().tolist()
        st = sorted(r[:n])
        us = lambda a, b: (b - a) / hz * 1e6  # noqa: E731
        print(f"{name} iter {it}: back-to-back stamp {us(r[n], r[n + 1]):.1f} us, backward span "
              f"{us(st[0], st[-1]):.0f} us", flush=True)
    state["stop"] = True
    for h in hooks:
        h.remove()


lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
print("priority range", lo, hi)
WANT = set(sys.argv[1:])
if WANT:
    import os

    from cs744_distributed_data_parallel_amd import distributed as dist

    run("plain")
    run("side stream, normal priority", torch.cuda.Stream(priority=0))
    run("side stream, reused first event", torch.cuda.Stream(priority=0), reuse_event=True)
    run("side stream, event polled by a thread", torch.cuda.Stream(priority=0), poll=True)
    if "comm" in WANT:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29557")
        dist.init_process_group("rccl", rank=0, world_size=1)
        run("side stream after RCCL init", torch.cuda.Stream(priority=0))
        run("native communicator all_reduce (one rank: events only)", comm=dist.native_communicator())
        run("side stream after RCCL init, again", torch.cuda.Stream(priority=0))
    sys.exit(0)
run("plain")
run("side stream, normal priority", torch.cuda.Stream(priority=0))
run("side stream, high priority", torch.cuda.Stream(priority=-1))
run("side stream, normal priority, kernel", torch.cuda.Stream(priority=0), kernel_on_side=True)
run("side stream, high priority, kernel", torch.cuda.Stream(priority=-1), kernel_on_side=True)
run("plain again")
