"""Does a replayed hipGraph step compute bitwise what the same step computes eagerly? Model E steps
eagerly, model G (same init) by replaying its captured step, both on the same batches; parameters
are compared after every step. argv[1] = "second": capture a third model's step after G's (never
replayed) -- does a later capture perturb an earlier live graph?"""
import sys

import torch

import cs744_distributed_data_parallel_amd as cdp

second = len(sys.argv) > 1 and sys.argv[1] == "second"
# "eager" / "graph": run only E (eager) or only G (replayed) and print the losses
only = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] in ("eager", "graph") else None
# E's work between replays: "step" (default), "fwd" (no_grad forward), "fwdbwd" (no SGD);
# "grab": after G's capture, hold every free cached block of the general pool (E cannot reuse them)
ework = sys.argv[2] if len(sys.argv) > 2 else "step"
grab = "grab" in sys.argv
crit = cdp.CrossEntropyLoss()
g = torch.Generator(device="cuda").manual_seed(1)
xs = [torch.randn(32, 3, 32, 32, device="cuda", generator=g).contiguous(memory_format=torch.channels_last) for _ in range(3)]
ys = [torch.randint(0, 10, (32,), device="cuda", generator=g) for _ in range(3)]
xb = torch.empty_like(xs[0]); yb = torch.empty_like(ys[0])


def make():
    torch.manual_seed(0)
    m = cdp.VGG11().cuda()
    return m, cdp.SGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)


E, G = make(), make()


def body(m, o):
    o.zero_grad()
    loss = crit(m(xb), yb)
    loss.backward()
    o.step()
    return loss


def cmp(tag):
    d = [(n, (a - b).abs().max().item()) for (n, a), b in zip(E[0].named_parameters(), G[0].parameters())
         if not torch.equal(a, b)]
    print(tag, "equal" if not d else f"{len(d)} differ, max {max(v for _, v in d):.3g} first {d[0][0]}", flush=True)


def prep_ok(m):
    arena = next(m.parameters())._cdp_arena
    if arena._prep_plan is None or arena.prep_request is None:
        return "no plan"
    plan = arena._prep_plan[1]
    weights, want = arena.prep_request
    amax, wts = cdp._native.lib().weight_prep(list(weights), list(want))
    a_ok = sum(torch.equal(a, b.reshape(a.shape)) for a, b in zip(plan["amax_views"], amax))
    w_ok = sum(torch.equal(a, b) for a, b in zip(plan["wts"], wts) if a is not None and b is not None)
    return f"amax {a_ok}/{len(amax)} wts {w_ok} valid={arena.prep_valid is not None}"


def bufs_equal():
    be = all(torch.equal(a, b) for a, b in zip(E[0].buffers(), G[0].buffers()))
    me = all(torch.equal(E[1].state[a]["momentum_buffer"], G[1].state[b]["momentum_buffer"])
             for a, b in zip(E[0].parameters(), G[0].parameters()))
    return f"buffers equal {be} momentum equal {me}"


def capture(m, o):
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body(m, o)
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        lo = body(m, o)
    torch.cuda.synchronize()
    return gr, lo


if only:
    M = make()
    k, out = 0, []
    for _ in range(5):
        xb.copy_(xs[k % 3]); yb.copy_(ys[k % 3]); k += 1
        out.append(body(*M).item())
    if only == "graph":
        k -= 1  # the capture's side-stream warmup step replaces the fifth eager step
        M = make()
        for _ in range(4):
            xb.copy_(xs[0 if False else 0] if False else xs[(_) % 3]); yb.copy_(ys[_ % 3])
            body(*M)
        k = 4
        xb.copy_(xs[k % 3]); yb.copy_(ys[k % 3]); k += 1
        gr, lo = capture(*M)
    for i in range(12):
        xb.copy_(xs[k % 3]); yb.copy_(ys[k % 3]); k += 1
        if only == "graph":
            gr.replay()
            out.append(lo.item())
        else:
            out.append(body(*M).item())
    print(only, " ".join(f"{v:.9g}" for v in out[-12:]), flush=True)
    sys.exit(0)

k = 0
for _ in range(4):
    xb.copy_(xs[k % 3]); yb.copy_(ys[k % 3]); k += 1
    body(*E); body(*G)
cmp("eager")
xb.copy_(xs[k % 3]); yb.copy_(ys[k % 3]); k += 1
body(*E)
print("=== capture G", flush=True)
gr, lo = capture(*G)  # its side-stream warmup ran the same step
print("=== captured", flush=True)
cmp("after capture")
held = []
if grab:
    snap = torch.cuda.memory_snapshot()
    sizes = []
    for seg in snap:
        pool = tuple(seg.get("segment_pool_id", (0, 0)))
        for b in seg["blocks"]:
            if b["state"] == "inactive" and pool == (0, 0):
                sizes.append(b["size"])
    sizes.sort(reverse=True)
    print("free general-pool blocks:", len(sizes), "bytes", sum(sizes), "largest", sizes[:12], flush=True)
    for n in sizes:
        held.append(torch.empty(n, dtype=torch.uint8, device="cuda"))
if second:
    H = make()
    body(*H)
    capture(*H)
    print("captured a second model", flush=True)
for i in range(12):
    xb.copy_(xs[k % 3]); yb.copy_(ys[k % 3]); k += 1
    print(f"=== step {i}: E", flush=True)
    if ework == "step":
        le = body(*E).item()
    elif ework == "fwd":
        with torch.no_grad():
            le = crit(E[0](xb), yb).item()
    else:
        E[1].zero_grad()
        l_ = crit(E[0](xb), yb)
        l_.backward()
        le = l_.item()
    gr.replay()
    torch.cuda.synchronize()
    if ework == "step":
        cmp(f"step {i} loss {le:.9g} / {lo.item():.9g}")
    else:
        print(f"step {i} G loss {lo.item():.9g}", flush=True)
