"""Diagnose the single-device overlapped step under hipGraph replay: which parameters diverge from
the end-of-step SGD after the first replay, for several bucket caps."""
import sys

import torch

import cs744_distributed_data_parallel_amd as cdp

cap = float(sys.argv[1])
order = (True, False) if len(sys.argv) > 2 and sys.argv[2] == "swap" else (False, True)
# which runs overlap: "bo" = first plain, second overlapped (default); "bb" = both plain; "oo" = both overlapped
kinds = sys.argv[3] if len(sys.argv) > 3 else "bo"
crit = cdp.CrossEntropyLoss()
g = torch.Generator(device="cuda").manual_seed(1)
xs = [torch.randn(32, 3, 32, 32, device="cuda", generator=g).contiguous(memory_format=torch.channels_last) for _ in range(3)]
ys = [torch.randint(0, 10, (32,), device="cuda", generator=g) for _ in range(3)]


def make(variant):
    torch.manual_seed(0)
    model = cdp.VGG11().cuda()
    opt = cdp.SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    if kinds[int(variant)] == "o":
        model = cdp.parallel.overlapped_step(model, opt, bucket_cap_mb=cap)
    return model, opt


runs = {k: make(k) for k in (False, True)}
xb = torch.empty_like(xs[0]); yb = torch.empty_like(ys[0])
names = [n for n, _ in runs[False][0].named_parameters()]


def body(model, opt):
    opt.zero_grad()
    loss = crit(model(xb), yb)
    loss.backward()
    opt.step()
    return loss


def prep_ok(k):
    m = runs[k][0]
    mod = m.module if hasattr(m, "module") else m
    arena = next(mod.parameters())._cdp_arena
    if arena._prep_plan is None or arena.prep_request is None:
        return "no plan"
    plan = arena._prep_plan[1]
    weights, want = arena.prep_request
    amax, wts = cdp._native.lib().weight_prep(list(weights), list(want))
    a_ok = sum(torch.equal(a, b.reshape(a.shape)) for a, b in zip(plan["amax_views"], amax)) if amax is not None else None
    w_ok = [torch.equal(a, b) for a, b in zip(plan["wts"], wts) if a is not None and b is not None]
    return f"amax {a_ok} wts {sum(w_ok)}/{len(w_ok)} valid={arena.prep_valid is not None}"


def diff(tag):
    if "-v" in sys.argv:
        print(tag, "prep base:", prep_ok(False), "| variant:", prep_ok(True), flush=True)
    pa = list(runs[False][0].parameters()); pb = list(runs[True][0].parameters())
    bad = [(n, (a - b).abs().max().item()) for n, a, b in zip(names, pa, pb) if not torch.equal(a, b)]
    ga = [p.grad for p in pa]; gb = [p.grad for p in pb]
    gbad = [n for n, a, b in zip(names, ga, gb) if a is not None and b is not None and not torch.equal(a, b)]
    print(tag, "param diffs:", bad[:8], "grad diffs:", gbad[:8], flush=True)


for step in range(4):
    xb.copy_(xs[step % 3]); yb.copy_(ys[step % 3])
    ls = [body(*runs[k]).item() for k in (False, True)]
    print("eager", step, ls, flush=True)
diff("eager")
graphs = {}
for k in order:
    m, o = runs[k]
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body(m, o)
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        lo = body(m, o)
    graphs[k] = (gr, lo)
    print("captured", k, flush=True)
torch.cuda.synchronize()
diff("after capture")
for step in range(6):
    xb.copy_(xs[step % 3]); yb.copy_(ys[step % 3])
    for k in (False, True):
        graphs[k][0].replay()
        torch.cuda.synchronize()
    print("replay", step, graphs[False][1].item(), graphs[True][1].item(), flush=True)
    diff(f"replay {step}")
