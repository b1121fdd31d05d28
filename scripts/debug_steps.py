"""Multi-step check: native VGG-11 + (cdp.SGD | torch.optim.SGD) vs fp64 torch, per-step grads."""
import sys
import torch
import cs744_distributed_data_parallel_amd as cdp

mode = sys.argv[1] if len(sys.argv) > 1 else "cdp"
torch.manual_seed(0)
ref = cdp.VGG11(channels_last=False).double()
model = cdp.VGG11().cuda()
model.load_state_dict({k: v.float().cuda() for k, v in ref.state_dict().items()})
if mode == "cdp":
    opt = cdp.SGD(model.parameters(), lr=0.005, momentum=0.9, weight_decay=1e-4)
else:
    opt = torch.optim.SGD(model.parameters(), lr=0.005, momentum=0.9, weight_decay=1e-4)
opt_r = torch.optim.SGD(ref.parameters(), lr=0.005, momentum=0.9, weight_decay=1e-4)
g = torch.Generator().manual_seed(1)
for step in range(3):
    x = torch.randn(32, 3, 32, 32, generator=g)
    y = torch.randint(0, 10, (32,), generator=g)
    opt.zero_grad()
    loss = cdp.CrossEntropyLoss()(model(x.cuda()), y.cuda())
    loss.backward()
    opt_r.zero_grad()
    loss_r = torch.nn.functional.cross_entropy(ref(x.double()), y)
    loss_r.backward()
    worst = []
    for (n, p), (n2, q) in zip(model.named_parameters(), ref.named_parameters()):
        e = ((p.grad.double().cpu() - q.grad).abs().max() / q.grad.abs().max().clamp_min(1e-12)).item()
        if q.grad.abs().max() > 1e-10:
            worst.append((e, n))
    worst.sort(reverse=True)
    pw = []
    for (n, p), (n2, q) in zip(model.named_parameters(), ref.named_parameters()):
        e = ((p.detach().double().cpu() - q.detach()).abs().max() / q.abs().max().clamp_min(1e-12)).item()
        pw.append((e, n))
    pw.sort(reverse=True)
    print(f"[{mode}] step {step} loss {loss.item():.6f} ref {loss_r.item():.6f} worst grad {worst[:2]} worst param(before step) {pw[:2]}")
    opt.step()
    opt_r.step()
for (n, p), (n2, q) in zip(model.state_dict().items(), ref.state_dict().items()):
    if p.dtype.is_floating_point:
        e = ((p.double().cpu() - q).abs().max() / q.abs().max().clamp_min(1e-12)).item()
        if e > 1e-4:
            print(f"   final {n} rel {e:.2e} max|ref| {q.abs().max().item():.3e}")
