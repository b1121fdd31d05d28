"""Determinism + sensitivity probe: same input twice through the native model; compare to fp64 and fp32-torch."""
import torch
import cs744_distributed_data_parallel_amd as cdp

torch.manual_seed(0)
ref = cdp.VGG11(channels_last=False).double()
g = torch.Generator().manual_seed(1)
x = torch.randn(32, 3, 32, 32, generator=g)
y = torch.randint(0, 10, (32,), generator=g)

def native_grads():
    m = cdp.VGG11().cuda()
    m.load_state_dict({k: v.float().cuda() for k, v in ref.state_dict().items()})
    loss = cdp.CrossEntropyLoss()(m(x.cuda()), y.cuda())
    loss.backward()
    return {n: p.grad.detach().double().cpu() for n, p in m.named_parameters()}, m

def torch32_grads():
    m = cdp.VGG11(channels_last=False).cuda()
    m.load_state_dict({k: v.float().cuda() for k, v in ref.state_dict().items()})
    import os
    os.environ["CDP_FORCE_REFERENCE"] = "1"
    loss = torch.nn.functional.cross_entropy(m(x.cuda()), y.cuda())
    loss.backward()
    os.environ["CDP_FORCE_REFERENCE"] = "0"
    return {n: p.grad.detach().double().cpu() for n, p in m.named_parameters()}

loss_r = torch.nn.functional.cross_entropy(ref(x.double()), y)
loss_r.backward()
R = {n: p.grad for n, p in ref.named_parameters()}
A, mA = native_grads()
B, _ = native_grads()
T = torch32_grads()
for n in R:
    if "bias" in n and n.startswith("layers") and int(n.split(".")[1]) % 4 in (0, 3) and R[n].abs().max() < 1e-10:
        continue
    den = R[n].abs().max().item()
    eAB = (A[n] - B[n]).abs().max().item() / den
    eAR = (A[n] - R[n]).abs().max().item() / den
    eTR = (T[n] - R[n]).abs().max().item() / den
    print(f"{n:18s} native-vs-native {eAB:.1e}  native-vs-fp64 {eAR:.1e}  torch32-vs-fp64 {eTR:.1e}")
# where is layers.25.weight different?
d = (A["layers.25.weight"] - R["layers.25.weight"]).abs().sum((1, 2, 3))
print("layer25 out-channels with error:", (d > 1e-3 * d.max()).nonzero().flatten()[:20].tolist(), "count", int((d > 1e-3*d.max()).sum()))
