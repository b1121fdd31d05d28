"""Is a captured VGG-11 training step (plain model, end-of-step SGD) deterministic across processes?
Prints the loss of 10 eager steps and 12 replays at full precision plus a parameter checksum; run it
in several processes (and engines, CDP_CONV_GEMM) and compare the lines."""
import sys

import torch

import cs744_distributed_data_parallel_amd as cdp

lr = float(sys.argv[1]) if len(sys.argv) > 1 else 0.05
crit = cdp.CrossEntropyLoss()
g = torch.Generator(device="cuda").manual_seed(1)
xs = [torch.randn(32, 3, 32, 32, device="cuda", generator=g).contiguous(memory_format=torch.channels_last) for _ in range(3)]
ys = [torch.randint(0, 10, (32,), device="cuda", generator=g) for _ in range(3)]
torch.manual_seed(0)
model = cdp.VGG11().cuda()
opt = cdp.SGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)
xb = torch.empty_like(xs[0]); yb = torch.empty_like(ys[0])


def body():
    opt.zero_grad()
    loss = crit(model(xb), yb)
    loss.backward()
    opt.step()
    return loss


def csum():
    return sum(float(p.double().abs().sum()) for p in model.parameters())


out = []
for step in range(4):
    xb.copy_(xs[step % 3]); yb.copy_(ys[step % 3])
    out.append(f"{body().item():.9g}")
print("eager", " ".join(out), f"{csum():.15g}", flush=True)
s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    body()
torch.cuda.current_stream().wait_stream(s)
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    lo = body()
torch.cuda.synchronize()
out = []
for step in range(12):
    xb.copy_(xs[step % 3]); yb.copy_(ys[step % 3])
    gr.replay()
    out.append(f"{lo.item():.9g}")
print("replay", " ".join(out), f"{csum():.15g}", flush=True)
