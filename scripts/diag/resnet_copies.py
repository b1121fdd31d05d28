"""Diagnostic: where do ResNet-50's per-step device copies
(`__amd_rocclr_copyBuffer` in the kernel traces) come from? Two eager training steps at 64 images
under torch.profiler with Python stacks; prints every aten::copy_ / to / contiguous call site that
launched device work, grouped, with counts per step."""
import collections
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, ".")
import cs744_distributed_data_parallel_amd as cdp  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
model = cdp.get_model("resnet50").cuda()
opt = cdp.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
crit = cdp.CrossEntropyLoss()
x = torch.randn(B, 3, 224, 224, device="cuda").contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (B,), device="cuda")


def step():
    opt.zero_grad()
    crit(model(x), y).backward()
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    for _ in range(2):
        step()
    torch.cuda.synchronize()
sites = collections.Counter()
for ev in prof.events():
    if ev.name in ("aten::copy_", "aten::_to_copy", "aten::clone", "aten::contiguous", "aten::fill_", "aten::zero_"):
        stack = [s for s in (ev.stack or []) if "cs744" in s or "bench" in s or "torch/nn" in s][:3]
        sites[(ev.name, " <- ".join(stack) or "(no python frame)")] += 1
print(f"| op | call site | per step |\n|---|---|---|")
for (name, site), n in sites.most_common(40):
    print(f"| {name} | {site} | {n / 2:.1f} |")
kern = collections.Counter(e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA)
print("\n| device kernel | per step |\n|---|---|")
for k, n in kern.most_common(60):
    if "copy" in k.lower() or "Memcpy" in k or "fill" in k.lower() or "elementwise" in k.lower():
        print(f"| {k[:90]} | {n / 2:.1f} |")
