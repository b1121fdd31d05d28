"""Loss trajectory of the VGG-11 bench step (256 images, 30 eager steps, fixed seed) under the
current process's CDP_TILE_STATS; prints one JSON list (compare two runs)."""
import json

import torch

import cs744_distributed_data_parallel_amd as cdp

torch.manual_seed(0)
model = cdp.VGG11().cuda()
opt = cdp.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
crit = cdp.CrossEntropyLoss()
g = torch.Generator(device="cuda").manual_seed(1)
out = []
for i in range(30):
    x = torch.randn(256, 3, 32, 32, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (256,), device="cuda", generator=g)
    opt.zero_grad()
    loss = crit(model(x), y)
    loss.backward()
    opt.step()
    out.append(loss.item())
rm = [m.running_mean.abs().sum().item() for m in model.modules() if isinstance(m, torch.nn.BatchNorm2d)]
print(json.dumps({"loss": out, "rm": rm}))
