"""Per-parameter gradient differences of the channel-owner BN fusion (CDP_CHAN) against the unfused
path and against an fp64 torch reference, VGG-11 at a given batch (diagnostic)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import cs744_distributed_data_parallel_amd as cdp  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
torch.manual_seed(0)
model = cdp.VGG11().cuda()
init = {k: v.clone() for k, v in model.state_dict().items()}
x = torch.randn(B, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
t = torch.randint(0, 10, (B,), device="cuda")
crit = cdp.CrossEntropyLoss()


def run(env):
    for k, v in env.items():
        os.environ[k] = v
    model.load_state_dict(init)
    model.zero_grad(set_to_none=True)
    loss = crit(model(x), t)
    loss.backward()
    torch.cuda.synchronize()
    return [p.grad.detach().double().cpu().clone() for p in model.parameters()]


ref = cdp.VGG11(channels_last=False).double()
ref.load_state_dict({k: v.double().cpu() for k, v in init.items()})
os.environ["CDP_FORCE_REFERENCE"] = "1"
ref.zero_grad(set_to_none=True)
torch.nn.CrossEntropyLoss()(ref(x.double().cpu().contiguous()), t.cpu()).backward()
g64 = [p.grad.detach().clone() for p in ref.parameters()]
os.environ.pop("CDP_FORCE_REFERENCE")
arms = {
    "chan": {"CDP_CHAN": "1", "CDP_CHAN_MAXROWS": "8192"},
    "chan4096": {"CDP_CHAN": "1", "CDP_CHAN_MAXROWS": "4096"},
    "nochan": {"CDP_CHAN": "0"},
}
res = {k: run(v) for k, v in arms.items()}
names = [n for n, _ in model.named_parameters()]
print(f"B={B}  rel L2 error per parameter")
print("param".ljust(20) + "".join(k.rjust(12) for k in arms) + "chan-vs-no".rjust(12))
for i, n in enumerate(names):
    b = g64[i]
    row = [((res[k][i] - b).norm() / b.norm().clamp_min(1e-30)).item() for k in arms]
    d = ((res["chan"][i] - res["nochan"][i]).norm() / res["nochan"][i].norm().clamp_min(1e-30)).item()
    print(n.ljust(20) + "".join(f"{e:12.2e}" for e in row) + f"{d:12.2e}")
