"""Per-parameter gradient check of one VGG-11 step: native (with / without flat arena) vs fp64 torch."""
import torch
import cs744_distributed_data_parallel_amd as cdp
from cs744_distributed_data_parallel_amd.utils import FlatArena

torch.manual_seed(0)
ref = cdp.VGG11(channels_last=False).double()
x = torch.randn(32, 3, 32, 32)
y = torch.randint(0, 10, (32,))
loss_r = torch.nn.functional.cross_entropy(ref(x.double()), y)
loss_r.backward()
gref = {n: p.grad for n, p in ref.named_parameters()}

for use_arena in (False, True):
    model = cdp.VGG11().cuda()
    model.load_state_dict({k: v.float().cuda() for k, v in ref.state_dict().items()})
    if use_arena:
        FlatArena(list(model.parameters()))
        model.zero_grad(set_to_none=True)
    loss = cdp.CrossEntropyLoss()(model(x.cuda()), y.cuda())
    loss.backward()
    torch.cuda.synchronize()
    print(f"--- arena={use_arena} loss {loss.item():.6f} ref {loss_r.item():.6f}")
    for n, p in model.named_parameters():
        g = p.grad.double().cpu()
        r = gref[n]
        err = ((g - r).abs().max() / r.abs().max().clamp_min(1e-30)).item()
        flag = "  <<<<" if err > 1e-3 else ""
        print(f"{n:20s} rel {err:.2e} |g| {r.abs().max().item():.3e}{flag}")
