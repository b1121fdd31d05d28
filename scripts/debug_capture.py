import sys, torch
import cs744_distributed_data_parallel_amd as cdp
torch.manual_seed(0)
model = cdp.VGG11().cuda()
x = torch.randn(32, 3, 32, 32, device="cuda"); y = torch.randint(0, 10, (32,), device="cuda")
crit = cdp.CrossEntropyLoss()
opt = cdp.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
what = sys.argv[1]
def body():
    if what in ("step",):
        opt.zero_grad()
    out = model(x)
    if what == "fwd":
        return out
    loss = crit(out, y)
    loss.backward()
    if what == "step":
        opt.step()
    return loss
for _ in range(3): body()
s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    body()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
try:
    with torch.cuda.graph(g):
        body()
    g.replay(); torch.cuda.synchronize()
    print(what, "CAPTURE_OK")
except Exception as e:
    print(what, "CAPTURE_FAIL", repr(e)[:300])
