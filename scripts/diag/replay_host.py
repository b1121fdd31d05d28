"""Is the replayed step host-bound early on? Captures the VGG-11 256-image training step (as
bench.py does), then for K = 20 / 60 / 200 replays measures the host time of the replay() calls
alone (enqueue) and the GPU time of the K replays (events), after a sleep that lets the GPU idle
(as the bench's capture does)."""
import time

import torch

import cs744_distributed_data_parallel_amd as cdp

torch.manual_seed(0)
dev = torch.device("cuda")
model = cdp.VGG11().to(dev)
opt = cdp.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
crit = cdp.CrossEntropyLoss()
x = torch.randn(256, 3, 32, 32, device=dev).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (256,), device=dev)
seed = None


def body():
    global seed
    opt.zero_grad()
    loss = crit(model(x), y)
    if seed is None:
        seed = torch.ones_like(loss)
    loss.backward(seed)
    opt.step()


for _ in range(5):
    body()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    body()
    body()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
cs = torch.cuda.Stream()
cs.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(cs):
    g.capture_begin()
    body()
    g.capture_end()
torch.cuda.current_stream().wait_stream(cs)
torch.cuda.synchronize()
for K in (20, 60, 200, 20, 600, 20):
    time.sleep(0.3)  # GPU idle, as during a capture
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in range(K):
        g.replay()
    t1 = time.perf_counter()
    e1.record()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"K={K}: host enqueue {1e3 * (t1 - t0) / K:.3f} ms/replay, wall {1e3 * (t2 - t0) / K:.3f}, "
          f"GPU {e0.elapsed_time(e1) / K:.3f} ms/step", flush=True)
