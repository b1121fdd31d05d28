"""Which general-pool tensors does a captured VGG-11 step reference after they were freed? Records
the caching allocator's history around the capture and lists every block that was allocated before
the capture began and freed after, with the Python frames of its allocation."""
import torch

import cs744_distributed_data_parallel_amd as cdp

crit = cdp.CrossEntropyLoss()
g = torch.Generator(device="cuda").manual_seed(1)
xb = torch.randn(32, 3, 32, 32, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
yb = torch.randint(0, 10, (32,), device="cuda", generator=g)
torch.manual_seed(0)
m = cdp.VGG11().cuda()
o = cdp.SGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)


def body():
    o.zero_grad()
    loss = crit(m(xb), yb)
    loss.backward()
    o.step()
    return loss


for _ in range(4):
    body()
torch.cuda.memory._record_memory_history(max_entries=200000)
s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    body()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
MARK = torch.empty(12345, dtype=torch.uint8, device="cuda")  # marker allocation: capture begins after it
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    lo = body()
torch.cuda.synchronize()
MARK2 = torch.empty(54321, dtype=torch.uint8, device="cuda")
snap = torch.cuda.memory._snapshot()
torch.cuda.memory._record_memory_history(enabled=None)
ev = snap["device_traces"][0]
t0 = next(i for i, e in enumerate(ev) if e["action"] == "alloc" and e["size"] in (12345, 12800))  # 12345 rounded to 512
t1 = next(i for i, e in enumerate(ev) if e["action"] == "alloc" and e["size"] in (54321, 54784))
live_before = {}
for e in ev[:t0]:
    if e["action"] == "alloc":
        live_before[e["addr"]] = e
    elif e["action"] in ("free_requested", "free_completed"):
        live_before.pop(e["addr"], None)
print("capture window events", t1 - t0)
seen = set()
for e in ev[t0:t1]:
    if e["action"] == "free_requested" and e["addr"] in live_before and e["addr"] not in seen:
        seen.add(e["addr"])
        a = live_before[e["addr"]]
        fr = [f"{f['filename'].split('/')[-1]}:{f['line']}:{f['name']}" for f in a.get("frames", [])
              if "cs744" in f["filename"] or "scripts" in f["filename"]][:6]
        fr2 = [f"{f['filename'].split('/')[-1]}:{f['line']}:{f['name']}" for f in e.get("frames", [])
               if "cs744" in f["filename"] or "scripts" in f["filename"]][:4]
        print(f"freed in capture: {a['size']} B stream {a.get('stream')} alloc@ {fr} free@ {fr2}")
from collections import Counter

allocs = [e for e in ev[t0:t1] if e["action"] == "alloc"]
cnt = Counter(e.get("stream") for e in allocs)
print("allocs in capture window by stream:", dict(cnt))
main = cnt.most_common(1)[0][0]
for e in allocs:
    if e.get("stream") != main:
        fr = [f"{f['filename'].split('/')[-1]}:{f['line']}:{f['name']}" for f in e.get("frames", [])
              if "cs744" in f["filename"] or "scripts" in f["filename"]][:6]
        print(f"alloc on stream {e.get('stream')}: {e['size']} B @ {fr}")
segs = {}
for seg in snap["segments"]:
    segs[seg["address"]] = (seg["total_size"], tuple(seg.get("segment_pool_id", (0, 0))))
def pool_of(addr):
    for a, (n, p) in segs.items():
        if a <= addr < a + n:
            return p
    return None
pc = Counter(pool_of(e["addr"]) for e in allocs)
print("allocs in capture window by pool:", dict(pc))
for e in allocs:
    if pool_of(e["addr"]) == (0, 0):
        fr = [f"{f['filename'].split('/')[-1]}:{f['line']}:{f['name']}" for f in e.get("frames", [])
              if "cs744" in f["filename"] or "scripts" in f["filename"]][:6]
        print(f"general-pool alloc in capture: {e['size']} B stream {e.get('stream')} @ {fr}")
