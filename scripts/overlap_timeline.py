"""One-GPU timeline of DDP's bucketed all-reduce against backward (run under rocprofv3).

    rocprofv3 --kernel-trace --marker-trace --output-format csv -d OUT -o run -- \
        python scripts/overlap_timeline.py
    python scripts/overlap_summary.py OUT/run_kernel_trace.csv OUT/run_marker_api_trace.csv out.md

World size 1 over the native RCCL communicator: the ring all-reduce of one rank moves no data, so
each bucket's collective is made visible by the test post-op (CDP_REDUCER_TEST_POSTOP=1:1, a ~µs
``delay_scale_kernel`` with scale 1 enqueued on the communicator stream right behind the
collective) and by the roctx range ``cdp.bucket_allreduce[b]`` around the host-side launch
(CDP_ROCTX=1). The timeline then shows where in backward each bucket becomes ready and launches.
"""
import os
import sys

os.environ.setdefault("CDP_ROCTX", "1")
os.environ.setdefault("CDP_REDUCER_TEST_POSTOP", "1:1")
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import cs744_distributed_data_parallel_amd as cdp  # noqa: E402
from cs744_distributed_data_parallel_amd import distributed as dist  # noqa: E402
from cs744_distributed_data_parallel_amd.utils import profiling  # noqa: E402


def main(steps=6, B=256, cap=None):
    dist.init_process_group("rccl", rank=0, world_size=1)
    torch.manual_seed(0)
    model = cdp.DistributedDataParallel(cdp.VGG11().cuda(), bucket_cap_mb=cap)
    opt = cdp.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    crit = cdp.CrossEntropyLoss()
    x = torch.randn(B, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (B,), device="cuda")
    for i in range(steps):
        with profiling.range(f"step{i}"):
            with profiling.range("forward"):
                opt.zero_grad()
                out = model(x)
            with profiling.range("backward"):
                loss = crit(out, y)
                loss.backward()
            with profiling.range("optimizer.step"):
                opt.step()
    torch.cuda.synchronize()
    print("buckets (bytes):", model.bucket_sizes_bytes())
    dist.destroy_process_group()


if __name__ == "__main__":
    main(cap=float(sys.argv[1]) if len(sys.argv) > 1 else None)
