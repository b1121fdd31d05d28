"""Diagnostic: does a collective on the communicator's stream hold back the compute stream? One
GPU, native RCCL at W = 1 with the test post-op forcing a real RCCL kernel per all-reduce. Two
back-to-back one-thread stamp kernels on the compute stream while a bucket-sized all-reduce runs on
the comm stream, for the GPU_MAX_HW_QUEUES of this process (set by the caller)."""
import os
import sys

import torch

sys.path.insert(0, ".")
os.environ["CDP_REDUCER_TEST_POSTOP"] = "0:1.0000002"  # keeps the RCCL kernel at one rank
import cs744_distributed_data_parallel_amd as cdp  # noqa: E402
from cs744_distributed_data_parallel_amd import distributed as dist  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29547")
dist.init_process_group("rccl", rank=0, world_size=1)
C = cdp._native.lib()
comm = dist.native_communicator()
hz = C.gpu_wall_clock_khz() * 1e3
buf = torch.zeros(9437184 // 4, device="cuda")
ts = torch.zeros(64, dtype=torch.int64, device="cuda")
for rep in range(3):
    torch.cuda.synchronize()
    C.gpu_sleep(2000.0)  # host enqueues everything below ahead of the GPU
    C.gpu_timestamp(ts, 0)
    w = comm.all_reduce(buf, "sum", True)
    for i in range(1, 21):
        C.gpu_timestamp(ts, i)
    w.wait()
    torch.cuda.synchronize()
    r = ts.cpu().tolist()
    gaps = [(r[i + 1] - r[i]) / hz * 1e6 for i in range(0, 20)]
    print(f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES', 'default')} rep {rep}: compute-stream stamp gaps us "
          + " ".join(f"{g:.1f}" for g in gaps), flush=True)
dist.destroy_process_group()
