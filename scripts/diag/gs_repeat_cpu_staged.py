"""gs_repeat with the gloo gather / scatter staged through CPU tensors by hand (diagnostic: is the
run-to-run difference in torch's gloo-on-device-tensor path?)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from _dist_util import run_ranks  # noqa: E402


def _train_cpu_staged(rank, world, strategy):
    import torch.distributed as tdist

    from cs744_distributed_data_parallel_amd.parallel import comm as CM
    from test_multirank_gpu import _train_gpu

    def gather(self, t, gather_list=None, dst=0):
        torch.cuda.synchronize()
        tc = t.cpu()
        lst = [torch.empty_like(tc) for _ in range(self.size)] if self.rank == dst else None
        tdist.gather(tc, lst, dst=dst, group=self.group)
        if self.rank == dst:
            for o, s in zip(gather_list, lst):
                o.copy_(s)
        torch.cuda.synchronize()

    def scatter(self, t, scatter_list=None, src=0):
        torch.cuda.synchronize()
        tc = torch.empty(t.shape, dtype=t.dtype)
        lst = [s.cpu() for s in scatter_list] if self.rank == src else None
        tdist.scatter(tc, lst, src=src, group=self.group)
        t.copy_(tc)
        torch.cuda.synchronize()

    CM.TorchCommunicator.gather = gather
    CM.TorchCommunicator.scatter = scatter
    return _train_gpu(rank, world, strategy)


if __name__ == "__main__":
    first = None
    for k in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8):
        (a1, a3), la, _ = run_ranks(_train_cpu_staged, 2, ("gather_scatter",), timeout=300)[0]
        if first is None:
            first = (a1, a3)
            print(k, "reference", la, flush=True)
            continue
        rel = float(np.linalg.norm(a3 - first[1]) / np.linalg.norm(first[1]))
        print(k, f"step1-maxabs={float(np.abs(a1 - first[0]).max()):.2e} step3-rel={rel:.2e}", la, flush=True)
