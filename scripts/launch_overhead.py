"""Per-dispatch cost of a chain of dependent kernels on MI355X, eager vs hipGraph replay.

Decides whether fusing the step's ~60 small BN / split-K-reduce / slab-sum kernels (each moves
only 1-16 MB) can pay: if a dependent dispatch costs ~1 us under hipGraph, fusion buys little; if it
costs several us, kernel count is the lever.

    python scripts/launch_overhead.py
"""
import time

import torch

from cs744_distributed_data_parallel_amd import _native


def timed(fn, reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    C = _native.lib()
    dev = torch.device("cuda:0")
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    sizes = {"1 thread": None, "64 KiB": 1 << 14, "2 MiB": 1 << 19, "8 MiB": 1 << 21, "32 MiB": 1 << 23}
    for name, n in sizes.items():
        x = torch.ones(n or 1, device=dev)
        for chain in (50, 200):
            def body():
                for _ in range(chain):
                    if n is None:
                        C.counter_inc(ctr)
                    else:
                        C.scale_(x, 1.0)
            body()
            eager = timed(body, 5)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                body()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                body()
            g.replay()
            graph = timed(g.replay, 20)
            print(f"{name:>8} chain {chain:4d}: eager {eager / chain * 1e6:6.2f} us/kernel, "
                  f"graph {graph / chain * 1e6:6.2f} us/kernel", flush=True)
            del g


if __name__ == "__main__":
    main()
