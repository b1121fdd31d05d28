"""Helpers to run a function on W gloo ranks (one process per rank, 127.0.0.1 rendezvous)."""
import os
import socket
import sys
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, args, q, init_kwargs=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world)
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    import torch

    torch.set_num_threads(1)
    try:
        from cs744_distributed_data_parallel_amd import distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world, **(init_kwargs or {}))
        try:
            out = fn(rank, world, *args)
        finally:
            dist.destroy_process_group()
        q.put((rank, "ok", out))
    except Exception:  # pragma: no cover - reported to the parent
        q.put((rank, "err", traceback.format_exc()))


def run_ranks(fn, world=2, args=(), timeout=240, init_kwargs=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q, init_kwargs)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, status, out = q.get(timeout=timeout)
            if status != "ok":
                raise AssertionError(f"rank {rank} failed:\n{out}")
            results[rank] = out
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
    return [results[r] for r in range(world)]
