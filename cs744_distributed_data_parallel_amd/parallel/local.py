"""In-process multi-rank test double of the communicator interface (threads + shared memory).

SURVEY.md §4 asks for reducer / strategy tests that run "with an in-process multi-rank test double
of the communicator interface (threads, shared memory) so they execute without GPUs". A
:class:`LocalGroup` of ``world`` ranks runs one Python thread per rank; every collective is a
rendezvous on a shared slot table guarded by a barrier, so all ranks must issue the same
collectives in the same order -- exactly the contract of RCCL and gloo, which makes ordering bugs
(e.g. buckets launched in rank-dependent order) deadlock here too instead of passing silently.
A broken rank aborts the barrier, so the others fail fast with :class:`threading.BrokenBarrierError`.

Semantics match :class:`~.comm.TorchCommunicator` (and the reference's
``dist.gather``/``dist.scatter``/``dist.all_reduce``, ``/root/reference/src/Part 2a/main.py:117-127``,
``src/Part 2b/main.py:116-119``); reductions run in fp64 in rank order, so results are
deterministic.
"""
from __future__ import annotations

import threading
import traceback
from typing import Callable, List, Optional

import torch

from .comm import Communicator, Work, _norm_op


class LocalGroup:
    def __init__(self, world: int, timeout_s: float = 60.0):
        if world < 1:
            raise ValueError("world must be >= 1")
        self.world = world
        self.timeout_s = timeout_s
        self._slots: List[object] = [None] * world
        self._barrier = threading.Barrier(world, timeout=timeout_s)

    def communicator(self, rank: int) -> "LocalCommunicator":
        return LocalCommunicator(self, rank)

    # one rendezvous: publish, wait for everyone, read everyone, wait until all have read
    def _exchange(self, rank: int, item):
        self._slots[rank] = item
        self._barrier.wait()
        data = list(self._slots)
        self._barrier.wait()
        return data

    def run(self, fn: Callable, *args) -> list:
        """Run ``fn(rank, world, comm, *args)`` on every rank (one thread each); return results."""
        results: List[object] = [None] * self.world
        errors: List[Optional[str]] = [None] * self.world

        def body(r):
            try:
                results[r] = fn(r, self.world, self.communicator(r), *args)
            except BaseException:  # noqa: BLE001 - reported below
                errors[r] = traceback.format_exc()
                self._barrier.abort()

        threads = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(self.world)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(self.timeout_s * 4)
        first = next((e for e in errors if e and "BrokenBarrierError" not in e), None) or next(
            (e for e in errors if e), None)
        if first:
            raise RuntimeError(f"a rank of the local group failed:\n{first}")
        if any(t.is_alive() for t in threads):
            raise RuntimeError("local group timed out (collectives issued in different orders?)")
        return results


def _reduce(data: List[torch.Tensor], op: str) -> torch.Tensor:
    acc = data[0].double().clone()
    for d in data[1:]:
        d = d.double()
        if op in ("sum", "avg"):
            acc += d
        elif op == "prod":
            acc *= d
        elif op == "max":
            acc = torch.maximum(acc, d)
        elif op == "min":
            acc = torch.minimum(acc, d)
    if op == "avg":
        acc /= len(data)
    return acc


class LocalCommunicator(Communicator):
    kind = "local"

    def __init__(self, group: LocalGroup, rank: int):
        self.group, self.rank, self.size = group, rank, group.world

    def _x(self, item):
        return self.group._exchange(self.rank, item)

    def all_reduce(self, t, op="sum", async_op=False):
        data = self._x(t.detach().clone())
        t.copy_(_reduce(data, _norm_op(op)).to(t.dtype))
        return Work() if async_op else None

    def reduce(self, t, dst=0, op="sum", async_op=False):
        data = self._x(t.detach().clone())
        if self.rank == dst:
            t.copy_(_reduce(data, _norm_op(op)).to(t.dtype))
        return Work() if async_op else None

    def broadcast(self, t, src=0, async_op=False):
        data = self._x(t.detach().clone() if self.rank == src else None)
        t.copy_(data[src])
        return Work() if async_op else None

    def gather(self, t, gather_list=None, dst=0):
        data = self._x(t.detach().clone())
        if self.rank == dst:
            for out, d in zip(gather_list, data):
                out.copy_(d.view_as(out))

    def scatter(self, t, scatter_list=None, src=0):
        data = self._x([s.detach().clone() for s in scatter_list] if self.rank == src else None)
        t.copy_(data[src][self.rank].view_as(t))

    def all_gather(self, out, t, async_op=False):
        data = self._x(t.detach().clone().reshape(-1))
        out.copy_(torch.cat(data).view_as(out))
        return Work() if async_op else None

    def reduce_scatter(self, out, t, op="sum", async_op=False):
        data = self._x(t.detach().clone().reshape(-1))
        red = _reduce(data, _norm_op(op)).to(out.dtype)
        out.copy_(red.chunk(self.size)[self.rank].view_as(out))
        return Work() if async_op else None

    def all_to_all(self, out, t, async_op=False):
        data = self._x(list(t.detach().clone().reshape(-1).chunk(self.size)))
        out.copy_(torch.cat([d[self.rank] for d in data]).view_as(out))
        return Work() if async_op else None

    def send(self, t, dst):
        raise NotImplementedError("point-to-point is not modelled by the local test double")

    def recv(self, t, src):
        raise NotImplementedError("point-to-point is not modelled by the local test double")

    def barrier(self):
        self._x(None)
