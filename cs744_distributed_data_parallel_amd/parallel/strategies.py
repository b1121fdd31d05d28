"""The four gradient-synchronisation strategies of the reference, on the MI355X communicator.

=====================  ==============================================  =====================================
name                   what it does                                    reference
=====================  ==============================================  =====================================
``gather_scatter``     per parameter: gather to rank 0, mean, scatter  ``src/Part 2a/main.py:117-127``
``allreduce_blocking`` per parameter: blocking all_reduce(SUM), /= W   ``src/Part 2b/main.py:116-119``
``bucketed_overlap``   autograd-hook bucketed all-reduce overlapped    north-star "Part 2b" (BASELINE.json)
                       with backward (native C++ reducer)
``ddp``                :class:`~.ddp.DistributedDataParallel` wrapper  ``src/Part 3/main.py:61``
=====================  ==============================================  =====================================

The first two are called between ``loss.backward()`` and ``optimizer.step()`` exactly like the
reference's ``average_gradients(model[, rank])``; all four leave ``p.grad`` holding the average
over ranks, so with identical seeds they produce the same training trajectory (SURVEY.md §4,
"equivalence oracle").
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import _native
from .comm import Communicator


def flat_alias(t: torch.Tensor) -> torch.Tensor:
    """1-D alias of a dense tensor's memory (any dense stride order, e.g. channels_last)."""
    if t.is_contiguous():
        return t.view(-1)
    return t.as_strided((t.numel(),), (1,), t.storage_offset())


def _comm(t, comm: Optional[Communicator]) -> Communicator:
    if comm is not None:
        return comm
    from .. import distributed as D

    return D.communicator_for(t)


def _mean_of(inputs, out):
    if out.is_cuda and not _native.force_reference():
        _native.lib().stack_mean(inputs, out)
    else:
        out.copy_(torch.mean(torch.stack(inputs), dim=0))


def _scale(t, a):
    if t.is_cuda and not _native.force_reference():
        _native.lib().scale_(t, a)
    else:
        t.mul_(a)


@torch.no_grad()
def average_gradients_gather_scatter(model, rank: Optional[int] = None, comm: Optional[Communicator] = None):
    """Part 2a: rank 0 gathers every gradient, averages and scatters it back (one param at a time)."""
    for p in model.parameters():
        if p.grad is None:
            continue
        c = _comm(p.grad, comm)
        r = c.rank if rank is None else rank
        g = flat_alias(p.grad)
        if r == 0:
            inputs = [torch.empty_like(g) for _ in range(c.size)]
            c.gather(g, inputs, 0)
            avg = torch.empty_like(g)
            _mean_of(inputs, avg)
            c.scatter(g, [avg for _ in range(c.size)], 0)
        else:
            c.gather(g, None, 0)
            c.scatter(g, None, 0)


@torch.no_grad()
def average_gradients_allreduce(model, comm: Optional[Communicator] = None):
    """Part 2b: blocking per-parameter ``all_reduce(SUM)`` then ``grad /= world_size``."""
    for p in model.parameters():
        if p.grad is None:
            continue
        c = _comm(p.grad, comm)
        g = flat_alias(p.grad)
        c.all_reduce(g, "sum")
        _scale(g, 1.0 / c.size)


# reference names (src/Part 2a/main.py:117, src/Part 2b/main.py:116)
average_gradients = average_gradients_gather_scatter


class BucketedOverlap:
    """Backward-hook bucketed all-reduce overlapped with autograd, on a plain (unwrapped) model.

    Usage mirrors the reference's explicit-sync stages::

        sync = BucketedOverlap(model)
        out = model(x); sync.prepare(out)      # arm the hooks for this backward
        loss.backward()                        # buckets all-reduce while backward runs
        optimizer.step()                       # grads already averaged
    """

    def __init__(self, model, comm: Optional[Communicator] = None, bucket_cap_mb: float = None,
                 first_bucket_cap_mb: float = None, find_unused_parameters: bool = False,
                 rebuild_in_ready_order: bool = True):
        from ..utils.arena import arena_for
        from .buckets import DEFAULT_BUCKET_CAP_MB, DEFAULT_FIRST_BUCKET_CAP_MB
        from .reducer import GradReducer

        params = [p for p in model.parameters() if p.requires_grad]
        self.comm = _comm(params[0], comm)
        self.arena = arena_for(params)
        self.reducer = GradReducer(
            self.arena,
            self.comm,
            bucket_cap_mb if bucket_cap_mb is not None else DEFAULT_BUCKET_CAP_MB,
            first_bucket_cap_mb if first_bucket_cap_mb is not None else DEFAULT_FIRST_BUCKET_CAP_MB,
            find_unused_parameters,
            timed_plan=bucket_cap_mb is None and first_bucket_cap_mb is None and rebuild_in_ready_order,
        )
        self._rebuild = rebuild_in_ready_order
        self._rebuilt = False
        # bucket rebuild and AccumulateGrad re-binding must happen BEFORE the forward that builds
        # the autograd graph: afterwards that graph holds the old AccumulateGrad nodes (bound to
        # the stream they were created on, illegal to run inside a hipGraph capture on another)
        self._pre_hook = model.register_forward_pre_hook(self._before_forward)

    def _before_forward(self, module, inputs):
        if not torch.is_grad_enabled():
            return None
        if self._rebuild and not self._rebuilt and self.reducer.iterations >= 1:
            self.reducer.rebuild_in_ready_order()
            self._rebuilt = True
        self.reducer.rebind_if_stream_changed()
        return None

    def remove(self):
        """Detach from the model (autograd hooks and the forward pre-hook)."""
        self._pre_hook.remove()
        self.reducer.remove()

    def prepare(self, *outputs):
        outs = []
        for o in outputs:
            if isinstance(o, torch.Tensor):
                outs.append(o)
            elif isinstance(o, (list, tuple)):
                outs.extend(x for x in o if isinstance(x, torch.Tensor))
        self.reducer.prepare_for_backward(outs)

    def __call__(self, model=None):  # strategy-callable form (no-op: sync already happened in backward)
        return None


STRATEGIES = ("gather_scatter", "allreduce_blocking", "bucketed_overlap", "ddp", "none")
