"""Bucketed, backward-overlapped gradient averaging (Python orchestration of the native reducer).

:class:`GradReducer` owns the bucket plan over a :class:`~..utils.arena.FlatArena` and drives the
C++ ``_C.Reducer`` (autograd post-hooks in C++, RCCL launches on the communicator's stream, see
``csrc/runtime/reducer.cpp``). A pure-Python reducer with identical semantics
(``register_post_accumulate_grad_hook`` + an engine callback) is used when the extension is not
built (CPU-only environments); both are exercised by the CPU test-suite with gloo.

Reference: the bucketed all-reduce that ``DDP(model)`` performs inside torch's Reducer
(``/root/reference/src/Part 3/main.py:61``), and the north-star "Part 2b: backward-hook bucketed
all-reduce overlapped with autograd" (BASELINE.json).
"""
from __future__ import annotations

import os

import threading
import time
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as tdist

from .. import _native
from ..utils.arena import ALIGN, FlatArena
from .buckets import DEFAULT_BUCKET_CAP_MB, DEFAULT_FIRST_BUCKET_CAP_MB, fit_comm_model, plan_buckets, plan_buckets_timed
from .comm import Communicator, RcclCommunicator, TorchCommunicator


def _aligned(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


class _PyReducer:
    """Semantics twin of ``_C.Reducer`` (used when the native extension is unavailable)."""

    def __init__(self, params, grad_views, bucket_views, bucket_starts, comm: Communicator, find_unused, average):
        self.params, self.grad_views, self.bucket_views = params, grad_views, bucket_views
        self.comm, self.find_unused, self.average = comm, find_unused, average
        nb = len(bucket_views)
        self.bucket_of = [-1] * len(params)
        self.bucket_size = [0] * nb
        for b in range(nb):
            lo, hi = sorted((bucket_starts[b], bucket_starts[b + 1]))
            for i in range(lo, hi):
                self.bucket_of[i] = b
                self.bucket_size[b] += 1
        self.pending = [0] * nb
        self.works = [None] * nb
        self.ready = [False] * len(params)
        self.armed = False
        self.next_launch = 0
        self.callback_queued = False
        self.order: List[int] = []
        self.record_order = True
        self.have_order = False
        self.iterations = 0
        self.launched_total = 0
        self._lock = threading.Lock()
        self.trace = False
        self.defer = False  # hold bucket launches until the end of backward (timed calibration)
        self.log: List[Tuple[str, int, int]] = []
        self._handles = [p.register_post_accumulate_grad_hook(self._make_hook(i)) for i, p in enumerate(params)]

    @property
    def num_buckets(self):
        return len(self.bucket_views)

    def _make_hook(self, i):
        def hook(p):
            with self._lock:
                if self.armed:
                    self._mark(i, True)

        return hook

    def remove_hooks(self):
        for h in self._handles:
            h.remove()
        self._handles = []

    def disarm(self):
        self.armed = False

    def set_trace(self, on):
        self.trace, self.log = bool(on), []

    def set_defer(self, on):
        with self._lock:
            self.defer = bool(on)

    def trace_log(self):
        return list(self.log)

    def prepare_for_backward(self, outputs):
        with self._lock:
            if self.armed and self.next_launch != 0:
                raise RuntimeError(
                    "Expected to have finished reduction in the prior iteration before starting a new one."
                )
            self.pending = list(self.bucket_size)
            self.ready = [False] * len(self.params)
            self.works = [None] * len(self.works)
            self.next_launch = 0
            self.callback_queued = False
            self.armed = True
            if not self.find_unused:
                return
            seen = set()
            stack = [o.grad_fn for o in outputs if isinstance(o, torch.Tensor) and o.grad_fn is not None]
            while stack:
                fn = stack.pop()
                if fn is None or fn in seen:
                    continue
                seen.add(fn)
                for nxt, _ in fn.next_functions:
                    if nxt is not None:
                        stack.append(nxt)
            reached = {id(getattr(fn, "variable", None)) for fn in seen if hasattr(fn, "variable")}
            for i, p in enumerate(self.params):
                if id(p) not in reached:
                    self._mark(i, False)

    def _mark(self, i, from_hook):
        if self.ready[i]:
            return
        self.ready[i] = True
        p = self.params[i]
        view = self.grad_views[i]
        if p.grad is None:
            view.zero_()
            p.grad = view
        elif p.grad.data_ptr() != view.data_ptr():
            view.copy_(p.grad)
            p.grad = view
        if from_hook:
            if self.record_order:
                self.order.append(i)
            if self.trace:
                self.log.append(("h", i, time.monotonic_ns()))
            if not self.callback_queued:
                self.callback_queued = True
                torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
        b = self.bucket_of[i]
        self.pending[b] -= 1
        if self.pending[b] == 0 and not self.defer:
            while self.next_launch < len(self.pending) and self.pending[self.next_launch] == 0:
                self._launch(self.next_launch)
                self.next_launch += 1

    def _launch(self, b):
        if self.trace:
            self.log.append(("l", b, time.monotonic_ns()))
        self.works[b] = self.comm.all_reduce(self.bucket_views[b], "avg" if self.average else "sum", async_op=True)
        self.launched_total += 1

    def _finalize(self):
        with self._lock:
            if not self.armed:
                return
            if self.trace:
                self.log.append(("f", -1, time.monotonic_ns()))
            # parameters whose hook never fired are marked ready FIRST, so the launch loop below
            # counts every bucket -- also in the deferred (calibration) iteration (csrc reducer.cpp)
            missing = [i for i, r in enumerate(self.ready) if not r]
            if missing and not self.find_unused:
                self.armed = False
                raise RuntimeError(
                    f"DistributedDataParallel: parameters with indices {missing} did not receive gradients "
                    "in this iteration. Enable find_unused_parameters=True."
                )
            for i in missing:
                self._mark(i, False)
            while self.next_launch < len(self.pending) and self.pending[self.next_launch] == 0:
                self._launch(self.next_launch)
                self.next_launch += 1
            if self.next_launch != len(self.pending):
                raise RuntimeError(f"reducer: {len(self.pending) - self.next_launch} bucket(s) left unlaunched")
            for w in self.works:
                if w is not None:
                    w.wait()
            if self.record_order:
                self.record_order = False
                self.have_order = True
            self.iterations += 1
            self.armed = False
            self.next_launch = 0

    def ready_order(self):
        return list(self.order) if self.have_order else []


class GradReducer:
    """Bucket plan + reducer over a flat gradient arena.

    ``launch_order`` lists arena indices in the order gradients are expected to become ready; each
    bucket is a contiguous arena range in that order.
    """

    def __init__(
        self,
        arena: FlatArena,
        comm: Communicator,
        bucket_cap_mb: float = DEFAULT_BUCKET_CAP_MB,
        first_bucket_cap_mb: float = DEFAULT_FIRST_BUCKET_CAP_MB,
        find_unused_parameters: bool = False,
        average: bool = True,
        arena_in_ready_order: bool = False,
        timed_plan: bool = False,
    ):
        self.arena, self.comm = arena, comm
        self.cap, self.first_cap = bucket_cap_mb, first_bucket_cap_mb
        self.find_unused, self.average = find_unused_parameters, average
        self.arena_in_ready_order = arena_in_ready_order
        self._impl = None
        self._stream = None
        self._groups_override = None  # bucket plan chosen at the ready-order rebuild (timed planner)
        self.plan_info = {"planner": "cap"}
        self._timing = None
        self._build()
        if timed_plan:
            self.start_ready_timing()

    # ------------------------------------------------------------------ plan
    def _build(self):
        a = self.arena
        n = len(a.params)
        launch = list(range(n)) if self.arena_in_ready_order else list(range(n - 1, -1, -1))
        nbytes = [a.numels[i] * a.data.element_size() for i in launch]
        groups = self._groups_override or plan_buckets(nbytes, self.cap, self.first_cap)
        starts = [launch[0] if self.arena_in_ready_order else n]
        views = []
        self.bucket_ranges: List[Tuple[int, int]] = []
        for g in groups:
            idx = [launch[j] for j in g]
            lo, hi = min(idx), max(idx)
            s = a.offsets[lo]
            e = a.offsets[hi] + _aligned(a.numels[hi])
            self.bucket_ranges.append((s, e))
            views.append(a.grad[s:e])
            starts.append(hi + 1 if self.arena_in_ready_order else lo)
        self.bucket_starts = starts
        grad_views = a.grad_views()
        if self._impl is not None and getattr(self, "_trace", False):
            self._old_log = self._old_log + [tuple(e) for e in self._impl.trace_log()]  # keep across rebuilds
        if self._impl is not None:
            if hasattr(self._impl, "join_post_broadcast"):
                # an early buffer broadcast still pending on the old reducer: ordered before anything
                # that follows, and still counted for the next forward
                self._impl.join_post_broadcast()
                self._carry_issued = getattr(self, "_carry_issued", 0) + int(self._impl.take_post_issued())
            # drop every reference to the old AccumulateGrad nodes first so that fresh ones are
            # created on the current stream (see rebind_if_stream_changed)
            self._impl.remove_hooks()
            self._impl = None
        self._stream = torch.cuda.current_stream(a.device) if a.device.type == "cuda" else None
        # CDP_PY_REDUCER=1: the Python twin of the C++ reducer (tests run both on the same cases)
        use_native = _native.available() and os.environ.get("CDP_PY_REDUCER", "0") != "1" and (
            isinstance(self.comm, RcclCommunicator) or isinstance(self.comm, TorchCommunicator)
        )
        if use_native:
            C = _native.lib()
            rccl = self.comm.native if isinstance(self.comm, RcclCommunicator) else None
            pg = None
            if rccl is None:
                pg = self.comm.group if self.comm.group is not None else tdist.group.WORLD
            self._impl = C.Reducer(list(a.params), grad_views, views, starts, rccl, pg, self.find_unused, self.average)
        else:
            self._impl = _PyReducer(list(a.params), grad_views, views, starts, self.comm, self.find_unused, self.average)
        if getattr(self, "_trace", False):
            self._impl.set_trace(True)
        if getattr(self, "_timing", None) is not None:
            self._impl.set_defer(True)
        if getattr(self, "_post_bcast", None) and hasattr(self._impl, "set_post_broadcast"):
            self._impl.set_post_broadcast(self._post_bcast)

    # early buffer broadcast (DistributedDataParallel.early_buffer_broadcast): kept across rebuilds
    def set_post_broadcast(self, tensors):
        """Broadcast ``tensors`` from rank 0 behind the last bucket at the end of every synced backward
        (native reducer on the RCCL communicator only)."""
        if not self.native or not isinstance(self.comm, RcclCommunicator):
            raise RuntimeError("the end-of-backward buffer broadcast needs the native reducer on the RCCL communicator")
        self._post_bcast = list(tensors)
        self._impl.set_post_broadcast(self._post_bcast)

    def join_post_broadcast(self) -> int:
        """The current stream waits for the pending end-of-backward broadcasts; returns their count."""
        return int(self._impl.join_post_broadcast()) if hasattr(self._impl, "join_post_broadcast") else 0

    def take_post_issued(self) -> int:
        """End-of-backward broadcasts issued since the last call."""
        n = getattr(self, "_carry_issued", 0)
        self._carry_issued = 0
        if hasattr(self._impl, "take_post_issued"):
            n += int(self._impl.take_post_issued())
        return n

    @property
    def native(self) -> bool:
        return not isinstance(self._impl, _PyReducer)

    @property
    def num_buckets(self) -> int:
        return self._impl.num_buckets

    @property
    def iterations(self) -> int:
        return self._impl.iterations

    def bucket_sizes_bytes(self) -> List[int]:
        es = self.arena.data.element_size()
        return [(e - s) * es for s, e in self.bucket_ranges]

    def plan_summary(self, names=None) -> dict:
        """The bucket plan in launch order (the order backward makes them ready and the comm stream
        runs them): per bucket its bytes, tensor count and first / last parameter (``names`` maps
        ``id(param)`` to a name; arena indices otherwise), plus the caps it was planned with."""
        a = self.arena
        es = a.data.element_size()
        n = len(a.params)
        rows = []
        for b, (s, e) in enumerate(self.bucket_ranges):
            lo, hi = sorted((self.bucket_starts[b], self.bucket_starts[b + 1]))
            idx = list(range(lo, hi))
            if not self.arena_in_ready_order:
                idx = idx[::-1]  # model-order arena: the bucket's launch order runs backwards
            label = (lambda i: names.get(id(a.params[i]), str(i))) if names else str
            rows.append({"bytes": (e - s) * es, "tensors": len(idx), "first": label(idx[0]) if idx else None,
                         "last": label(idx[-1]) if idx else None})
        out = {"count": len(rows), "ready_order_layout": bool(self.arena_in_ready_order), "params": n,
               "launch_order": rows}
        out.update(self.plan_info)
        if self.plan_info.get("planner") == "cap":
            out.update(cap_mb=self.cap, first_cap_mb=self.first_cap)
        return out

    def rebind_if_stream_changed(self) -> bool:
        """Re-create the autograd hooks when the caller switched streams (e.g. hipGraph capture).

        The reducer keeps each parameter's AccumulateGrad node alive across iterations; autograd runs
        that node on the stream it was created on. If forward/backward later run on another stream
        (graph capture uses its own), the gradient accumulation would be issued on the old stream --
        illegal inside a capture. Rebinding creates the nodes anew on the current stream.
        """
        if self.arena.device.type != "cuda":
            return False
        cur = torch.cuda.current_stream(self.arena.device)
        if self._stream is not None and cur == self._stream:
            return False
        self._build()
        return True

    def prepare_for_backward(self, outputs: Sequence[torch.Tensor]):
        if self._timing is not None:
            armed = self._timing[4]
            if (not armed[0] and self._timing[2] and _native.available()
                    and not torch.cuda.is_current_stream_capturing()):
                # the timed backward is eager: at small batches the host enqueues kernels slower than
                # the GPU runs them, so the events would time the host. A few ms of idle GPU first
                # lets the host enqueue the whole backward ahead; the events then time the GPU's
                # back-to-back execution (what a replayed hipGraph step sees). Once per reducer.
                C = _native.lib()
                C.gpu_sleep(self.CALIBRATION_SLEEP_US)
                n = len(self._timing[3])
                C.gpu_timestamp(self._timing[5], n)  # two back-to-back stamps: the cost of one
                C.gpu_timestamp(self._timing[5], n + 1)
            armed[0] = True
        self._impl.prepare_for_backward(list(outputs))

    CALIBRATION_SLEEP_US = 5000.0
    MAX_STAMP_COST_US = 8.0  # two back-to-back stamps: 1.6-2.1 us on MI355X when dispatches are not held
    stamp_cost_us = None

    def disarm(self):
        self._impl.disarm()

    def can_step_buckets(self) -> bool:
        """Per-bucket optimizer steps need the native reducer on the RCCL communicator (collectives
        on a stream the step stream can wait on) and buckets that are arena ranges in launch order."""
        return self.native and isinstance(self.comm, RcclCommunicator) and bool(self.arena_in_ready_order)

    def set_bucket_steps(self, steps):
        """Register this backward's per-bucket SGD launches (``SGD.bucket_steps``); None clears."""
        if not self.native:  # the Python twin runs no bucket steps (can_step_buckets is False)
            if steps:
                raise RuntimeError("per-bucket optimizer steps need the native reducer")
            return
        self._impl.clear_bucket_steps()
        for b, kw in enumerate(steps or []):
            self._impl.set_bucket_step(b, **kw)

    def stepped_buckets(self) -> int:
        return int(self._impl.stepped_buckets) if self.native else 0

    def set_trace(self, on: bool = True):
        """Record ('h', param) at every gradient-ready hook, ('l', bucket) at every bucket
        launch and ('f', -1) at the end-of-backward callback (see :meth:`trace_log`)."""
        self._trace = bool(on)
        self._old_log = []
        self._impl.set_trace(bool(on))

    def trace_log(self) -> List[Tuple[str, int, int]]:
        return list(getattr(self, "_old_log", [])) + [tuple(e) for e in self._impl.trace_log()]

    def ready_order(self) -> List[int]:
        return list(self._impl.ready_order())

    # ------------------------------------------------------------------ timed bucket plan
    def start_ready_timing(self):
        """Record when each gradient becomes ready (GPU events on the compute stream, host clock on
        the CPU) until the ready-order rebuild, which plans the buckets from it."""
        self.stop_ready_timing()
        cuda = self.arena.device.type == "cuda" and _native.available()
        n = len(self.arena.params)
        stamps = {}  # param index -> host time (CPU) or timestamp slot (GPU)
        handles = []
        armed = [False]  # set by prepare_for_backward: only synchronised backwards are timed
        # GPU: one device int64 slot per parameter (+ 2 reference stamps) written by a one-thread
        # kernel reading the GPU wall clock; a timing event would end in a release barrier
        # (tens of us each on this stack) and stretch the very timeline it measures
        ts = torch.zeros(n + 2, dtype=torch.int64, device=self.arena.device) if cuda else None

        for i, p in enumerate(self.arena.params):
            def hook(_p, i=i):
                if not armed[0]:
                    return
                if cuda:
                    if torch.cuda.is_current_stream_capturing():
                        return  # a captured step records nothing
                    _native.lib().gpu_timestamp(ts, i)
                    stamps[i] = i
                else:
                    stamps[i] = time.perf_counter()
            handles.append(p.register_post_accumulate_grad_hook(hook))
        self._timing = (stamps, handles, cuda, list(self.arena.params), armed, ts)
        # the timed backward launches its buckets only at its end: its timeline is the compute's own
        # (a bucket all-reduce running beside it would stretch it), the plan then models the overlap
        if self._impl is not None:
            self._impl.set_defer(True)

    def stop_ready_timing(self):
        if self._timing is not None:
            for h in self._timing[1]:
                h.remove()
            if self._impl is not None:
                self._impl.set_defer(False)
        self._timing = None

    def _ready_times(self):
        """{param object id: seconds after the first recorded gradient} from the last timed backward."""
        if self._timing is None:
            return None
        stamps, _, cuda, params, _, ts = self._timing
        n = len(params)
        if len(stamps) != n:
            return None
        if cuda:
            torch.cuda.synchronize(self.arena.device)
            raw = ts.cpu().tolist()
            hz = _native.lib().gpu_wall_clock_khz() * 1e3
            # every stamp is one more dispatch on the stream: subtract the cost of the stamps that
            # precede each one (the back-to-back reference pair written before backward)
            # (capped at 4 us: two back-to-back one-thread kernels measured 1.8-2.1 us on MI355X)
            per_raw = max(0, raw[n + 1] - raw[n])
            self.stamp_cost_us = per_raw / hz * 1e6
            if self.stamp_cost_us > self.MAX_STAMP_COST_US:
                # the compute stream did not run its dispatches back to back during the timed
                # backward (each one waited tens of us): its timeline is not the step's, so no plan
                # is designed from it (the caller keeps the fixed-cap plan)
                return None
            per = min(per_raw, int(4e-6 * hz))
            order = sorted(range(n), key=lambda i: raw[i])
            t = {i: (raw[i] - k * per) / hz for k, i in enumerate(order)}
        else:
            t = dict(stamps)
        t0 = min(t.values())
        return {id(params[i]): v - t0 for i, v in t.items()}

    def _measure_comm(self, sizes_mb=(0.25, 2.0, 8.0), reps=3):
        """Fit alpha + beta * S to all-reduces of this communicator (every rank runs the same ones)."""
        cuda = self.arena.device.type == "cuda"
        # GPU: timed on the GPU wall clock between two stamps on the compute stream around the
        # (synchronous) collective, after a short GPU sleep so the host is ahead -- the host's
        # launch-and-synchronize round trip (~100 us) is not part of what overlaps the backward
        stamped = cuda and _native.available() and self._stream_ordered_comm()
        if stamped:
            C = _native.lib()
            hz = C.gpu_wall_clock_khz() * 1e3
            stamp = torch.zeros(2, dtype=torch.int64, device=self.arena.device)
        xs, ts = [], []
        for mb in sizes_mb:
            n = max(4, int(mb * 1024 * 1024) // 4)
            buf = torch.zeros(n, device=self.arena.device, dtype=torch.float32)
            samples = []
            for r in range(reps + 1):
                if cuda:
                    torch.cuda.synchronize(self.arena.device)
                if stamped:
                    C.gpu_sleep(300.0)
                    C.gpu_timestamp(stamp, 0)
                t0 = time.perf_counter()
                self.comm.all_reduce(buf, "sum")
                if stamped:
                    C.gpu_timestamp(stamp, 1)
                if cuda:
                    torch.cuda.synchronize(self.arena.device)
                if r:
                    if stamped:
                        a, b = stamp.tolist()
                        samples.append(max(0, b - a) / hz)
                    else:
                        samples.append(time.perf_counter() - t0)
            samples.sort()
            xs.append(n * 4)
            ts.append(samples[len(samples) // 2])
            del buf
        return fit_comm_model(xs, ts)

    def _stream_ordered_comm(self) -> bool:
        """Collectives enqueued on GPU streams (RCCL), which GPU stamps around them can time; gloo
        runs them on the host."""
        if isinstance(self.comm, RcclCommunicator):
            return True
        if isinstance(self.comm, TorchCommunicator):
            try:
                return tdist.get_backend(self.comm.group) == "nccl"
            except Exception:  # pragma: no cover - no default group
                return False
        return False

    def rebuild_in_ready_order(self, order: Optional[Sequence[int]] = None) -> bool:
        """Relayout the arena in gradient-ready order (rank 0's order, broadcast) and re-bucket.

        With ready times from the first iteration (``timed_plan``), rank 0 also designs the bucket
        plan (buckets.plan_buckets_timed over its measured timeline and this communicator's fitted
        alpha / beta) and broadcasts it with the order, so every rank buckets identically."""
        if order is None:
            order = self.ready_order()
        n = len(self.arena.params)
        order = list(order)
        # parameters that never fired (unused) go last, in reverse model order
        seen = set(order)
        order += [i for i in range(n - 1, -1, -1) if i not in seen]
        timed = self._timing is not None
        sizes = [0] * n
        info = {}
        if timed:
            rt = self._ready_times()
            alpha, beta = self._measure_comm()  # collective on every rank (same calls everywhere)
            if rt is None and self.comm.rank == 0:
                info = {"fallback": "timeline not measured" if self.stamp_cost_us is None else
                        f"timeline distorted (back-to-back dispatch {self.stamp_cost_us:.0f} us)"}
            if rt is not None and self.comm.rank == 0:
                ps = self.arena.params
                nbytes = [self.arena.numels[i] * self.arena.data.element_size() for i in order]
                ready = [rt[id(ps[i])] for i in order]
                groups, info = plan_buckets_timed(nbytes, ready, alpha, beta)
                for k, g in enumerate(groups):
                    sizes[k] = len(g)
        t = torch.tensor(order + [1 if timed else 0] + sizes, dtype=torch.int64)
        if self.comm.size > 1:
            t = t.to(self.arena.device)
            self.comm.broadcast(t, 0)
            t = t.cpu()
        vals = t.tolist()
        order, sizes = vals[:n], [k for k in vals[n + 1:] if k > 0]
        self.stop_ready_timing()
        changed = not (order == list(range(n)) and self.arena_in_ready_order)
        if timed and not (sizes and sum(sizes) == n) and info:
            self.plan_info = dict({"planner": "cap"}, **info)  # rank 0's reason (other ranks: cap)
        if sizes and sum(sizes) == n:
            groups, pos = [], 0
            for k in sizes:
                groups.append(list(range(pos, pos + k)))
                pos += k
            self._groups_override = groups
            self.plan_info = dict({"planner": "timed"}, **info) if info else {"planner": "timed"}
            changed = True
        if not changed:
            return False
        self.arena.relayout(order)
        self.arena_in_ready_order = True
        self._build()
        return True

    def remove(self):
        self.stop_ready_timing()
        if self._impl is not None:
            self._impl.remove_hooks()
            self._impl = None
