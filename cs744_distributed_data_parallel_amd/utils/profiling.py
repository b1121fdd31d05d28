"""Tracing: roctx ranges (visible in rocprofv3 ``--marker-trace`` timelines) and a per-rank chrome
trace of training phases.

The reference only prints host wall-clock deltas. Here every training phase
(forward, backward+sync, step, bucket all-reduce) can be bracketed by a roctx range, and
:class:`TraceRecorder` writes a ``chrome://tracing`` JSON of GPU-event-timed phases per rank.
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import time
from typing import List, Optional

import torch

_roctx = None


def _lib():
    global _roctx
    if _roctx is None:
        for name in ("librocprofiler-sdk-roctx.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so", "libroctx64.so",
                     "/opt/rocm/lib/libroctx64.so"):
            try:
                _roctx = ctypes.CDLL(name)
                _roctx.roctxRangePushA.argtypes = [ctypes.c_char_p]
                _roctx.roctxMarkA.argtypes = [ctypes.c_char_p]
                break
            except OSError:
                continue
        if _roctx is None:
            _roctx = False
    return _roctx or None


def enabled() -> bool:
    return os.environ.get("CDP_ROCTX", "0") == "1"


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors nvtx/roctx naming
    lib = _lib() if enabled() else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(name: str):
    lib = _lib() if enabled() else None
    if lib is not None:
        lib.roctxMarkA(name.encode())


class TraceRecorder:
    """Chrome-trace JSON of training phases (GPU-event timed, resolved at ``dump``) plus the
    reducer's host-side events (gradient-ready hooks, bucket launches, end of backward).

    Track ``tid 0`` holds the phases (forward / backward / sync / step), placed on the host clock
    at the moment their first event was recorded; ``tid 1`` holds instant events from
    :meth:`GradReducer.trace_log <..parallel.reducer.GradReducer.trace_log>` (CLOCK_MONOTONIC, the
    same clock), so bucket launches can be read against backward.
    """

    def __init__(self, rank: int = 0, device: Optional[torch.device] = None):
        self.rank = rank
        self.gpu = device is not None and device.type == "cuda"
        self._events: List[tuple] = []
        self._host: List[tuple] = []
        self._t0 = None
        self._t0_ns = None

    def _ev(self):
        if self.gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    @contextlib.contextmanager
    def phase(self, name: str):
        a = self._ev()
        if self._t0 is None:
            self._t0 = a
            self._t0_ns = time.monotonic_ns()
        with range(name):
            yield
        self._events.append((name, a, self._ev()))

    def add_reducer_log(self, log, label: str = "reducer"):
        """Append ``(kind, index, monotonic_ns)`` records (``'h'`` hook, ``'l'`` launch, ``'f'`` finalize)."""
        names = {"h": "grad_ready[{}]", "l": "bucket_allreduce_launch[{}]", "f": "backward_done"}
        for kind, idx, t_ns in log:
            self._host.append((names.get(kind, kind + "[{}]").format(idx), int(t_ns), label))

    def dump(self, path: str):
        if self.gpu and self._events:
            self._events[-1][2].synchronize()
        base = self._t0_ns
        if base is None and self._host:
            base = min(t for _, t, _ in self._host)
        out = []
        for name, a, b in self._events:
            if self.gpu:
                ts = self._t0.elapsed_time(a) * 1e3
                dur = a.elapsed_time(b) * 1e3
            else:
                ts = (a - self._t0) * 1e6
                dur = (b - a) * 1e6
            out.append({"name": name, "ph": "X", "ts": ts, "dur": dur, "pid": self.rank, "tid": 0})
        for name, t_ns, label in self._host:
            out.append({"name": name, "ph": "i", "s": "t", "ts": (t_ns - base) / 1e3, "pid": self.rank, "tid": 1,
                        "args": {"src": label}})
        meta = [{"name": "thread_name", "ph": "M", "pid": self.rank, "tid": 0, "args": {"name": "phases"}},
                {"name": "thread_name", "ph": "M", "pid": self.rank, "tid": 1, "args": {"name": "reducer (host)"}}]
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as fh:
            json.dump({"traceEvents": meta + out}, fh)
        return path
