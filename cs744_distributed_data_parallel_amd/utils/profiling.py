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
        for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
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
    """Chrome-trace JSON of phases timed by GPU events (resolved at ``dump``)."""

    def __init__(self, rank: int = 0, device: Optional[torch.device] = None):
        self.rank = rank
        self.gpu = device is not None and device.type == "cuda"
        self._events: List[tuple] = []
        self._t0 = None

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
        with range(name):
            yield
        self._events.append((name, a, self._ev()))

    def dump(self, path: str):
        if self.gpu and self._events:
            self._events[-1][2].synchronize()
        out = []
        for name, a, b in self._events:
            if self.gpu:
                ts = self._t0.elapsed_time(a) * 1e3
                dur = a.elapsed_time(b) * 1e3
            else:
                ts = (a - self._t0) * 1e6
                dur = (b - a) * 1e6
            out.append({"name": name, "ph": "X", "ts": ts, "dur": dur, "pid": self.rank, "tid": 0})
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as fh:
            json.dump({"traceEvents": out}, fh)
        return path
