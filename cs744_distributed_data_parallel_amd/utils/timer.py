"""Phase timers with the reference's log semantics, measured correctly on the GPU.

The reference times phases with host ``time.time()`` (``/root/reference/src/Part 1/main.py:33-43``):
"Forward" = zero_grad + forward, "Backward" = loss + backward + sync + step, averaged over windows
of 20 iterations with the first window discarded. On a GPU those host deltas only measure launch
time, so :class:`PhaseTimer` records HIP events on the current stream at phase boundaries and
resolves them lazily (one host sync per report window, never per iteration).
"""
from __future__ import annotations

import time
from collections import defaultdict
from typing import Dict, List, Optional

import torch


class PhaseTimer:
    def __init__(self, device: Optional[torch.device] = None, enabled: bool = True):
        self.gpu = device is not None and device.type == "cuda" and torch.cuda.is_available()
        self.enabled = enabled
        self._marks: List[tuple] = []  # (name, event_or_time)
        self.totals: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)

    def _now(self):
        if self.gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def mark(self, name: str):
        """Boundary: the phase ``name`` ends here (the previous mark starts it)."""
        if self.enabled:
            self._marks.append((name, self._now()))

    def resolve(self):
        """Fold recorded marks into totals (syncs the GPU once)."""
        if not self._marks:
            return
        if self.gpu:
            self._marks[-1][1].synchronize()
        prev = None
        for name, t in self._marks:
            if prev is not None and name != "start":
                dt = prev.elapsed_time(t) / 1e3 if self.gpu else (t - prev)
                self.totals[name] += dt
                self.counts[name] += 1
            prev = t
        self._marks = []

    def pop(self, name: str) -> float:
        self.resolve()
        v = self.totals.pop(name, 0.0)
        self.counts.pop(name, None)
        return v

    def reset(self):
        self._marks = []
        self.totals.clear()
        self.counts.clear()


class Stopwatch:
    """Wall-clock region timer that synchronises the device at both ends."""

    def __init__(self, device: Optional[torch.device] = None):
        self.cuda = device is not None and device.type == "cuda"

    def __enter__(self):
        if self.cuda:
            torch.cuda.synchronize()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *a):
        if self.cuda:
            torch.cuda.synchronize()
        self.elapsed = time.perf_counter() - self.t0
