"""Loader for the native runtime (``_C``: gfx950 kernels, RCCL communicator, bucketed reducer).

The extension is built in-tree by :mod:`._build` (``python -m cs744_distributed_data_parallel_amd._build``
or ``__graft_entry__.build()``). GPU code paths never fall back silently: if a GPU tensor reaches
an op and the extension is missing, :func:`require` raises with the build instructions. CPU tensors
use the PyTorch reference math (that is what the CPU test-suite exercises).
"""
from __future__ import annotations

import importlib
import os

_C = None
_err: Exception | None = None


def _load():
    global _C, _err
    if _C is not None or _err is not None:
        return _C
    try:
        import torch  # noqa: F401  (libtorch must be loaded first)

        _C = importlib.import_module(__package__ + "._C")
    except Exception as e:  # pragma: no cover - depends on the build
        _err = e
        _C = None
    return _C


def available() -> bool:
    return _load() is not None


def lib():
    """Return the extension module, raising a descriptive error if it is unavailable."""
    m = _load()
    if m is None:
        raise RuntimeError(
            "cs744_distributed_data_parallel_amd native runtime (_C) is not available: "
            f"{_err!r}. Build it with `python -m cs744_distributed_data_parallel_amd._build` "
            "(hipcc, --offload-arch=gfx950)."
        )
    return m


def require(*tensors) -> bool:
    """True if any tensor lives on the GPU (=> the native kernels must be used; raises if missing)."""
    on_gpu = any(t is not None and getattr(t, "is_cuda", False) for t in tensors)
    if on_gpu:
        lib()
    return on_gpu


def import_error() -> str | None:
    _load()
    return None if _err is None else repr(_err)


def so_path() -> str | None:
    m = _load()
    return getattr(m, "__file__", None) if m is not None else None


def force_reference() -> bool:
    """CDP_FORCE_REFERENCE=1 routes GPU tensors through torch ops (for A/B timing only)."""
    return os.environ.get("CDP_FORCE_REFERENCE", "0") == "1"
