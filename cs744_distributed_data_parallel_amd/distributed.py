"""``torch.distributed``-shaped API over the native RCCL communicator.

Mirrors the subset of ``torch.distributed`` the reference scripts call
(``/root/reference/src/Part 2a/main.py:8,121-127,148-152``; ``Part 2b/main.py:118-119``):
``init_process_group`` (env:// rendezvous: ``MASTER_ADDR``/``MASTER_PORT``), ``get_world_size``,
``get_rank``, ``all_reduce``, ``gather``, ``scatter``, ``broadcast``, ``all_gather``, ``barrier``,
``ReduceOp`` and the deprecated ``reduce_op`` alias, so ``import cs744_distributed_data_parallel_amd.distributed
as dist`` is a drop-in for the reference's ``import torch.distributed as dist``.

Backends:
  * ``"rccl"`` (default on GPU) / ``"nccl"``: a torch ``nccl`` (=RCCL) process group for
    bootstrap/object collectives plus the native :class:`~.parallel.comm.RcclCommunicator`, which
    carries every tensor collective issued through this module (own stream, watchdog timeout);
  * ``"gloo"``: CPU tensors (the reference's backend, ``src/Part 2a/main.py:148``).
"""
from __future__ import annotations

import datetime
import os
import warnings
from typing import List, Optional

import torch
import torch.distributed as tdist

from . import _native
from .parallel.comm import Communicator, RcclCommunicator, TorchCommunicator, Work, _norm_op

__all__ = [
    "ReduceOp", "reduce_op", "init_process_group", "destroy_process_group", "is_initialized", "get_rank",
    "get_world_size", "get_local_rank", "get_backend", "all_reduce", "broadcast", "gather", "scatter", "all_gather",
    "all_gather_into_tensor", "reduce_scatter_tensor", "reduce", "barrier", "communicator_for", "device",
    "set_timeout", "healthy", "ranks_seen", "comm_fallback_reason", "collective_counts",
]


class ReduceOp:
    SUM = "sum"
    AVG = "avg"
    PRODUCT = "prod"
    MIN = "min"
    MAX = "max"


class _DeprecatedReduceOp:
    """``dist.reduce_op`` as used by the reference (``src/Part 2b/main.py:118``)."""

    def __getattr__(self, name):
        warnings.warn(
            "reduce_op is deprecated, please use ReduceOp instead", FutureWarning, stacklevel=2
        )
        return getattr(ReduceOp, name)


reduce_op = _DeprecatedReduceOp()


class _State:
    backend: Optional[str] = None
    rccl: Optional[RcclCommunicator] = None
    host: Optional[TorchCommunicator] = None
    device: Optional[torch.device] = None
    local_rank: int = 0
    fallback_reason: Optional[str] = None  # why the native communicator is not in use (CDP_RCCL_FALLBACK)


_S = _State()


def _local_rank(rank: int) -> int:
    if "LOCAL_RANK" in os.environ:
        return int(os.environ["LOCAL_RANK"])
    n = torch.cuda.device_count() or 1
    return rank % n


_init_generation = 0


def _init_native_rccl(rank, world_size, local, store, timeout_s) -> Optional[RcclCommunicator]:
    """Start the native communicator; every rank makes the SAME choice.

    Each rank posts ok/fail to the TCP store and reads every peer's flag before deciding, so a
    failure on one rank can never leave the others on a different communicator (which would hang or
    mismatch the next collective). Any failure is fatal on every rank unless
    ``CDP_RCCL_FALLBACK=1``, in which case all ranks agree to use the torch nccl (=RCCL) group.
    """
    global _init_generation
    _init_generation += 1
    gen = _init_generation
    comm, err = None, ""
    try:
        comm = RcclCommunicator(rank, world_size, local, store, timeout_s, tag=f"g{gen}")
    except RuntimeError as e:  # e.g. an RCCL build without this topology
        err = str(e) or "RuntimeError"
    store.set(f"cdp_rccl_ok/g{gen}/{rank}", "0" if comm is None else "1")
    keys = [f"cdp_rccl_ok/g{gen}/{r}" for r in range(world_size)]
    store.wait(keys, datetime.timedelta(seconds=max(60.0, timeout_s)))
    failed = [r for r, k in enumerate(keys) if store.get(k) != b"1"]
    if not failed:
        return comm
    if comm is not None:
        comm.shutdown()
    msg = f"native RCCL communicator failed on rank(s) {failed}" + (f" (here: {err})" if err else "")
    if os.environ.get("CDP_RCCL_FALLBACK", "0") != "1":
        raise RuntimeError(msg + "; set CDP_RCCL_FALLBACK=1 to run every rank on the torch nccl process group")
    warnings.warn(msg + "; all ranks use the torch nccl process group")
    _S.fallback_reason = msg
    return None


def init_process_group(
    backend: Optional[str] = None,
    init_method: Optional[str] = None,
    rank: int = -1,
    world_size: int = -1,
    timeout: Optional[datetime.timedelta] = None,
    device_id: Optional[int] = None,
    comm_timeout_s: Optional[float] = None,
):
    """Initialise the default group (env:// by default, like the reference)."""
    if backend is None:
        backend = "rccl" if torch.cuda.is_available() else "gloo"
    backend = backend.lower()
    if rank < 0:
        rank = int(os.environ.get("RANK", "0"))
    if world_size < 0:
        world_size = int(os.environ.get("WORLD_SIZE", "1"))
    timeout = timeout or datetime.timedelta(minutes=30)
    _S.fallback_reason = None
    if backend in ("rccl", "nccl"):
        local = _local_rank(rank) if device_id is None else int(device_id)
        torch.cuda.set_device(local)
        _S.device = torch.device("cuda", local)
        _S.local_rank = local
        tdist.init_process_group("nccl", init_method=init_method, rank=rank, world_size=world_size, timeout=timeout)
        if backend == "rccl" and _native.available():
            store = tdist.distributed_c10d._get_default_store()
            t = comm_timeout_s if comm_timeout_s is not None else timeout.total_seconds()
            _S.rccl = _init_native_rccl(rank, world_size, local, store, t)
        elif backend == "rccl":
            _S.fallback_reason = "native extension not importable: " + (_native.import_error() or "unknown")
    elif backend == "gloo":
        tdist.init_process_group("gloo", init_method=init_method, rank=rank, world_size=world_size, timeout=timeout)
        _S.device = torch.device("cpu")
    else:
        raise ValueError(f"unknown backend {backend!r} (rccl | nccl | gloo)")
    _S.backend = backend
    _S.host = TorchCommunicator()
    return _S.host


def destroy_process_group():
    if _S.rccl is not None:
        _S.rccl.shutdown()
        _S.rccl = None
    if tdist.is_initialized():
        tdist.destroy_process_group()
    _S.backend = None
    _S.host = None


def is_initialized() -> bool:
    return tdist.is_initialized()


def get_rank() -> int:
    return tdist.get_rank() if tdist.is_initialized() else 0


def get_world_size() -> int:
    return tdist.get_world_size() if tdist.is_initialized() else 1


def get_local_rank() -> int:
    return _S.local_rank


def get_backend() -> Optional[str]:
    return _S.backend


def device() -> torch.device:
    return _S.device or torch.device("cpu")


def communicator_for(t: Optional[torch.Tensor] = None) -> Communicator:
    """Native RCCL for GPU tensors (when the rccl backend is up), else the torch process group."""
    if t is not None and t.is_cuda and _S.rccl is not None:
        return _S.rccl
    if t is None and _S.rccl is not None:
        return _S.rccl
    if _S.host is None:
        if not tdist.is_initialized():
            raise RuntimeError("Default process group has not been initialized, call init_process_group")
        _S.host = TorchCommunicator()
    return _S.host


def native_communicator() -> Optional[RcclCommunicator]:
    return _S.rccl


def comm_fallback_reason() -> Optional[str]:
    """Why tensor collectives run on torch's nccl group instead of the native communicator (None when
    the native communicator is up, or when a non-rccl backend was asked for)."""
    return _S.fallback_reason


def collective_counts() -> Optional[dict]:
    """{"captured": n, "eager": n}: native-communicator collectives enqueued inside / outside a
    hipGraph capture so far (None without the native communicator)."""
    if _S.rccl is None:
        return None
    return {"captured": int(_S.rccl.native.captured_collectives()), "eager": int(_S.rccl.native.eager_collectives())}


def ranks_seen() -> int:
    """How many ranks the data-path communicator actually formed: ``ncclCommCount`` on the native
    RCCL communicator, else a SUM all-reduce of ones over the process group (gloo / torch nccl)."""
    if not tdist.is_initialized():
        return 1
    if _S.rccl is not None:
        return _S.rccl.count()
    dev = _S.device if (_S.device is not None and _S.device.type == "cuda") else torch.device("cpu")
    t = torch.ones(1, dtype=torch.int64, device=dev)
    tdist.all_reduce(t)
    return int(t.item())


def set_timeout(seconds: float):
    if _S.rccl is not None:
        _S.rccl.set_timeout(seconds)


def healthy() -> bool:
    return _S.rccl.healthy() if _S.rccl is not None else True


# ---------------------------------------------------------------------- collectives
def all_reduce(tensor, op=ReduceOp.SUM, group=None, async_op=False):
    return communicator_for(tensor).all_reduce(tensor, _norm_op(op), async_op=async_op)


def reduce(tensor, dst=0, op=ReduceOp.SUM, group=None, async_op=False):
    return communicator_for(tensor).reduce(tensor, dst, _norm_op(op), async_op=async_op)


def broadcast(tensor, src=0, group=None, async_op=False):
    return communicator_for(tensor).broadcast(tensor, src, async_op=async_op)


def gather(tensor, gather_list: Optional[List[torch.Tensor]] = None, dst: int = 0, group=None, async_op=False):
    communicator_for(tensor).gather(tensor, gather_list, dst)


def scatter(tensor, scatter_list: Optional[List[torch.Tensor]] = None, src: int = 0, group=None, async_op=False):
    communicator_for(tensor).scatter(tensor, scatter_list, src)


def all_gather(tensor_list: List[torch.Tensor], tensor, group=None, async_op=False):
    inp = tensor.contiguous().reshape(-1)
    out = torch.empty(len(tensor_list) * inp.numel(), dtype=tensor.dtype, device=tensor.device)
    communicator_for(tensor).all_gather(out, inp)
    for i, t in enumerate(tensor_list):
        t.copy_(out[i * inp.numel() : (i + 1) * inp.numel()].view_as(t))


def all_gather_into_tensor(output, tensor, group=None, async_op=False):
    return communicator_for(tensor).all_gather(output, tensor, async_op=async_op)


def reduce_scatter_tensor(output, tensor, op=ReduceOp.SUM, group=None, async_op=False):
    return communicator_for(tensor).reduce_scatter(output, tensor, _norm_op(op), async_op=async_op)


def barrier(group=None):
    if _S.rccl is not None:
        _S.rccl.barrier()
    else:
        communicator_for(None).barrier()


Work = Work
