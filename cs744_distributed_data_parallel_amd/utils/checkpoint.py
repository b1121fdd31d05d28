"""Checkpoint / resume in the standard PyTorch layout.

The reference never saves; the implied compatible layout is PyTorch's own:
model ``state_dict`` (58 keys for VGG-11: ``layers.{i}.weight|bias|running_mean|running_var|
num_batches_tracked``, ``fc1.weight|bias``; ``module.``-prefixed under DDP) and the SGD
``state_dict`` (``param_groups`` + per-parameter ``momentum_buffer``). Files written here load with
``torch.load(..., weights_only=True)`` into a plain ``torch.nn`` model / ``torch.optim.SGD`` and
vice versa; tensors are saved contiguous (NCHW) even though the runtime keeps them channels_last in
flat arenas. Writes are atomic (tmp file + rename) and only rank 0 writes.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

import torch


def _plain(sd):
    out = {}
    for k, v in sd.items():
        if isinstance(v, torch.Tensor):
            out[k] = v.detach().to("cpu").contiguous().clone()
        elif isinstance(v, dict):
            out[k] = _plain(v)
        elif isinstance(v, list):
            out[k] = [_plain(x) if isinstance(x, dict) else x for x in v]
        else:
            out[k] = v
    return out


def unwrap(model):
    return getattr(model, "module", model)


def model_state_dict(model, strip_ddp_prefix: bool = False) -> Dict[str, torch.Tensor]:
    m = unwrap(model) if strip_ddp_prefix else model
    return _plain(m.state_dict())


def save_checkpoint(path: str, model, optimizer=None, epoch: int = 0, iteration: int = 0,
                    extra: Optional[Dict[str, Any]] = None, rank: int = 0) -> Optional[str]:
    if rank != 0:
        return None
    state = {
        "model": _plain(model.state_dict()),
        "epoch": int(epoch),
        "iteration": int(iteration),
        "rng_cpu": torch.get_rng_state(),
    }
    if optimizer is not None:
        state["optimizer"] = _plain(optimizer.state_dict())
    if extra:
        state["extra"] = extra
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)
    return path


def load_checkpoint(path: str, model=None, optimizer=None, map_location="cpu", strict: bool = True) -> Dict[str, Any]:
    """Load with ``weights_only=True`` (nothing in the file is executed).

    Accepts checkpoints saved from a DDP-wrapped or a bare model (``module.`` prefixes are matched
    to whatever ``model`` expects).
    """
    state = torch.load(path, map_location=map_location, weights_only=True)
    if model is not None:
        sd = state["model"]
        target_keys = list(model.state_dict().keys())
        wants_prefix = bool(target_keys) and target_keys[0].startswith("module.")
        has_prefix = bool(sd) and next(iter(sd)).startswith("module.")
        if has_prefix and not wants_prefix:
            sd = {k[len("module."):]: v for k, v in sd.items()}
        elif wants_prefix and not has_prefix:
            sd = {"module." + k: v for k, v in sd.items()}
        with torch.no_grad():
            model.load_state_dict(sd, strict=strict)
    if optimizer is not None and "optimizer" in state:
        optimizer.load_state_dict(state["optimizer"])
    return state


def latest_checkpoint(directory: str, prefix: str = "ckpt_") -> Optional[str]:
    if not os.path.isdir(directory):
        return None
    c = [f for f in os.listdir(directory) if f.startswith(prefix) and f.endswith(".pt")]
    if not c:
        return None
    c.sort(key=lambda f: int("".join(ch for ch in f[len(prefix):-3] if ch.isdigit()) or 0))
    return os.path.join(directory, c[-1])
