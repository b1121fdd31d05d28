"""Flat parameter / gradient / momentum arenas.

MI355X-first memory layout: all parameters of a model live in ONE contiguous fp32
allocation, every ``p.grad`` is a view into ONE gradient allocation and the optimizer's momentum
buffers into a third. Consequences:

* a gradient bucket is a contiguous arena range -> the RCCL all-reduce runs in place, zero copies
  (PyTorch DDP calls this ``gradient_as_bucket_view``);
* the SGD step is one vectorised kernel over the whole arena instead of 34 (VGG-11) / 161
  (ResNet-50) per-tensor launches;
* the construction-time parameter broadcast and the per-forward buffer broadcast are single
  collectives;
* every view keeps its parameter's shape *and strides* (conv weights stay channels_last), so
  ``state_dict`` / ``load_state_dict`` / AccumulateGrad's layout contract are unaffected.

Offsets are padded to 16 bytes so every view is float4-aligned for the kernels.
"""
from __future__ import annotations

from typing import Iterable, List, Sequence

import torch

ALIGN = 4  # elements (16 B for fp32)


def weight_max_elems(co: int, ci: int) -> int:
    """Floats of a conv weight's f16x2 maxima (csrc/kernels/kernels.h ``weight_max_elems``): the per-co
    partials of every 32-wide ci block, then the per-ci partials of every 32-wide co block."""
    return ((ci + 31) // 32) * co + ((co + 31) // 32) * ci


def act_max_elems(n: int, c: int, copies: int = 8) -> int:
    """int32 slots of an activation's f16x2 act max (csrc ``act_max_elems``): one per image, then
    ``copies`` (kActCopies) x one per channel."""
    return n + copies * c


def refresh_prep_after_load(module, incompatible_keys=None):
    """``load_state_dict`` post-hook: the weights were written in place, which a replayed hipGraph step
    cannot notice (it reads the W^T / f16x2 maxima its previous replay's fused optimizer step wrote).
    Re-derive those products from the loaded weights now (FlatArena.prep_refresh), or drop them when
    no fused plan exists yet, so the next replay -- or eager forward -- uses the loaded weights."""
    seen = set()
    for p in module.parameters():
        a = getattr(p, "_cdp_arena", None)
        if a is None or id(a) in seen:
            continue
        seen.add(id(a))
        if not a.prep_refresh():
            a.prep_valid = None


def install_load_hooks(module) -> None:
    """Register :func:`refresh_prep_after_load` on ``module`` once (models and the DDP wrapper)."""
    if not getattr(module, "_cdp_load_hook", False):
        module.register_load_state_dict_post_hook(refresh_prep_after_load)
        module._cdp_load_hook = True


def _dense(t: torch.Tensor) -> bool:
    return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))


def _view_like(flat: torch.Tensor, offset: int, ref: torch.Tensor) -> torch.Tensor:
    return flat.as_strided(ref.size(), ref.stride(), flat.storage_offset() + offset)


class FlatArena:
    """Owns the flat storages for a fixed, ordered list of parameters."""

    def __init__(self, params: Sequence[torch.nn.Parameter], with_grad: bool = True):
        params = list(params)
        if not params:
            raise ValueError("FlatArena needs at least one parameter")
        dev, dt = params[0].device, params[0].dtype
        for p in params:
            if p.device != dev or p.dtype != dt:
                raise ValueError("all arena parameters must share device and dtype")
            if not _dense(p.data):
                p.data = p.data.contiguous()
        self.device, self.dtype = dev, dt
        self.params: List[torch.nn.Parameter] = params
        self._layout(params)
        self.data = torch.empty(self.total, device=dev, dtype=dt)
        self.data.zero_()
        for p, off in zip(params, self.offsets):
            v = _view_like(self.data, off, p.data)
            v.copy_(p.data)
            p.data = v
        self.grad = None
        self.momentum = None
        self.claimed = [False] * len(params)
        # next-step weight preparation by the optimizer (see prep_lookup / prep_plan_for)
        self.layout_gen = 0
        self.prep_request = None  # (weights, want_t) registered by a model's forward
        self._prep_plan = None  # (key, plan tensors) from _C.sgd_prep_plan
        self.prep_valid = None  # (key, weight versions) after a fused optimizer step
        if with_grad:
            self.attach_grads()
        for i, p in enumerate(params):
            p._cdp_arena = self
            p._cdp_index = i

    # ------------------------------------------------------------------ layout
    def _layout(self, params):
        self.offsets, self.numels = [], []
        off = 0
        for p in params:
            n = p.numel()
            self.offsets.append(off)
            self.numels.append(n)
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        self.total = max(off, ALIGN)

    def index(self, p) -> int:
        return p._cdp_index

    def attach_grads(self):
        """(Re)point every ``p.grad`` at its arena slot (keeping any existing values)."""
        if self.grad is None:
            self.grad = torch.zeros(self.total, device=self.device, dtype=self.dtype)
        for p, off in zip(self.params, self.offsets):
            v = _view_like(self.grad, off, p.data)
            if p.grad is not None and p.grad.data_ptr() != v.data_ptr():
                v.copy_(p.grad)
            p.grad = v
        return self.grad

    # ------------------------------------------------------------------ direct-write gradient slots
    def claim(self, p) -> torch.Tensor | None:
        """Arena slot for a kernel to write ``p``'s gradient into directly.

        Valid only while ``p.grad is None`` (after ``zero_grad(set_to_none=True)``): the returned view is
        handed to autograd as the gradient, and AccumulateGrad *steals* it (no copy, no add), so
        ``p.grad`` ends up as the arena view. Each slot is claimed at most once per iteration (a
        parameter used twice gets a fresh tensor for its second use and autograd sums them).
        """
        i = p._cdp_index
        if self.grad is None or p.grad is not None or self.claimed[i]:
            return None
        self.claimed[i] = True
        return _view_like(self.grad, self.offsets[i], p.data)

    def reset_claims(self):
        self.claimed = [False] * len(self.params)

    def ensure_grads_in_arena(self, params=None) -> bool:
        """Make every ``p.grad`` (of ``params``) its arena view, copying foreign tensors in."""
        ok = True
        for p in (params if params is not None else self.params):
            if p.grad is None:
                ok = False
                continue
            i = p._cdp_index
            v = _view_like(self.grad, self.offsets[i], p.data)
            if p.grad.data_ptr() != v.data_ptr():
                v.copy_(p.grad)
                p.grad = v
        return ok

    def grad_views(self) -> List[torch.Tensor]:
        return [_view_like(self.grad, off, p.data) for p, off in zip(self.params, self.offsets)]

    def param_views(self) -> List[torch.Tensor]:
        return [_view_like(self.data, off, p.data) for p, off in zip(self.params, self.offsets)]

    def momentum_buffer(self) -> torch.Tensor:
        if self.momentum is None:
            self.momentum = torch.zeros(self.total, device=self.device, dtype=self.dtype)
        return self.momentum

    def momentum_views(self) -> List[torch.Tensor]:
        buf = self.momentum_buffer()
        return [_view_like(buf, off, p.data) for p, off in zip(self.params, self.offsets)]

    def zero_grad(self):
        if self.grad is not None:
            self.grad.zero_()
            self.attach_grads()

    def range_of(self, first: int, last: int):
        """Flat [start, end) element range covering parameters first..last (inclusive, arena order)."""
        s = self.offsets[first]
        e = self.offsets[last] + (self.numels[last] + ALIGN - 1) // ALIGN * ALIGN
        return s, e

    def contiguous_range(self, params: Iterable[torch.nn.Parameter]):
        """If ``params`` cover a gap-free run of arena slots, return its flat [start, end); else None."""
        idx = sorted(p._cdp_index for p in params if getattr(p, "_cdp_arena", None) is self)
        if not idx:
            return None
        if idx != list(range(idx[0], idx[-1] + 1)):
            return None
        return self.range_of(idx[0], idx[-1])

    # ------------------------------------------------------------------ fused weight preparation
    # The forward of a model with f16x2 / data-gradient GEMMs needs, per conv weight, |max| partials
    # and W^T (ops.functional.weight_prep). The optimizer's step is the last writer of the weights, so
    # it can emit both in the same pass (csrc sgd_prep_kernel) instead of a separate launch re-reading
    # the 37 MB arena at the next forward. The forward registers what it needs (prep_request); the
    # optimizer plans once per layout (prep_plan_for) and marks the products valid for the weights'
    # versions at that step (prep_valid); the next forward takes them (prep_lookup) only if no weight
    # changed since (an in-place edit, load_state_dict or a step without the fused kernel all bump a
    # version or clear prep_valid) and otherwise prepares the weights itself.
    def _prep_key(self, weights, want):
        return (self.layout_gen, tuple(id(w) for w in weights), tuple(bool(f) for f in want))

    def prep_lookup(self, weights, want):
        """(amax partial views, W^T list) written by the last optimizer step, or None."""
        v = self.prep_valid
        if v is None or self._prep_plan is None:
            return None
        key, versions = v
        if key != self._prep_key(weights, want) or key != self._prep_plan[0]:
            return None
        if any(w._version != ver for w, ver in zip(weights, versions)):
            return None
        plan = self._prep_plan[1]
        return plan["amax_views"], plan["wts"]

    def prep_plan_for(self, start: int, end: int):
        """The fused-step plan for the flat range [start, end) if the registered request lies in it."""
        req = self.prep_request
        if req is None:
            return None
        weights, want = req
        key = self._prep_key(weights, want)
        if self._prep_plan is not None and self._prep_plan[0] == key:
            rng = self._prep_plan[2]
            if rng == (start, end):
                return self._prep_plan[1]
            if isinstance(rng[0], tuple) and rng[0][0] == start and rng[-1][1] == end:
                return self._prep_plan[1]  # a split plan tiling this range (its sub-plans run in turn)
        if any(getattr(w, "_cdp_arena", None) is not self for w in weights):
            return None
        offs = [self.offsets[w._cdp_index] for w in weights]
        if any(o < start or o + w.numel() > end for o, w in zip(offs, weights)):
            return None
        if any(w.dim() != 4 or not w.is_contiguous(memory_format=torch.channels_last) for w in weights):
            return None
        from .. import _native

        r = _native.lib().sgd_prep_plan(self.data, start, end, [w.data for w in weights], list(want))
        desc, meta, amax, wts = r[0], r[1], r[2], list(r[3:])
        # each weight's maxima: per-co partials [ceil(Ci/32), Co] then per-ci [ceil(Co/32), Ci]
        # (csrc weight_max_elems), back to back in plan order
        sizes = [weight_max_elems(w.shape[0], w.shape[1]) for w in weights]
        views, b0 = [], 0
        for n in sizes:
            views.append(amax.narrow(0, b0, n))
            b0 += n
        plan = {"desc": desc, "meta": meta, "amax": amax, "amax_views": views,
                "wts": [t if f else None for t, f in zip(wts, want)], "weights": list(weights)}
        self._prep_plan = (key, plan, (start, end))
        return plan

    def prep_plan_ranges(self, ranges):
        """The fused-step plan split over consecutive flat ranges (the buckets of an overlapped
        optimizer step, each stepped by its own launch): ONE maxima tensor and one W^T per weight in
        the request's order, as :meth:`prep_lookup` hands them to the forward, plus one sub-plan per
        range covering the weights inside it (None for a range with no prepared weight). None when
        a weight straddles two ranges or the request does not lie in them."""
        req = self.prep_request
        if req is None:
            return None
        ranges = tuple((int(s), int(e)) for s, e in ranges)
        weights, want = req
        key = self._prep_key(weights, want)
        if self._prep_plan is not None and self._prep_plan[0] == key and self._prep_plan[2] == ranges:
            return self._prep_plan[1]
        if any(getattr(w, "_cdp_arena", None) is not self for w in weights):
            return None
        if any(w.dim() != 4 or not w.is_contiguous(memory_format=torch.channels_last) for w in weights):
            return None
        offs = [self.offsets[w._cdp_index] for w in weights]
        where = []
        for o, w in zip(offs, weights):
            r = [k for k, (s, e) in enumerate(ranges) if s <= o and o + w.numel() <= e]
            if len(r) != 1:
                return None
            where.append(r[0])
        from .. import _native

        sizes = [weight_max_elems(w.shape[0], w.shape[1]) for w in weights]
        starts = [sum(sizes[:k]) for k in range(len(sizes))]
        amax = torch.empty(max(1, sum(sizes)), device=self.device, dtype=self.dtype)
        wts = [None] * len(weights)
        subs = []
        for k, (s, e) in enumerate(ranges):
            idx = [j for j, r in enumerate(where) if r == k]
            if not idx:
                subs.append(None)
                continue
            r = _native.lib().sgd_prep_plan(self.data, s, e, [weights[j].data for j in idx], [bool(want[j]) for j in idx],
                                            amax, [starts[j] for j in idx])
            subs.append({"desc": r[0], "meta": r[1]})
            for t, j in zip(r[3:], idx):
                wts[j] = t if want[j] else None
        views = [amax.narrow(0, st, n) for st, n in zip(starts, sizes)]
        plan = {"amax": amax, "amax_views": views, "wts": wts, "weights": list(weights), "subs": subs,
                "ranges": ranges}
        self._prep_plan = (key, plan, ranges)
        return plan

    def prep_refresh(self) -> bool:
        """Recompute the fused-step products from the current weights, in place (same buffers).

        A captured hipGraph step reads these buffers at its forward and rewrites them at its optimizer
        step, so the graph never re-checks the weights on the host: weights changed outside the graph
        between replays (copy_, load_state_dict, ...) must be followed by this call (SGD.refresh_weight_prep)
        before the next replay. Eager steps detect such edits themselves (prep_lookup)."""
        if self._prep_plan is None or self.prep_request is None:
            return False
        weights, want = self.prep_request
        plan = self._prep_plan[1]
        from .. import _native

        _native.lib().weight_prep_into([w.data for w in weights], list(want), plan["amax"], plan["wts"])
        self.prep_mark_valid()
        return True

    def prep_mark_valid(self):
        req = self.prep_request
        if req is None or self._prep_plan is None:
            self.prep_valid = None
            return
        weights, want = req
        self.prep_valid = (self._prep_key(weights, want), [w._version for w in weights])

    # ------------------------------------------------------------------ relayout
    def relayout(self, new_order: Sequence[int]):
        """Permute the arena into ``new_order`` (indices into the current parameter list).

        Used after the first iteration to lay gradients out in their observed ready order, so every
        bucket is a contiguous range. Parameter values, gradients and momentum move with their
        parameters; all views are re-pointed.
        """
        new_order = list(new_order)
        if sorted(new_order) != list(range(len(self.params))):
            raise ValueError("relayout order must be a permutation of the parameter indices")
        old_params, old_offsets = self.params, self.offsets
        old_data, old_grad, old_mom = self.data, self.grad, self.momentum
        params = [old_params[i] for i in new_order]
        self._layout(params)
        self.params = params
        self.data = torch.zeros(self.total, device=self.device, dtype=self.dtype)
        self.grad = None if old_grad is None else torch.zeros_like(self.data)
        self.momentum = None if old_mom is None else torch.zeros_like(self.data)
        for new_i, old_i in enumerate(new_order):
            p = params[new_i]
            o_off, n_off = old_offsets[old_i], self.offsets[new_i]
            v = _view_like(self.data, n_off, p.data)
            v.copy_(_view_like(old_data, o_off, p.data))
            p.data = v
            if old_grad is not None:
                _view_like(self.grad, n_off, p.data).copy_(_view_like(old_grad, o_off, p.data))
            if old_mom is not None:
                _view_like(self.momentum, n_off, p.data).copy_(_view_like(old_mom, o_off, p.data))
            p._cdp_index = new_i
        self.claimed = [False] * len(params)
        self.layout_gen += 1  # offsets moved: any fused-step plan / products are stale
        self._prep_plan = None
        self.prep_valid = None
        if old_grad is not None:
            for p, off in zip(self.params, self.offsets):
                if p.grad is not None:
                    p.grad = _view_like(self.grad, off, p.data)
        for cb in getattr(self, "_relayout_callbacks", []):
            cb(self)

    def on_relayout(self, cb):
        if not hasattr(self, "_relayout_callbacks"):
            self._relayout_callbacks = []
        self._relayout_callbacks.append(cb)


def arena_for(params: Sequence[torch.nn.Parameter], create: bool = True) -> FlatArena | None:
    """Return the arena shared by ``params`` (creating one over exactly these params if needed)."""
    params = [p for p in params if p.requires_grad]
    arenas = {id(getattr(p, "_cdp_arena", None)) for p in params}
    if len(arenas) == 1:
        a = getattr(params[0], "_cdp_arena", None)
        if a is not None:
            return a
    if not create:
        return None
    return FlatArena(params)


class BufferArena:
    """Flat arena for module buffers (BN running stats) so they broadcast as ONE collective.

    Every buffer, whatever its dtype (fp32 running stats, int64 ``num_batches_tracked``), is a
    typed view into one byte storage; DDP's per-forward buffer sync is then a single ``uint8``
    broadcast instead of one per dtype (each collective costs a launch-latency round at N>1).
    """

    def __init__(self, buffers: Sequence[torch.Tensor]):
        self.buffers = list(buffers)
        self.groups = {}
        by_dtype = {}
        for b in self.buffers:
            by_dtype.setdefault(b.dtype, []).append(b)
        layout, nbytes = [], 0
        for dt, bufs in by_dtype.items():
            es = torch.empty((), dtype=dt).element_size()
            nbytes = (nbytes + 15) // 16 * 16  # 16-B aligned groups
            total = sum(b.numel() for b in bufs)
            layout.append((dt, bufs, nbytes, total))
            nbytes += total * es
        self.bytes = torch.empty(max(nbytes, 1), device=self.buffers[0].device, dtype=torch.uint8)
        for dt, bufs, start, total in layout:
            es = torch.empty((), dtype=dt).element_size()
            flat = self.bytes[start : start + total * es].view(dt)
            off = 0
            for b in bufs:
                n = b.numel()
                v = flat[off : off + n].view(b.shape)
                v.copy_(b.data)
                b.data = v
                off += n
            self.groups[dt] = flat

    def flats(self) -> List[torch.Tensor]:
        """The storages to broadcast: one byte tensor covering every buffer."""
        return [self.bytes]
