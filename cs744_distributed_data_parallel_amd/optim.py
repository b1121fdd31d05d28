"""Fused SGD (momentum, dampening, weight decay, Nesterov, maximize) over flat arenas.

Drop-in for ``torch.optim.SGD`` as used by every reference stage
(``optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=0.0001)``,
``/root/reference/src/Part 1/main.py:114-115``): it *is* a ``torch.optim.Optimizer`` subclass, so
``param_groups``, ``state_dict()`` / ``load_state_dict()`` (``momentum_buffer`` per parameter) and
LR schedulers behave exactly like torch's.

MI355X path: parameters, gradients and momentum live in :class:`~.utils.arena.FlatArena` storages,
so a param group whose parameters form one contiguous arena run is updated by ONE vectorised HIP
kernel (float4, fma order matching ATen's ``add(alpha=...)``) instead of one launch per tensor.
``zero_grad`` zeroes the gradient arena in place (the arena views stay attached, which keeps the
bucketed reducer zero-copy). The learning rate can live on the device (``lr_tensor``) so a captured
hipGraph step follows an LR schedule without re-capture.
"""
from __future__ import annotations

import torch
from torch.optim import Optimizer

from . import _native
from .utils.arena import arena_for


class SGD(Optimizer):
    def __init__(
        self,
        params,
        lr: float = 1e-3,
        momentum: float = 0.0,
        dampening: float = 0.0,
        weight_decay: float = 0.0,
        nesterov: bool = False,
        *,
        maximize: bool = False,
        flat: bool = True,
    ):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if momentum < 0.0:
            raise ValueError(f"Invalid momentum value: {momentum}")
        if weight_decay < 0.0:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(
            lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay, nesterov=nesterov,
            maximize=maximize, foreach=None, differentiable=False, fused=None,
        )
        super().__init__(params, defaults)
        # callables run at the end of every step (DistributedDataParallel.early_buffer_broadcast
        # joins its end-of-backward buffer broadcast here, after the SGD it overlaps)
        self._post_step_joins = []
        self._flat = flat
        self._arena = None
        self._lr_tensor = None
        self._steps = 0
        self.fused_prep = True  # emit the next step's weight preparation from the step (one arena pass)
        self._step_counter = None  # a device step counter this step advances (DeviceLoader.advance_with)
        self._counter_pending = None
        self._overlap = None  # this iteration's per-bucket steps, run by a DDP reducer (bucket_steps)
        all_params = [p for g in self.param_groups for p in g["params"]]
        if flat and all_params and all_params[0].is_cuda:
            self._arena = arena_for(all_params)
            self._arena.on_relayout(self._on_relayout)

    def _on_relayout(self, arena):
        # the arena moved the momentum values with their parameters; re-point the state views
        if arena.momentum is None:
            return
        views = arena.momentum_views()
        for p in arena.params:
            st = self.state.get(p)
            if st and st.get("momentum_buffer") is not None:
                st["momentum_buffer"] = views[p._cdp_index]

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._adopt_momentum()

    def _adopt_momentum(self):
        """Loaded momentum buffers are fresh tensors, while a replayed hipGraph step reads and writes
        the arena's momentum storage: copy them into their arena views now (not at the next eager
        step), so a replay after ``load_state_dict`` continues from the loaded state."""
        a = self._arena
        if a is None or a.momentum is None:
            return
        views = a.momentum_views()
        with torch.no_grad():
            for p in a.params:
                st = self.state.get(p)
                b = st.get("momentum_buffer") if st else None
                if b is not None and b.data_ptr() != views[p._cdp_index].data_ptr():
                    views[p._cdp_index].copy_(b)
                    st["momentum_buffer"] = views[p._cdp_index]

    # ------------------------------------------------------------------ fused weight preparation
    def refresh_weight_prep(self) -> bool:
        """Re-derive the next forward's weight |max| / W^T from the current weights (in place).

        With ``fused_prep`` (default) the step itself writes them for the next forward. Eager forwards
        notice weights edited since (a bumped version) and prepare them anew; a replayed hipGraph
        cannot, so after editing weights between replays of a captured step call this first."""
        return self._arena.prep_refresh() if self._arena is not None else False

    # ------------------------------------------------------------------ device-side LR
    def lr_tensor(self) -> torch.Tensor:
        """A 1-element device tensor holding the LR of param group 0 (graph-capture friendly)."""
        if self._lr_tensor is None:
            dev = self.param_groups[0]["params"][0].device
            self._lr_tensor = torch.tensor([self.param_groups[0]["lr"]], dtype=torch.float32, device=dev)
        return self._lr_tensor

    def sync_lr_tensor(self):
        if self._lr_tensor is not None:
            self._lr_tensor.fill_(self.param_groups[0]["lr"])

    # ------------------------------------------------------------------ zero_grad
    def zero_grad(self, set_to_none: bool = True):
        # set_to_none (torch's default) lets the next backward's kernels write each gradient straight
        # into its arena slot, which autograd then adopts as p.grad without a copy (FlatArena.claim).
        super().zero_grad(set_to_none=set_to_none)
        if self._arena is not None:
            self._arena.reset_claims()

    # ------------------------------------------------------------------ step
    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self._overlap is not None:
            ov, self._overlap = self._overlap, None
            done = ov["reducer"].stepped_buckets()
            if done == ov["n"]:
                self._finish_overlapped(ov)
                self._run_post_step_joins()
                return loss
            if done:
                raise RuntimeError(f"overlapped optimizer step: only {done} of {ov['n']} buckets were stepped")
        self._counter_pending = self._step_counter
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            if self._arena is not None:
                self._arena.prep_valid = None  # re-marked below only by a fused step
            if params[0].is_cuda and not _native.force_reference():
                self._step_native(gi, group, params)
            else:
                self._step_reference(group, params)
        if self._counter_pending is not None:  # no fused launch took it (per-tensor / reference paths)
            c = self._counter_pending
            if c.is_cuda and not _native.force_reference():
                _native.lib().counter_inc(c)
            else:
                c += 1
            self._counter_pending = None
        self._steps += 1
        self._run_post_step_joins()
        return loss

    def add_post_step_join(self, fn):
        """Run ``fn()`` at the end of every ``step()`` (e.g. to order the current stream after
        communication issued during backward; see ``DistributedDataParallel.early_buffer_broadcast``)."""
        if fn not in self._post_step_joins:
            self._post_step_joins.append(fn)

    def _run_post_step_joins(self):
        for fn in getattr(self, "_post_step_joins", ()):
            fn()

    # ------------------------------------------------------------------ overlapped step (DDP)
    def bucket_steps(self, ranges, reducer):
        """Split this iteration's step over gradient buckets (``DistributedDataParallel.overlap_optimizer``).

        ``ranges``: the buckets' flat arena ranges in launch order. Returns one keyword dict per
        bucket for the reducer's ``set_bucket_step`` -- the SGD of that range, run on the reducer's
        step stream right after the bucket's all-reduce -- or None when the step cannot be split
        this iteration (several param groups, parameters outside one arena run, first and later
        momentum steps mixed, no native kernels). The next ``step()`` then only does the
        bookkeeping, provided the reducer stepped every bucket; hyperparameters are those at the
        time of this call (the forward), the first-step momentum rule (buf = d_p) is kept."""
        if self._arena is None or len(self.param_groups) != 1 or _native.force_reference():
            return None
        group = self.param_groups[0]
        params, arena = group["params"], self._arena
        if len(params) != len(arena.params) or any(not p.is_cuda for p in params):
            return None
        rng = arena.contiguous_range(params)
        ranges = [(int(s), int(e)) for s, e in ranges]
        if rng is None or not ranges or ranges[0][0] != rng[0] or ranges[-1][1] != rng[1]:
            return None
        if any(ranges[k][1] != ranges[k + 1][0] for k in range(len(ranges) - 1)):
            return None
        m = group["momentum"]
        first = True
        if m != 0.0:
            mviews = arena.momentum_views()
            bufs = [self.state[p].get("momentum_buffer") for p in params]
            if any(b is not None and b.data_ptr() != mviews[p._cdp_index].data_ptr() for b, p in zip(bufs, params)):
                return None  # e.g. loaded buffers not yet adopted: a normal step moves them in
            firsts = [b is None for b in bufs]
            if any(firsts) and not all(firsts):
                return None
            first = all(firsts)
        plan = arena.prep_plan_ranges(ranges) if self.fused_prep else None
        mom = arena.momentum_buffer() if m != 0.0 else None
        lr_t = self._lr_tensor
        out = []
        for k, (s, e) in enumerate(ranges):
            a = dict(p=arena.data[s:e], g=arena.grad[s:e], buf=mom[s:e] if mom is not None else None, lr_t=lr_t,
                     lr=group["lr"], momentum=m, dampening=group["dampening"], wd=group["weight_decay"],
                     nesterov=group["nesterov"], first=first, maximize=group["maximize"],
                     counter=self._step_counter if k == len(ranges) - 1 else None)
            sub = plan["subs"][k] if plan is not None else None
            if sub is not None:
                a.update(desc=sub["desc"], meta=sub["meta"], amax=plan["amax"])
            out.append(a)
        self._overlap = {"reducer": reducer, "n": len(out), "first": first and m != 0.0, "prep": plan is not None,
                         "params": list(params)}
        return out

    def cancel_bucket_steps(self):
        self._overlap = None

    def _finish_overlapped(self, ov):
        """Bookkeeping of a step the reducer ran bucket by bucket (no kernel here)."""
        arena = self._arena
        if ov["first"]:
            mviews = arena.momentum_views()
            for p in ov["params"]:
                self.state[p]["momentum_buffer"] = mviews[p._cdp_index]
        arena.prep_valid = None
        if ov["prep"]:
            arena.prep_mark_valid()
        self._counter_pending = None  # advanced by the last bucket's kernel
        self._steps += 1

    def advance_each_step(self, counter: torch.Tensor):
        """Advance ``counter`` (a device int64 step counter, e.g. a DeviceLoader's) by one in every
        ``step()``, inside the SGD kernel itself: one dispatch less per training step. Only for
        loops that fetch exactly one batch per optimizer step; ``None`` stops it."""
        self._step_counter = counter

    def _first_flags(self, params):
        firsts = [self.state[p].get("momentum_buffer") is None for p in params]
        return firsts

    def _step_native(self, gi, group, params):
        C = _native.lib()
        lr, m, damp, wd = group["lr"], group["momentum"], group["dampening"], group["weight_decay"]
        nest, maxim = group["nesterov"], group["maximize"]
        lr_t = self._lr_tensor if (gi == 0 and self._lr_tensor is not None) else None
        arena = self._arena
        rng = None
        if arena is not None and len(params) == len(group["params"]):
            rng = arena.contiguous_range(params)
            if rng is not None:
                arena.ensure_grads_in_arena(params)
        if rng is not None and m != 0.0:
            # momentum buffers must be the arena's views (first step: buf = d_p)
            firsts = self._first_flags(params)
            mom = arena.momentum_buffer()
            mviews = arena.momentum_views()
            consistent = all(
                (self.state[p].get("momentum_buffer") is None)
                or self.state[p]["momentum_buffer"].data_ptr() == mviews[p._cdp_index].data_ptr()
                for p in params
            )
            if not consistent:
                # e.g. after load_state_dict: move loaded buffers into the arena
                for p in params:
                    b = self.state[p].get("momentum_buffer")
                    if b is not None:
                        mviews[p._cdp_index].copy_(b)
                        self.state[p]["momentum_buffer"] = mviews[p._cdp_index]
                firsts = self._first_flags(params)
            if all(firsts) or not any(firsts):
                s, e = rng
                self._flat_step(C, arena, s, e, mom[s:e], lr_t, lr, m, damp, wd, nest, all(firsts), maxim)
                if all(firsts):
                    for p in params:
                        self.state[p]["momentum_buffer"] = mviews[p._cdp_index]
                return
        elif rng is not None and m == 0.0:
            s, e = rng
            self._flat_step(C, arena, s, e, None, lr_t, lr, 0.0, damp, wd, nest, True, maxim)
            return
        # general path: one launch per parameter (non-arena / partial groups)
        for p in params:
            st = self.state[p]
            buf = st.get("momentum_buffer")
            first = buf is None
            if m != 0.0 and first:
                buf = torch.empty_like(p, memory_format=torch.contiguous_format)
            pv = p.data if p.data.is_contiguous() else None
            g = p.grad
            if pv is None or not g.is_contiguous():
                # strided (channels_last) tensors: update through flat contiguous copies
                pc = p.data.contiguous()
                gc = g.contiguous()
                bc = buf.contiguous() if buf is not None else None
                C.sgd_step(pc.view(-1), gc.view(-1), bc.view(-1) if bc is not None else None, lr_t, lr, m, damp, wd,
                           1.0, nest, first, maxim)
                p.data.copy_(pc)
                if buf is not None and bc is not buf:
                    buf.copy_(bc)
            else:
                C.sgd_step(pv.view(-1), g.view(-1), buf.view(-1) if buf is not None else None, lr_t, lr, m, damp,
                           wd, 1.0, nest, first, maxim)
            if m != 0.0:
                st["momentum_buffer"] = buf

    def _flat_step(self, C, arena, s, e, mom, lr_t, lr, m, damp, wd, nest, first, maxim):
        """One launch over the arena range: plain SGD, or SGD that also writes the next forward's
        weight |max| partials and W^T (FlatArena.prep_plan_for) when a model registered them."""
        plan = arena.prep_plan_for(s, e) if self.fused_prep else None
        ctr, self._counter_pending = self._counter_pending, None
        if plan is None:
            C.sgd_step(arena.data[s:e], arena.grad[s:e], mom, lr_t, lr, m, damp, wd, 1.0, nest, first, maxim, ctr)
            return
        if "subs" in plan:  # the split plan of an overlapped step (same buffers): its ranges in turn
            last = len(plan["ranges"]) - 1
            for k, ((a, b), sub) in enumerate(zip(plan["ranges"], plan["subs"])):
                mk = mom[a - s:b - s] if mom is not None else None
                c = ctr if k == last else None
                if sub is None:
                    C.sgd_step(arena.data[a:b], arena.grad[a:b], mk, lr_t, lr, m, damp, wd, 1.0, nest, first, maxim, c)
                else:
                    C.sgd_step_prep(arena.data[a:b], arena.grad[a:b], mk, lr_t, lr, m, damp, wd, 1.0, nest, first,
                                    maxim, sub["desc"], sub["meta"], plan["amax"], c)
            arena.prep_mark_valid()
            return
        C.sgd_step_prep(arena.data[s:e], arena.grad[s:e], mom, lr_t, lr, m, damp, wd, 1.0, nest, first, maxim,
                        plan["desc"], plan["meta"], plan["amax"], ctr)
        arena.prep_mark_valid()

    def _step_reference(self, group, params):
        lr, m, damp, wd = group["lr"], group["momentum"], group["dampening"], group["weight_decay"]
        for p in params:
            d_p = p.grad if not group["maximize"] else -p.grad
            if wd != 0:
                d_p = d_p.add(p, alpha=wd)
            if m != 0:
                st = self.state[p]
                buf = st.get("momentum_buffer")
                if buf is None:
                    buf = torch.clone(d_p).detach()
                    st["momentum_buffer"] = buf
                else:
                    buf.mul_(m).add_(d_p, alpha=1 - damp)
                d_p = d_p.add(buf, alpha=m) if group["nesterov"] else buf
            p.add_(d_p, alpha=-lr)
