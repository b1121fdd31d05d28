"""Autograd-visible fused ops backed by the gfx950 kernels.

Each public function takes the same modules / tensors as its ``torch.nn`` counterpart and is
numerically the same op; GPU tensors run the native HIP kernels (no silent fallback: a missing
extension raises), CPU tensors run the PyTorch reference composition (used by the CPU tests and
as the parity oracle).

Reference anchors: the VGG block ``Conv2d -> BatchNorm2d -> ReLU [-> MaxPool2d]`` of
``/root/reference/src/Part 1/model.py:11-27``; ``fc1`` (``:40,45``); ``CrossEntropyLoss``
(``/root/reference/src/Part 1/main.py:110``).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .. import _native

__all__ = [
    "GradSink",
    "conv_bn_act",
    "linear",
    "cross_entropy",
    "max_pool2d",
    "global_avg_pool",
    "use_native",
]


def use_native(*tensors) -> bool:
    if _native.force_reference():
        return False
    return _native.require(*tensors)


def _slot(p, needed: bool):
    """Arena view to write ``p``'s gradient into directly (None -> let the kernel allocate)."""
    if not needed or p is None:
        return None
    a = getattr(p, "_cdp_arena", None)
    return a.claim(p) if a is not None else None


def _bn_momentum(bn) -> float:
    return -1.0 if bn.momentum is None else float(bn.momentum)


# f16x2 conv engine: a tensor produced by one of our kernels carries its producer's "act max" --
# the per-image and per-channel |max| of what it wrote (csrc/kernels/act_max.h), from which the
# GEMMs that consume it derive one power-of-two scale per GEMM row -- tagged with the tensor's
# version so an in-place change after production invalidates it (the consumer then measures the
# tensor itself).
def _get_amax(t):
    tag = getattr(t, "_cdp_amax", None)
    if tag is None or tag[1] != t._version:
        return None
    return tag[0]


def _set_amax(t, amax):
    if amax is not None:
        t._cdp_amax = (amax, t._version)


def weight_amax(weights):
    """f16x2 engine: a model's conv weights' maxima (per output channel and per input channel, the
    operand scales of the forward and data-gradient GEMMs) in ONE launch -- a list, one entry per
    weight, for :func:`conv_bn_act`'s ``w_amax``; None for the other engines. Computed from the
    current weights, so it is valid whatever changed them."""
    if not weights or not use_native(weights[0]):
        return None
    parts, _ = _native.lib().weight_prep(list(weights), [False] * len(weights))
    return parts if parts else None


def weight_prep(weights, need_dgrad=None):
    """Per-step preparation of a model's conv weights in ONE launch (csrc weight_prep_kernel):
    ``(amax, wts)`` -- the f16x2 |max| partials per weight (None for the other engines) and the
    transposed data-gradient operand W^T per weight (None where ``need_dgrad[i]`` is False, e.g.
    the first conv, whose input needs no gradient). Both are computed from the current weights at
    every forward, so they are valid whatever changed the weights."""
    if not weights or not use_native(weights[0]):
        return None, None
    want = [True] * len(weights) if need_dgrad is None else [bool(f) for f in need_dgrad]
    C = _native.lib()
    # the last optimizer step may have prepared exactly these weights already (FlatArena.prep_lookup)
    arena = getattr(weights[0], "_cdp_arena", None)
    if arena is not None and all(getattr(w, "_cdp_arena", None) is arena for w in weights):
        hit = arena.prep_lookup(weights, want)
        if hit is not None:
            PREP_HITS[0] += 1
            amax, wts = hit
            return (amax if C.get_conv_gemm() == "f16x2" else None), wts
        arena.prep_request = (list(weights), want)
    amax, wts = C.weight_prep(list(weights), want)
    return (amax if amax else None), [t if f else None for t, f in zip(wts, want)]


PREP_HITS = [0]  # forwards that used the optimizer's fused weight preparation (tests read it)


# --------------------------------------------------------------------------- conv + BN + act
class GradSink:
    """Sums the two gradients of a tensor consumed by two fused ops without an autograd add.

    A ResNet block input x feeds conv1 and either the residual add of the last conv (identity
    block) or the downsample conv, so autograd would sum two full-size gradients with a separate
    add kernel. Both consumers share a sink: whichever backward runs first parks its gradient here
    and returns None for x; the second one accumulates the parked gradient into its own result --
    inside its data-gradient GEMM's epilogue when it is a conv -- and returns the sum. The result
    does not depend on the order in which autograd runs the two.
    """

    __slots__ = ("grad",)

    def __init__(self):
        self.grad = None

    @staticmethod
    def make(x):
        """A sink for ``x`` (None when x needs no gradient or CDP_GRAD_SINK=0)."""
        import os

        if not x.requires_grad or os.environ.get("CDP_GRAD_SINK", "1") == "0":
            return None
        return GradSink()


class _BNLink:
    """Backward hand-off between two chained blocks (``bn_link``): block L's output feeds only block
    L+1. Block L+1's backward, whose data-gradient reduction produces the gradient at block L's
    output anyway, also reduces block L's BatchNorm statistics from it in the same launch
    (csrc/kernels/bwd_fuse.hip) and leaves them in ``part``; block L's backward then skips its own
    statistics pass. ``gptr`` / ``gver`` pin the hand-off to that exact gradient tensor, unmodified
    (autograd accumulating a second consumer's gradient into it in place bumps its version), and
    ``consumers`` counts the fused blocks that read the tagged output: with two, neither takes the
    link and the producer reduces its own statistics."""

    __slots__ = ("y", "stats", "pool", "relu", "ps", "part", "gptr", "gver", "consumers")

    def __init__(self, y, stats, pool, relu, ps):
        self.y, self.stats, self.pool, self.relu, self.ps = y, stats, pool, relu, ps
        self.part, self.gptr, self.gver = None, None, None
        self.consumers = 0


LINK_HANDOFFS = [0]  # BN statistics reductions taken from the consumer block's backward (tests read it)


def pass_link(src, view):
    """Carry ``src``'s BN hand-off tag (:class:`_BNLink`) to ``view``, a view of it (same storage and
    version counter), e.g. the flatten between a block and the classifier."""
    tag = getattr(src, "_cdp_bnlink", None)
    if tag is not None and view.data_ptr() == src.data_ptr():
        view._cdp_bnlink = tag


def _get_link(t):
    tag = getattr(t, "_cdp_bnlink", None)
    if tag is None or tag[1] != t._version:
        return None
    return tag[0]


class _ConvBNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, gamma, beta, rm, rv, nbt, momentum, eps, training, stride, pad, pool, relu, residual,
                res_sink=None, dx_sink=None, w_amax=None, w_t=None, bn_link=False, defer_apply=False):
        C = _native.lib()
        # a residual that is a deferred BatchNorm branch (defer_apply below): its raw conv output and
        # stats go to this block's apply pass instead of the (never written) placeholder
        lazy = _get_deferred(residual) if residual is not None else None
        out, y, stats, xsave, out_amax, x_amax, w_amax, rmask = C.conv_bn_act_fwd(
            x, w, b, gamma, beta, rm, rv, nbt, momentum, eps, training, stride, pad, pool, relu,
            residual if lazy is None else None, _get_amax(x), w_amax,
            None if lazy is None else lazy[0], None if lazy is None else lazy[1], defer_apply,
        )
        if defer_apply:  # statistics only: `out` is a shape-only placeholder nothing may read
            out._cdp_deferred_bn = (y, stats, out._version)
        ctx.cfg = (stride, pad, pool, relu, training, b is not None, residual is not None)
        ctx.params = (w, b, gamma, beta)
        ctx.sinks = (res_sink, dx_sink)
        ctx.amax = (x_amax, w_amax)  # f16x2 engine only (else None): W and x are unchanged by backward
        ctx.w_t = w_t  # W^T from weight_prep (this step's weights), or None: dgrad transposes itself
        # a residual block's ReLU routing: its 1-bit-per-channel pass mask (1/16 of out's bytes) when
        # the kernel wrote one, else out itself
        zout = (rmask if rmask is not None else out) if residual is not None else None
        ctx.save_for_backward(xsave, w, y, stats, zout)  # xsave: x, or x zero-padded to 4k channels
        _set_amax(out, out_amax)
        # the producer of x handed over its BN (see _BNLink) if this block is its only consumer
        ctx.link_in = _get_link(x) if dx_sink is None else None
        if ctx.link_in is not None:
            ctx.link_in.consumers += 1
        ctx.link_out = None
        if bn_link and residual is None and _bwd_fuse_on():
            odd_pool = pool and (y.shape[2] % 2 == 1 or y.shape[3] % 2 == 1)
            ps = 3 if (b is not None and not odd_pool and training) else 2  # as conv_bn_act_bwd's
            ctx.link_out = _BNLink(y, stats, pool, relu, ps)
            out._cdp_bnlink = (ctx.link_out, out._version)
        return out

    @staticmethod
    def backward(ctx, gout):
        x, w, y, stats, zout = ctx.saved_tensors
        stride, pad, pool, relu, training, has_bias, has_res = ctx.cfg
        res_sink, dx_sink = ctx.sinks
        C = _native.lib()
        wp, bp, gp, betap = ctx.params
        nig = ctx.needs_input_grad
        addend, park_dx = None, False
        if dx_sink is not None and nig[0]:
            if dx_sink.grad is None:
                park_dx = True
            else:
                addend, dx_sink.grad = dx_sink.grad, None
        part_in, lo = None, ctx.link_out
        if lo is not None:
            if (lo.part is not None and lo.consumers == 1 and lo.gptr == gout.data_ptr()
                    and lo.gver == gout._version):
                part_in = lo.part
                LINK_HANDOFFS[0] += 1
            lo.part = lo.gptr = lo.gver = None
        li = ctx.link_in
        prev = (None, None, False, False, 2)
        if li is not None and li.consumers == 1 and nig[0] and not park_dx and addend is None:
            prev = (li.y, li.stats, li.pool, li.relu, li.ps)
        dx, dw, db, dgamma, dbeta, dres, prev_part, _ = C.conv_bn_act_bwd(
            gout, x, w, y, stats, stride, pad, pool, relu, nig[0], has_bias, zout, training,
            _slot(wp, nig[1]), _slot(bp, nig[2] and has_bias), _slot(gp, nig[3]), _slot(betap, nig[4]), addend,
            *ctx.amax, ctx.w_t, part_in, *prev, bp,
        )
        ctx.w_t = None
        if li is not None:
            li.part = prev_part if (prev_part is not None and dx is not None) else None
            li.gptr = dx.data_ptr() if li.part is not None else None
            li.gver = dx._version if li.part is not None else None
            ctx.link_in = None
        if park_dx:
            dx_sink.grad, dx = dx, None
        if has_res and res_sink is not None and nig[15]:
            if res_sink.grad is None:
                res_sink.grad, dres = dres, None
            else:
                dres = dres.add_(res_sink.grad)
                res_sink.grad = None
        return (
            dx if ctx.needs_input_grad[0] else None,  # None also when parked in dx_sink
            dw,
            db if has_bias else None,
            dgamma if ctx.needs_input_grad[3] else None,
            dbeta if ctx.needs_input_grad[4] else None,
            None, None, None, None, None, None, None, None, None, None,
            dres if has_res else None,
            None, None, None, None, None, None,
        )


def _get_deferred(t):
    """(raw conv output, stats) of a defer_apply placeholder that is still unmodified, else None."""
    tag = getattr(t, "_cdp_deferred_bn", None)
    if tag is None:
        return None
    if tag[2] != t._version:
        raise RuntimeError("a deferred BatchNorm placeholder was modified in place; it holds no values")
    return tag[0], tag[1]


def _bwd_fuse_on() -> bool:
    import os

    return os.environ.get("CDP_BWD_FUSE", "1") != "0"


def conv_bn_act(x, conv, bn, relu: bool = True, pool: bool = False, residual=None, res_sink=None, dx_sink=None,
                w_amax=None, w_t=None, bn_link: bool = False, defer_apply: bool = False):
    """``[maxpool2x2](act(bn(conv(x)) [+ residual]))`` for an ``nn.Conv2d`` / ``nn.BatchNorm2d`` pair.

    ``pool`` is the reference's ``MaxPool2d(kernel_size=2, stride=2)``; ``relu`` its
    ``ReLU(inplace=True)``; ``residual`` (ResNet) is added after BN and before the activation.
    ``res_sink`` / ``dx_sink`` (:class:`GradSink`, GPU path only) route the residual gradient of an
    identity block into the data-gradient GEMM of the block's first conv instead of an autograd add.
    ``w_amax`` (f16x2 engine): ``conv.weight``'s entry of :func:`weight_amax`, else measured here.
    ``w_t``: ``conv.weight``'s W^T from :func:`weight_prep` (else backward transposes it).
    ``bn_link``: the caller guarantees the result feeds exactly one op, the next ``conv_bn_act``
    (a VGG chain); its backward then reduces this block's BN statistics for it (:class:`_BNLink`).
    ``defer_apply`` (GPU path; no ``relu`` / ``pool`` / ``residual``): compute the conv and the BN
    statistics only and return a shape-only placeholder, to be passed as the ``residual`` of exactly
    one ``conv_bn_act``, which then applies this BatchNorm inside its own apply pass (a ResNet
    downsample branch: its normalized output is never written or read back).
    """
    stride = conv.stride[0]
    pad = conv.padding[0]
    if use_native(x):
        training = bn.training or not bn.track_running_stats
        track = bn.track_running_stats and bn.training
        return _ConvBNAct.apply(
            x,
            conv.weight,
            conv.bias,
            bn.weight,
            bn.bias,
            bn.running_mean if (track or not training) else None,
            bn.running_var if (track or not training) else None,
            bn.num_batches_tracked if track else None,
            _bn_momentum(bn),
            float(bn.eps),
            training,
            stride,
            pad,
            pool,
            relu,
            residual,
            res_sink,
            dx_sink,
            w_amax if w_amax is not None else getattr(conv, "_cdp_wamax", None),
            w_t if w_t is not None else getattr(conv, "_cdp_wt", None),
            bn_link,
            defer_apply,
        )
    y = F.conv2d(x, conv.weight, conv.bias, conv.stride, conv.padding)
    y = bn(y)
    if residual is not None:
        y = y + residual
    if relu:
        y = F.relu(y)
    if pool:
        y = F.max_pool2d(y, 2, 2)
    return y


# --------------------------------------------------------------------------- linear
class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        ctx.params = (w, b)
        ctx.narrow = w.shape[0] <= 16
        ctx.fused = None  # (dlogits, dx, dw, db) from a loss backward that did this backward too (_XEnt)
        # the producer of x (VGG's last block, through the flatten) handed over its BN statistics
        # reduction (_BNLink): the fused classifier backward can make it from the dX it forms
        ctx.link_in = _get_link(x) if ctx.narrow else None
        if ctx.link_in is not None:
            ctx.link_in.consumers += 1
        return _native.lib().linear_fwd(x, w, b)

    @staticmethod
    def backward(ctx, gy):
        f, ctx.fused = ctx.fused, None
        ctx.link_in = None
        if f is not None and gy.data_ptr() == f[0].data_ptr() and gy._version == f[0]._version:
            # the incoming gradient IS the cross-entropy gradient the fused launch started from
            # (with a second consumer of the logits autograd would have summed into a new tensor)
            return f[1], f[2], f[3]
        x, w = ctx.saved_tensors
        wp, bp = ctx.params
        nig = ctx.needs_input_grad
        dx, dw, db = _native.lib().linear_bwd(gy, x, w, nig[0], ctx.has_bias, _slot(wp, nig[1]),
                                              _slot(bp, nig[2] and ctx.has_bias))
        return (dx if ctx.needs_input_grad[0] else None), dw, (db if ctx.has_bias else None)


def linear(x, weight, bias=None):
    if use_native(x) and x.dim() == 2:
        return _Linear.apply(x, weight, bias)
    return F.linear(x, weight, bias)


# --------------------------------------------------------------------------- cross entropy
class _XEnt(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target):
        ctx.save_for_backward(logits, target)
        # logits straight from a narrow native Linear (VGG's fc1): its backward rides on ours
        node = logits.grad_fn
        ctx.lin = node if (getattr(node, "narrow", False) and hasattr(node, "fused")
                           and logits.shape[0] * logits.shape[1] <= _XENT_LIN_MAX) else None
        return _native.lib().xent_fwd(logits, target)

    @staticmethod
    def backward(ctx, g):
        logits, target = ctx.saved_tensors
        lin, ctx.lin = ctx.lin, None
        if lin is not None and os.environ.get("CDP_FUSED_CLASSIFIER", "1") != "0":
            x, w = lin.saved_tensors
            wp, bp = lin.params
            nig = lin.needs_input_grad
            has_b = lin.has_bias
            li, lin.link_in = lin.link_in, None
            link = li is not None and li.consumers == 1 and nig[0] and li.y.shape[2] == li.y.shape[3] == (
                2 if li.pool else 1)
            dl, dx, dw, db, part = _native.lib().xent_linear_bwd(
                g.reshape(1), logits, target, x, w, nig[0], has_b, _slot(wp, nig[1]), _slot(bp, nig[2] and has_b),
                li.y if link else None, li.stats if link else None, bool(li.pool) if link else False,
                bool(li.relu) if link else False, li.ps if link else 2)
            if link:  # the producer block's backward takes these partials if its gradient is this dX
                li.part, li.gptr, li.gver = part, dx.data_ptr(), dx._version
            lin.fused = (dl, dx if nig[0] else None, dw, db if has_b else None)
            return dl, None
        return _native.lib().xent_bwd(g.reshape(1), logits, target), None


_XENT_LIN_MAX = 8192  # batch x classes held in each block's LDS (csrc kernels.h kXentLinMax)


def cross_entropy(logits, target):
    """Mean-reduced softmax cross-entropy (``torch.nn.CrossEntropyLoss()`` defaults)."""
    if use_native(logits) and logits.dim() == 2 and logits.dtype == torch.float32:
        return _XEnt.apply(logits, target)
    return F.cross_entropy(logits, target)


def count_correct(logits, target, out=None):
    """Top-1 correct count (``output.max(1)`` + ``eq`` + ``sum``) as an int64 device tensor."""
    if use_native(logits):
        if out is None:
            out = torch.zeros(1, dtype=torch.long, device=logits.device)
        _native.lib().xent_fwd(logits.detach().float().contiguous(), target, out)
        return out
    c = logits.max(1)[1].eq(target).sum().reshape(1)
    if out is None:
        return c
    out += c
    return out


# --------------------------------------------------------------------------- pooling
class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, arg = _native.lib().maxpool2d_fwd(x, k, s, p)
        ctx.save_for_backward(arg)
        ctx.in_shape = list(x.shape)
        ctx.ksp = (k, s, p)
        _set_amax(y, _get_amax(x))  # max|maxpool(x)| <= max|x|: the input's bound still holds
        return y

    @staticmethod
    def backward(ctx, gy):
        (arg,) = ctx.saved_tensors
        return _native.lib().maxpool2d_bwd(gy, arg, ctx.in_shape, *ctx.ksp), None, None, None


def max_pool2d(x, kernel_size, stride=None, padding=0):
    stride = kernel_size if stride is None else stride
    if use_native(x) and x.shape[1] % 4 == 0:
        return _MaxPool.apply(x, int(kernel_size), int(stride), int(padding))
    return F.max_pool2d(x, kernel_size, stride, padding)


class _AvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.in_shape = list(x.shape)
        return _native.lib().avgpool_fwd(x)

    @staticmethod
    def backward(ctx, gy):
        return _native.lib().avgpool_bwd(gy, ctx.in_shape)


def global_avg_pool(x):
    """``AdaptiveAvgPool2d(1)`` + ``flatten(1)`` -> [N, C]."""
    if use_native(x):
        return _AvgPool.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
