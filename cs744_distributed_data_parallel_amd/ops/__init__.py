"""Fused, autograd-visible ops on the gfx950 kernels (see :mod:`.functional`)."""
from . import functional
from .functional import conv_bn_act, count_correct, cross_entropy, global_avg_pool, linear, max_pool2d, use_native
from .modules import CrossEntropyLoss

__all__ = [
    "functional", "conv_bn_act", "count_correct", "cross_entropy", "global_avg_pool", "linear", "max_pool2d",
    "use_native", "CrossEntropyLoss",
]
