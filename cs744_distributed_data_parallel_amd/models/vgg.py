"""VGG family for 3x32x32 inputs / 10 classes (the reference's only model).

Parity with ``/root/reference/src/Part 1/model.py``:
  * ``cfg`` table for VGG11/13/16/19 (``:3-8``); ints are conv output channels, ``'M'`` a 2x2 max-pool;
  * ``layers`` is an ``nn.Sequential`` of ``Conv2d(k3,s1,p1,bias) -> BatchNorm2d -> ReLU [-> MaxPool2d]``
    built exactly like ``_make_layers`` (``:11-27``), and ``fc1 = Linear(512, 10)`` (``:39-40``),
    so parameter creation order, default initialisation under a seed, and the 58-key
    ``state_dict`` layout (``layers.{i}.weight|bias|running_mean|running_var|num_batches_tracked``,
    ``fc1.weight|bias``) are identical to the reference -- checkpoints load both ways.
  * factories ``VGG11()`` .. ``VGG19()`` (the reference only exposes ``VGG11``, ``:49-50``).

MI355X execution: ``forward`` walks the same modules but runs each
``Conv -> BN -> ReLU [-> MaxPool]`` group as ONE fused autograd op on NHWC (channels_last)
activations (implicit-GEMM MFMA conv with the bias + BatchNorm statistics in its epilogue,
then a single BN-apply + ReLU + 2x2-max pass), and ``fc1`` on the MFMA GEMM. Conv weights are
kept channels_last (physical OHWI = the GEMM's B^T layout) so no per-step relayout is needed.
On CPU tensors the plain ``nn.Sequential`` path runs (reference semantics).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops import functional as CF
from ..utils.arena import install_load_hooks

cfg = {
    "VGG11": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "VGG13": [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "VGG16": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
    "VGG19": [
        64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M",
    ],
}


def make_layers(layer_cfg, in_channels: int = 3) -> nn.Sequential:
    layers = []
    for v in layer_cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers.append(nn.Conv2d(in_channels, v, kernel_size=3, stride=1, padding=1, bias=True))
            layers.append(nn.BatchNorm2d(v))
            layers.append(nn.ReLU(inplace=True))
            in_channels = v
    return nn.Sequential(*layers)


class VGG(nn.Module):
    """VGG module for 3x32x32 input, 10 classes (``_VGG`` in the reference)."""

    def __init__(self, name: str = "VGG11", num_classes: int = 10, channels_last: bool = True):
        super().__init__()
        install_load_hooks(self)  # loaded weights refresh the optimizer's prepared products
        self.name = name
        self.layers = make_layers(cfg[name])
        flatten_features = 512
        self.fc1 = nn.Linear(flatten_features, num_classes)
        # fused execution plan: (conv index, bn index, followed-by-pool)
        plan = []
        mods = list(self.layers)
        for i, m in enumerate(mods):
            if isinstance(m, nn.Conv2d):
                pool = i + 3 < len(mods) and isinstance(mods[i + 3], nn.MaxPool2d)
                plan.append((i, i + 1, pool))
        self._plan = plan
        if channels_last:
            self.to_channels_last()

    def to_channels_last(self):
        for m in self.layers:
            if isinstance(m, nn.Conv2d):
                m.weight.data = m.weight.data.contiguous(memory_format=torch.channels_last)
        return self

    def forward(self, x):
        if CF.use_native(x):
            x = x.contiguous(memory_format=torch.channels_last)
            layers = self.layers
            # one launch: f16x2 operand scales of every conv weight + W^T for the data gradients
            # (the first conv's input needs no gradient: no transpose)
            need = [k > 0 or x.requires_grad for k in range(len(self._plan))]
            weights = [layers[ci].weight for ci, _, _ in self._plan]
            wam, wts = CF.weight_prep(weights, need)
            for k, (ci, bi, pool) in enumerate(self._plan):
                # each block's output feeds only the next block -- the last one's only fc1, through
                # the flatten: its BN statistics reduction rides on that consumer's backward
                # (CF.conv_bn_act bn_link; for the last block the fused classifier backward)
                x = CF.conv_bn_act(x, layers[ci], layers[bi], relu=True, pool=pool,
                                   w_amax=wam[k] if wam is not None else None, w_t=wts[k], bn_link=True)
            y = x.reshape(x.size(0), -1)
            CF.pass_link(x, y)  # the flatten is a view: the hand-off follows it
            return CF.linear(y, self.fc1.weight, self.fc1.bias)
        y = self.layers(x)
        y = y.reshape(y.size(0), -1)
        return self.fc1(y)


def VGG11(**kw):
    return VGG("VGG11", **kw)


def VGG13(**kw):
    return VGG("VGG13", **kw)


def VGG16(**kw):
    return VGG("VGG16", **kw)


def VGG19(**kw):
    return VGG("VGG19", **kw)
