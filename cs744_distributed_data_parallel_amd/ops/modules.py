"""nn.Module wrappers of the fused ops."""
import torch.nn as nn

from . import functional as CF


class CrossEntropyLoss(nn.Module):
    """``torch.nn.CrossEntropyLoss()`` (mean reduction) on the fused softmax-xent kernel.

    Reference: ``torch.nn.CrossEntropyLoss().to(device)`` at ``/root/reference/src/Part 1/main.py:110``.
    """

    def forward(self, logits, target):
        return CF.cross_entropy(logits, target)
