"""Seeding exactly like the reference (``torch.manual_seed(0)``; ``numpy.random.seed(0)`` on every rank,
``/root/reference/src/Part 2a/main.py:20-21``): identical initial weights on all ranks even without
a broadcast (Parts 2a/2b rely on this)."""
import random

import numpy
import torch


def seed_everything(seed: int = 0):
    torch.manual_seed(seed)
    numpy.random.seed(seed)
    random.seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
