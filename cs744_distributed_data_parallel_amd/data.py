"""Data pipeline: CIFAR-10 / ImageNet-shaped datasets resident in GPU memory, rank sharding and a
fused on-GPU augmentation loader.

Reference pipeline (``/root/reference/src/Part 1/main.py:82-109``, ``src/Part 2a/main.py:24-55``):
torchvision ``CIFAR10`` -> ``RandomCrop(32, padding=4)`` -> ``RandomHorizontalFlip()`` ->
``ToTensor()`` -> ``Normalize(mean=[125.3,123.0,113.9]/255, std=[63.0,62.1,66.7]/255)``, a
``DistributedSampler(num_replicas=W, rank=r)`` (``set_epoch`` never called), ``DataLoader`` with
2 worker processes and ``pin_memory``; the test loader is not sharded.

MI355X design: the whole uint8 dataset (150 MB for CIFAR-10) is uploaded once to HBM; each batch is
one gather + crop + flip + normalize kernel that writes NHWC fp32 straight into the model's input
layout. No worker processes, no host->device copies in the training loop, and the per-sample
random crop / flip come from a counter-based hash on the device, so the loader is also
hipGraph-capturable. torchvision is not installed here, so datasets are either synthetic (random
images of the right shape, fixed seed) or read from the CIFAR-10 *binary* distribution
(``cifar-10-batches-bin/*.bin``, raw bytes -- no unpickling).
"""
from __future__ import annotations

import math
import os
from typing import Iterator, List, Optional

import numpy as np
import torch

from . import _native

CIFAR_MEAN = [x / 255.0 for x in [125.3, 123.0, 113.9]]
CIFAR_STD = [x / 255.0 for x in [63.0, 62.1, 66.7]]
IMAGENET_MEAN = [0.485, 0.456, 0.406]
IMAGENET_STD = [0.229, 0.224, 0.225]


class ImageDataset:
    """uint8 images ``[N, H, W, C]`` + int64 labels, optionally resident on a device."""

    def __init__(self, images: torch.Tensor, labels: torch.Tensor, mean, std, pad: int = 4, name: str = "dataset"):
        assert images.dtype == torch.uint8 and images.dim() == 4
        self.images, self.labels = images, labels.long()
        self.mean, self.std, self.pad, self.name = list(mean), list(std), pad, name

    def __len__(self):
        return self.images.shape[0]

    def to(self, device):
        return ImageDataset(self.images.to(device), self.labels.to(device), self.mean, self.std, self.pad, self.name)

    @property
    def shape(self):
        return tuple(self.images.shape[1:])


def synthetic_cifar10(n: int = 50000, seed: int = 0, device="cpu", train: bool = True,
                      learnable: bool = False) -> ImageDataset:
    """Random CIFAR-10-shaped data (uint8 32x32x3, 10 classes) -- a stand-in for the real set.

    ``learnable``: the label is a fixed function of the image (argmax of one fixed random projection
    of its 8x8-average-pooled, normalised pixels, the same projection for train and test), so the
    loss falls and test accuracy rises above chance -- a check of the whole pipeline that random
    labels cannot give."""
    g = torch.Generator().manual_seed(seed + (0 if train else 1))
    imgs = torch.randint(0, 256, (n, 32, 32, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (n,), dtype=torch.int64, generator=g)
    if learnable:
        proj = torch.randn(10, 3 * 4 * 4, generator=torch.Generator().manual_seed(12345))
        mean = torch.tensor(CIFAR_MEAN).view(1, 3, 1, 1)
        std = torch.tensor(CIFAR_STD).view(1, 3, 1, 1)
        for i in range(0, n, 4096):
            x = (imgs[i : i + 4096].permute(0, 3, 1, 2).float() / 255.0 - mean) / std
            feat = torch.nn.functional.avg_pool2d(x, 8).reshape(x.shape[0], -1)
            labels[i : i + 4096] = (feat @ proj.t()).argmax(1)
    return ImageDataset(imgs, labels, CIFAR_MEAN, CIFAR_STD, 4, "synthetic-cifar10").to(device)


def synthetic_imagenet(n: int = 1281, seed: int = 0, device="cpu", size: int = 224, classes: int = 1000) -> ImageDataset:
    g = torch.Generator().manual_seed(seed)
    imgs = torch.randint(0, 256, (n, size, size, 3), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, classes, (n,), dtype=torch.int64, generator=g)
    return ImageDataset(imgs, labels, IMAGENET_MEAN, IMAGENET_STD, 0, "synthetic-imagenet").to(device)


def cifar10_binary(root: str, train: bool = True, device="cpu") -> ImageDataset:
    """Read the CIFAR-10 binary release (``data_batch_{1..5}.bin`` / ``test_batch.bin``).

    Each record is 1 label byte + 3072 bytes (CHW, R then G then B planes).
    """
    d = root
    if os.path.isdir(os.path.join(root, "cifar-10-batches-bin")):
        d = os.path.join(root, "cifar-10-batches-bin")
    files = [f"data_batch_{i}.bin" for i in range(1, 6)] if train else ["test_batch.bin"]
    recs = []
    for f in files:
        raw = np.fromfile(os.path.join(d, f), dtype=np.uint8)
        recs.append(raw.reshape(-1, 3073))
    a = np.concatenate(recs, 0)
    labels = torch.from_numpy(a[:, 0].astype(np.int64))
    imgs = torch.from_numpy(a[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1).copy())
    return ImageDataset(imgs, labels, CIFAR_MEAN, CIFAR_STD, 4, "cifar10").to(device)


class DistributedSampler:
    """Same index semantics as ``torch.utils.data.distributed.DistributedSampler``.

    Pads to a multiple of ``num_replicas`` by repeating from the start, shuffles with a generator
    seeded by ``seed + epoch`` and takes ``indices[rank::num_replicas]``. As in the reference,
    ``set_epoch`` is optional (without it every epoch repeats the same permutation).
    """

    def __init__(self, dataset, num_replicas: int = 1, rank: int = 0, shuffle: bool = True, seed: int = 0,
                 drop_last: bool = False):
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"Invalid rank {rank}, rank should be in the interval [0, {num_replicas - 1}]")
        self.n = len(dataset)
        self.num_replicas, self.rank, self.shuffle, self.seed, self.drop_last = num_replicas, rank, shuffle, seed, drop_last
        self.epoch = 0
        if drop_last and self.n % num_replicas != 0:
            self.num_samples = math.ceil((self.n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(self.n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def indices(self) -> List[int]:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g).tolist()
        else:
            idx = list(range(self.n))
        if not self.drop_last:
            pad = self.total_size - len(idx)
            if pad <= len(idx):
                idx += idx[:pad]
            else:
                idx += (idx * math.ceil(pad / len(idx)))[:pad]
        else:
            idx = idx[: self.total_size]
        return idx[self.rank : self.total_size : self.num_replicas]

    def __iter__(self):
        return iter(self.indices())

    def __len__(self):
        return self.num_samples


class DeviceLoader:
    """Batches ``(data[B,C,H,W] fp32 channels_last, target[B] int64)`` from a device-resident dataset.

    ``train=True`` applies RandomCrop(pad)+RandomHorizontalFlip on the device; normalisation always.
    ``sampler`` (e.g. :class:`DistributedSampler`) picks the indices; without one the order is
    sequential (``shuffle=False``) or a seeded permutation (``shuffle=True``).
    """

    def __init__(self, dataset: ImageDataset, batch_size: int, sampler=None, shuffle: bool = False,
                 train: bool = True, drop_last: bool = False, seed: int = 0):
        self.ds, self.batch_size, self.sampler, self.shuffle = dataset, batch_size, sampler, shuffle
        self.train, self.drop_last, self.seed = train, drop_last, seed
        self.dev = dataset.images.device
        self._counter = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self._epoch = 0
        self._external_advance = False

    def _order(self) -> torch.Tensor:
        if self.sampler is not None:
            idx = torch.tensor(list(iter(self.sampler)), dtype=torch.int64)
        elif self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self._epoch)
            idx = torch.randperm(len(self.ds), generator=g)
        else:
            idx = torch.arange(len(self.ds), dtype=torch.int64)
        return idx.to(self.dev)

    def __len__(self):
        n = len(self.sampler) if self.sampler is not None else len(self.ds)
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def advance_with(self, optimizer) -> bool:
        """Let ``optimizer`` advance this loader's step counter inside its step kernel (cdp.SGD
        ``advance_each_step``) instead of a one-thread launch per batch. One batch per optimizer
        step only; GPU datasets only (returns False otherwise). ``advance_with(None)`` detaches it
        again (e.g. before gradient accumulation or an evaluation pass over the same loader): the
        loader then advances its counter at every batch itself. An eager batch() fetched twice
        without an optimizer step in between warns once (both batches would share a seed)."""
        prev = getattr(self, "_advancer", None)
        if optimizer is None:
            if prev is not None and getattr(prev, "_step_counter", None) is self._counter:
                prev.advance_each_step(None)
            self._advancer = None
            self._external_advance = False
            return True
        if self.dev.type != "cuda" or not hasattr(optimizer, "advance_each_step"):
            return False
        if prev is not None and prev is not optimizer:
            self.advance_with(None)
        optimizer.advance_each_step(self._counter)
        self._advancer = optimizer
        self._advance_seen = None
        self._external_advance = True
        return True

    def _check_one_batch_per_step(self):
        opt = getattr(self, "_advancer", None)
        if opt is None or torch.cuda.is_current_stream_capturing():
            return
        steps = getattr(opt, "_steps", None)
        if steps is not None and steps == self._advance_seen and not getattr(self, "_warned_reuse", False):
            import warnings

            warnings.warn("DeviceLoader: two batches without an optimizer step while the optimizer advances the "
                          "loader's step counter (advance_with): they share an augmentation seed and batch offset; "
                          "call advance_with(None) for gradient accumulation or evaluation", stacklevel=3)
            self._warned_reuse = True
        self._advance_seen = steps

    @property
    def dataset(self):
        return self.ds

    def batch(self, idx: torch.Tensor, offset: int, bsz: int, out: Optional[torch.Tensor] = None,
              nbatches: int = 0):
        """Produce one batch from ``idx[offset:offset+bsz]`` (graph-capturable on GPU).

        ``nbatches > 0``: the batch is ``idx[offset + (step % nbatches) * bsz :][:bsz]`` with ``step``
        the loader's on-device step counter, so one captured hipGraph walks the whole order with no
        per-step host work. The labels are gathered by the same kernel.
        """
        pad = self.ds.pad if self.train else 0
        flip = self.train
        if offset < 0 or offset + max(nbatches, 1) * bsz > idx.numel():
            raise ValueError(f"DeviceLoader.batch: offset {offset} + {max(nbatches, 1)} batches x {bsz} exceeds the "
                             f"{idx.numel()} indices of this shard")
        if self.dev.type == "cuda":
            C = _native.lib()
            target = torch.empty(bsz, dtype=torch.int64, device=self.dev)
            data = C.augment(self.ds.images, idx, offset, bsz, self.ds.mean, self.ds.std, pad, flip, self._counter,
                             self.seed, out, nbatches, self.ds.labels, target)
            if not self._external_advance:
                C.counter_inc(self._counter)
            else:
                self._check_one_batch_per_step()
            return data, target
        if nbatches > 0:
            offset += (int(self._counter.item()) % nbatches) * bsz
            if not pad:
                self._counter += 1  # (the padded path advances it itself)
        return self._cpu_batch(idx[offset : offset + bsz], pad, flip)

    def _cpu_batch(self, sel, pad, flip):
        imgs = self.ds.images.index_select(0, sel).permute(0, 3, 1, 2).float().div_(255.0)  # NCHW
        if pad:
            g = torch.Generator().manual_seed(self.seed * 1000003 + int(self._counter.item()))
            self._counter += 1
            B, C, H, W = imgs.shape
            padded = torch.nn.functional.pad(imgs, (pad, pad, pad, pad))
            out = torch.empty_like(imgs)
            oy = torch.randint(0, 2 * pad + 1, (B,), generator=g)
            ox = torch.randint(0, 2 * pad + 1, (B,), generator=g)
            fl = torch.rand(B, generator=g) < 0.5 if flip else torch.zeros(B, dtype=torch.bool)
            for b in range(B):
                crop = padded[b, :, oy[b] : oy[b] + H, ox[b] : ox[b] + W]
                out[b] = crop.flip(-1) if fl[b] else crop
            imgs = out
        mean = torch.tensor(self.ds.mean).view(1, -1, 1, 1)
        std = torch.tensor(self.ds.std).view(1, -1, 1, 1)
        imgs = (imgs - mean) / std
        return imgs.contiguous(memory_format=torch.channels_last), self.ds.labels.index_select(0, sel)

    def __iter__(self) -> Iterator:
        idx = self._order()
        n = idx.numel()
        self._epoch += 1
        b = self.batch_size
        stop = (n // b) * b if self.drop_last else n
        for off in range(0, stop, b):
            yield self.batch(idx, off, min(b, n - off))
