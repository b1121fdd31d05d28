"""MI355X-native distributed data-parallel training engine.

Capabilities of the CS744 "Distributed Data Parallel" reference (VGG-11 / CIFAR-10; single process,
gather/scatter sync, blocking all-reduce sync, DDP wrapper), re-designed for AMD Instinct MI355X
(gfx950): hand-written HIP/CDNA4 kernels (MFMA implicit-GEMM convolutions with fused BatchNorm
statistics, fused BN+ReLU+MaxPool, fused softmax cross-entropy, single-launch SGD over flat
arenas, on-GPU augmentation), a native C++ RCCL communicator and a C++ bucketed gradient reducer
overlapped with autograd.

Typical use (mirrors the reference API)::

    import cs744_distributed_data_parallel_amd as cdp
    cdp.distributed.init_process_group("rccl")
    model = cdp.parallel.DistributedDataParallel(cdp.models.VGG11().cuda())
    opt = cdp.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    loss = cdp.ops.CrossEntropyLoss()(model(x), y); loss.backward(); opt.step()
"""
from . import _native, data, distributed, models, ops, optim, parallel, utils
from .models import VGG11, VGG13, VGG16, VGG19, ResNet, get_model, resnet18, resnet34, resnet50, resnet101, resnet152
from .ops import CrossEntropyLoss
from .optim import SGD
from .parallel import DDP, DistributedDataParallel

__version__ = "0.1.0"

__all__ = [
    "_native", "data", "distributed", "models", "ops", "optim", "parallel", "utils",
    "VGG11", "VGG13", "VGG16", "VGG19", "get_model", "ResNet", "resnet18", "resnet34", "resnet50", "resnet101",
    "resnet152", "CrossEntropyLoss", "SGD",
    "DDP", "DistributedDataParallel", "native_available",
]


def native_available() -> bool:
    return _native.available()
