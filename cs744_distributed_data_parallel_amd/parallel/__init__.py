"""Data parallelism: communicators, the four gradient-sync strategies, bucketed reducer, DDP."""
from .comm import Communicator, RcclCommunicator, TorchCommunicator, Work
from .ddp import DistributedDataParallel
from .local import LocalCommunicator, LocalGroup
from .reducer import GradReducer
from .strategies import (
    STRATEGIES,
    BucketedOverlap,
    average_gradients,
    average_gradients_allreduce,
    average_gradients_gather_scatter,
    flat_alias,
)

DDP = DistributedDataParallel

__all__ = [
    "Communicator", "RcclCommunicator", "TorchCommunicator", "Work", "DistributedDataParallel", "DDP",
    "GradReducer", "STRATEGIES", "BucketedOverlap", "average_gradients", "average_gradients_allreduce",
    "average_gradients_gather_scatter", "flat_alias", "LocalGroup", "LocalCommunicator",
]
