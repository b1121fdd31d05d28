"""Training driver: the reference's four stages behind one CLI.

Reference entry points (each a standalone script there):
  * Part 1  ``/root/reference/src/Part 1/main.py``   single process          -> ``--strategy none``
  * Part 2a ``/root/reference/src/Part 2a/main.py``  gather/scatter sync     -> ``--strategy gather_scatter``
  * Part 2b ``/root/reference/src/Part 2b/main.py``  blocking all-reduce     -> ``--strategy allreduce_blocking``
  * Part 3  ``/root/reference/src/Part 3/main.py``   DDP wrapper             -> ``--strategy ddp``
  plus ``--strategy bucketed_overlap`` (hook-driven bucketed all-reduce on an unwrapped model).

Same flags with the same meaning (``--master``, ``--num-nodes``, ``--rank``, ``--epochs``; port 6585,
global batch 256 split as ``int(256 / W)``), the same seeding, optimizer, loss, train/test loops and
the exact log strings (``Training loss after {} iterations is {}``, ``Forward/Backward/Average Pass
time in iter {} is {}``, ``Test set: Average loss: ...``). Also runs under ``torchrun`` (RANK /
WORLD_SIZE / LOCAL_RANK from the environment).

Deliberate deviation (documented): the reference never calls ``model.train()`` again after the first
``test_model`` (``src/Part 1/main.py:62``), so later epochs train with BatchNorm in eval mode. We
call ``model.train()`` at the start of every epoch; ``--reference-bn-quirk`` restores the original
behaviour.
"""
from __future__ import annotations

import argparse
import os
import time

import torch

from . import distributed as dist
from .data import DeviceLoader, DistributedSampler, cifar10_binary, synthetic_cifar10, synthetic_imagenet
from .models import get_model
from .ops import CrossEntropyLoss, count_correct
from .optim import SGD
from .parallel import (
    BucketedOverlap,
    DistributedDataParallel,
    average_gradients_allreduce,
    average_gradients_gather_scatter,
)
from .utils import PhaseTimer, latest_checkpoint, load_checkpoint, save_checkpoint, seed_everything
from .utils import profiling
from .utils.profiling import TraceRecorder


def _phase(trace, name):
    """A traced phase (chrome trace + roctx) or just a roctx range (emitted when CDP_ROCTX=1)."""
    return trace.phase(name) if trace is not None else profiling.range(name)


def train_model(model, train_loader, optimizer, criterion, rank=0, sync=None, strategy="none", max_iters=None,
                timer=None, on_iter=None, trace=None, print_fn=print):
    """One epoch. ``sync`` is the reference's ``average_gradients`` hook (or a BucketedOverlap)."""
    iter_number = 1
    epoch_loss = 0
    timer = timer or PhaseTimer(None)
    # Part 1/2a/2b print "epochs", Part 3 "iterations" (src/Part 1/main.py:49, src/Part 2a/main.py:104,
    # src/Part 2b/main.py:104, src/Part 3/main.py:105)
    unit = "iterations" if strategy in ("ddp", "bucketed_overlap") else "epochs"
    for batch_idx, (data, target) in enumerate(train_loader):
        timer.mark("start")
        with _phase(trace, "forward"):
            optimizer.zero_grad()
            predictions = model(data)
            if isinstance(sync, BucketedOverlap):
                sync.prepare(predictions)
        timer.mark("forward")
        with _phase(trace, "backward"):
            loss = criterion(predictions, target)
            loss.backward()
        if strategy in ("gather_scatter", "allreduce_blocking"):
            with _phase(trace, "sync"):
                if strategy == "gather_scatter":
                    average_gradients_gather_scatter(model, rank)
                else:
                    average_gradients_allreduce(model)
        with _phase(trace, "step"):
            optimizer.step()
        timer.mark("backward")

        epoch_loss += loss.detach()
        if on_iter is not None:
            on_iter(iter_number, loss)
        if iter_number % 20 == 0:
            epoch_loss = epoch_loss / 20
            print_fn("Training loss after {} {} is {}".format(iter_number, unit, epoch_loss))
            epoch_loss = 0
            fwd = timer.pop("forward")
            bwd = timer.pop("backward")
            if iter_number != 20:
                print_fn("Forward Pass time in iter {} is {}".format(iter_number, fwd / 20.0))
                print_fn("Backward Pass time in iter {} is {}".format(iter_number, bwd / 20.0))
                print_fn("Average Pass time in iter {} is {}".format(iter_number, (fwd + bwd) / 20.0))
        if max_iters is not None and iter_number >= max_iters:
            break
        iter_number += 1
    return iter_number


def test_model(model, test_loader, criterion, print_fn=print):
    model.eval()
    test_loss = 0
    correct = None
    n = 0
    with torch.no_grad():
        for batch_idx, (data, target) in enumerate(test_loader):
            output = model(data)
            test_loss += criterion(output, target)
            correct = count_correct(output, target, correct)
            n += 1
    test_loss /= max(1, n)
    correct = int(correct.sum().item()) if correct is not None else 0
    total = len(test_loader.dataset)
    print_fn(
        "Test set: Average loss: {:.4f}, Accuracy: {}/{} ({:.0f}%)\n".format(
            float(test_loss), correct, total, 100.0 * correct / total
        )
    )
    return float(test_loss), correct


def build_data(args, device, train: bool):
    if args.data.startswith("cifar10-bin:"):
        return cifar10_binary(args.data.split(":", 1)[1], train=train, device=device)
    if args.model.startswith("resnet"):
        n = args.synthetic_size or (1281 if train else 500)
        return synthetic_imagenet(n, seed=0 if train else 1, device=device)
    n = args.synthetic_size or (50000 if train else 10000)
    return synthetic_cifar10(n, seed=0, device=device, train=train, learnable=args.data == "synthetic-learnable")


def run(rank, size, epochs, batch_size, args):
    seed_everything(args.seed)
    batch_size = int(batch_size / float(dist.get_world_size()))
    device = dist.device() if dist.is_initialized() else args.device_obj
    training_set = build_data(args, device, True)
    train_sampler = DistributedSampler(training_set, num_replicas=size, rank=rank) if size > 1 else None
    train_loader = DeviceLoader(training_set, batch_size, sampler=train_sampler, shuffle=(size == 1), train=True,
                                seed=args.seed)
    print("Size of training set is {}".format(len(train_loader)))
    test_set = build_data(args, device, False)
    test_loader = DeviceLoader(test_set, batch_size, shuffle=False, train=False)
    print("Size of test set is {}".format(len(test_loader)))

    if dist.is_initialized() and device.type == "cuda":
        # which communicator carries the gradient collectives (stderr: stdout keeps the reference's lines)
        import sys

        kind = "rccl-native" if dist.native_communicator() is not None else "torch-" + str(dist.get_backend())
        print(f"[cdp] rank {rank}: collectives on {kind}"
              + (f" ({dist.comm_fallback_reason()})" if dist.comm_fallback_reason() else ""), file=sys.stderr)
    criterion = CrossEntropyLoss()
    model = get_model(args.model).to(device)
    sync = None
    strategy = args.strategy
    if strategy == "ddp":
        model = DistributedDataParallel(model, bucket_cap_mb=args.bucket_cap_mb)
    elif strategy == "bucketed_overlap":
        sync = BucketedOverlap(model, bucket_cap_mb=args.bucket_cap_mb)
    optimizer = SGD(model.parameters(), lr=args.lr, momentum=0.9, weight_decay=0.0001)

    start_epoch = 0
    if args.resume and args.checkpoint_dir:
        path = _agreed_checkpoint(args.checkpoint_dir, size)
        if path:
            st = load_checkpoint(path, model, optimizer, map_location=device)
            start_epoch = st.get("epoch", 0)
            print("Resumed from {} (epoch {})".format(path, start_epoch))
    trace = TraceRecorder(rank, device) if args.trace else None
    reducer = _reducer_of(model, sync)
    if trace is not None and reducer is not None:
        reducer.set_trace(True)
    for epoch in range(start_epoch, epochs):
        if not args.reference_bn_quirk or epoch == 0:
            model.train()
        start_time = time.time()
        timer = PhaseTimer(device)
        train_model(model, train_loader, optimizer, criterion, rank, sync=sync, strategy=strategy,
                    max_iters=args.iters, timer=timer, trace=trace)
        if device.type == "cuda":
            torch.cuda.synchronize()
        print("Training time after {} epoch is {}".format(epoch + 1, (time.time() - start_time)))
        test_model(model, test_loader, criterion)
        if args.checkpoint_dir:
            save_checkpoint(os.path.join(args.checkpoint_dir, f"ckpt_{epoch + 1}.pt"), model, optimizer,
                            epoch=epoch + 1, rank=rank)
    if trace is not None:
        if reducer is not None:
            trace.add_reducer_log(reducer.trace_log())
        path = args.trace if size == 1 else "{}.rank{}{}".format(*os.path.splitext(args.trace)[:1], rank,
                                                                 os.path.splitext(args.trace)[1] or ".json")
        trace.dump(path)
    return model


def _reducer_of(model, sync):
    if isinstance(model, DistributedDataParallel):
        return model.reducer
    if isinstance(sync, BucketedOverlap):
        return sync.reducer
    return None


def _agreed_checkpoint(directory, size):
    """Rank 0 picks the checkpoint; every rank must be able to read that same file.

    Only rank 0 writes checkpoints, so without a shared filesystem other ranks would silently start
    from scratch while rank 0 resumes (diverged replicas, mismatched epoch counts, hung collectives).
    """
    path = latest_checkpoint(directory) if dist.get_rank() == 0 else None
    if size == 1 or not dist.is_initialized():
        return path
    import torch.distributed as tdist

    box = [path]
    tdist.broadcast_object_list(box, src=0)
    path = box[0]
    if path is None:
        return None
    ok = torch.tensor([1 if os.path.isfile(path) else 0], dtype=torch.int64,
                      device=dist.device() if dist.device().type == "cuda" else "cpu")
    tdist.all_reduce(ok, op=tdist.ReduceOp.MIN)
    if int(ok.item()) != 1:
        raise RuntimeError(f"--resume: checkpoint {path} (chosen by rank 0) is not readable on every rank; "
                           "use a shared --checkpoint-dir")
    return path


def init_process(master, port, rank, size, fn, epochs=1, batch_size=256, backend="rccl", args=None):
    """Initialize the distributed environment (``src/Part 2a/main.py:148-153``)."""
    os.environ["MASTER_ADDR"] = master
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group(backend, rank=rank, world_size=size)
    try:
        return fn(rank, size, epochs, batch_size, args)
    finally:
        dist.destroy_process_group()


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Process arguments for training")
    p.add_argument("--master", metavar="master-address", default=os.environ.get("MASTER_ADDR"),
                   help="The IP address of Master")
    p.add_argument("--num-nodes", metavar="total-nodes", type=int, default=None, help="Total number of nodes")
    p.add_argument("--rank", metavar="rank", type=int, default=None, help="Rank of this node")
    p.add_argument("--epochs", metavar="epochs", type=int, default=1, help="Number of epochs")
    p.add_argument("--port", default=os.environ.get("MASTER_PORT", "6585"))
    p.add_argument("--backend", default=None, choices=["rccl", "nccl", "gloo"])
    p.add_argument("--strategy", default=None,
                   choices=["none", "gather_scatter", "allreduce_blocking", "bucketed_overlap", "ddp"])
    p.add_argument("--model", default="vgg11")
    p.add_argument("--data", default="synthetic",
                   help="synthetic (random labels) | synthetic-learnable (labels a fixed function of the image) "
                        "| cifar10-bin:<root>")
    p.add_argument("--synthetic-size", type=int, default=None)
    p.add_argument("--batch-size", type=int, default=256, help="global batch (split int(B/W) per rank)")
    p.add_argument("--lr", type=float, default=0.1)
    p.add_argument("--iters", type=int, default=None, help="max iterations per epoch")
    p.add_argument("--bucket-cap-mb", type=float, default=None)
    p.add_argument("--device", default="auto", choices=["auto", "cpu", "cuda"])
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--checkpoint-dir", default=None)
    p.add_argument("--resume", action="store_true")
    p.add_argument("--trace", default=None,
                   help="write a chrome trace (phases + reducer hook/bucket-launch events) to this path "
                        "(.rankN suffix per rank when distributed)")
    p.add_argument("--num-threads", type=int, default=4,
                   help="CPU intra-op threads for the CPU path (the reference pins 4: src/Part 1/main.py:11)")
    p.add_argument("--reference-bn-quirk", action="store_true",
                   help="reproduce the reference's missing model.train() after the first eval")
    return p.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    size = args.num_nodes if args.num_nodes is not None else int(os.environ.get("WORLD_SIZE", "1"))
    rank = args.rank if args.rank is not None else int(os.environ.get("RANK", "0"))
    if args.device == "auto":
        args.device_obj = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    else:
        args.device_obj = torch.device(args.device)
    if args.device_obj.type == "cpu":
        torch.set_num_threads(args.num_threads)
    if args.strategy is None:
        args.strategy = "ddp" if size > 1 else "none"
    if size > 1 or args.strategy != "none":
        backend = args.backend or ("rccl" if args.device_obj.type == "cuda" else "gloo")
        master = args.master or "127.0.0.1"
        return init_process(master, args.port, rank, size, run, args.epochs, args.batch_size, backend, args)
    return run(0, 1, args.epochs, args.batch_size, args)


if __name__ == "__main__":
    main()
