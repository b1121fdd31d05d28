#!/usr/bin/env python
"""Headline benchmark: VGG-11 training throughput (images/sec, whole node) on CIFAR-shaped data.

Metric/config from BASELINE.json: "images/sec (whole node) VGG-11 CIFAR-shaped at 1/2/4/8 MI355X".
One step = the reference's full training iteration (``/root/reference/src/Part 3/main.py:88-97``):
batch fetch + RandomCrop/Flip/Normalize (on-GPU kernel), zero_grad, forward, CrossEntropy, backward
with the bucketed RCCL all-reduce overlapped (DDP wrapper when N > 1), SGD(momentum 0.9,
wd 1e-4) step. fp32 end to end (the reference's precision), random-init weights, synthetic uint8
CIFAR-10-shaped images resident on the GPU. Weak scaling by default: 256 images per GPU per step
(the reference's per-process batch); ``--scaling strong`` keeps the reference's global 256.

Usage:  python bench.py [--gpus N --steps K --warmup W]
        (N > 1 is launched by the driver with torch.distributed.run, one rank per GPU)
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

BASELINE_IMG_S = 322.9  # reference Part 1, single process, B=256 (measured, CPU)
METRIC = "images/sec (whole node) VGG-11 CIFAR-shaped at 1/2/4/8 MI355X; scaling eff"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--model", default="vgg11")
    p.add_argument("--local-batch", type=int, default=256)
    p.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    p.add_argument("--strategy", default="ddp", choices=["ddp", "bucketed_overlap", "allreduce_blocking",
                                                          "gather_scatter"])
    p.add_argument("--no-graph", action="store_true", help="eager steps instead of one hipGraph replay per step")
    p.add_argument("--graph", action="store_true",
                   help="force hipGraph capture also for N > 1 (default: graph on 1 GPU, eager multi-GPU: at "
                        "B=256/GPU the step is GPU-bound, eager and graph time within noise)")
    p.add_argument("--backend", default="native", choices=["native", "torch"],
                   help="torch = stock PyTorch-ROCm ops + torch DDP (comparison only)")
    p.add_argument("--precision", default="fp32", choices=["fp32", "bf16"],
                   help="fp32 (default, the reference's precision; conv GEMMs fp32-accurate via the f16x2 "
                        "split, or CDP_CONV_GEMM=x3|f32) or bf16 (conv GEMM operands rounded to bf16, fp32 accumulation: "
                        "the non-parity fast mode)")
    p.add_argument("--bucket-cap-mb", type=float, default=None)
    p.add_argument("--dataset-size", type=int, default=50000)
    return p.parse_args()


def _dbg(msg):
    if os.environ.get("CDP_BENCH_DEBUG"):
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def main():
    import faulthandler

    faulthandler.enable()
    args = parse()
    # hang guard: a stuck collective or kernel ends the process (with every thread's traceback)
    # instead of holding the node; generous against the ~1 min a run takes
    faulthandler.dump_traceback_later(float(os.environ.get("CDP_BENCH_TIMEOUT_S", "1200")), exit=True)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)

    import cs744_distributed_data_parallel_amd as cdp
    from cs744_distributed_data_parallel_amd import distributed as dist
    from cs744_distributed_data_parallel_amd.data import (
        DeviceLoader,
        DistributedSampler,
        synthetic_cifar10,
        synthetic_imagenet,
    )

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # collectives that stall longer than 5 minutes are aborted by the communicator's watchdog
        dist.init_process_group("rccl" if args.backend == "native" else "nccl", rank=rank, world_size=world,
                                comm_timeout_s=300.0)
    if args.backend == "native":
        cdp._native.lib()  # fail loudly if the HIP extension is missing
        if args.precision == "bf16":
            cdp._native.lib().set_conv_gemm("bf16")

    local_batch = args.local_batch if args.scaling == "weak" else max(1, 256 // world)
    global_batch = local_batch * world
    cdp.utils.seed_everything(0)

    imagenet = args.model.startswith("resnet")
    if imagenet:  # BASELINE.json config #5: ResNet-50, ImageNet-shaped synthetic
        ds = synthetic_imagenet(min(args.dataset_size, 4 * local_batch * world), seed=0, device=dev)
    else:
        ds = synthetic_cifar10(args.dataset_size, seed=0, device=dev)
    sampler = DistributedSampler(ds, num_replicas=world, rank=rank) if world > 1 else None
    loader = DeviceLoader(ds, local_batch, sampler=sampler, shuffle=(world == 1), train=True)

    if args.backend == "native":
        model = cdp.get_model(args.model).to(dev)
        if world > 1 and args.strategy == "ddp":
            model = cdp.DistributedDataParallel(model, bucket_cap_mb=args.bucket_cap_mb)
        sync = None
        if world > 1 and args.strategy == "bucketed_overlap":
            sync = cdp.parallel.BucketedOverlap(model, bucket_cap_mb=args.bucket_cap_mb)
        opt = cdp.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        crit = cdp.CrossEntropyLoss()
    else:
        os.environ["CDP_FORCE_REFERENCE"] = "1"
        model = cdp.get_model(args.model).to(dev).to(memory_format=torch.channels_last)
        sync = None
        if world > 1:
            model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local])
        opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        crit = torch.nn.CrossEntropyLoss()

    order = loader._order()
    nb = max(1, order.numel() // local_batch)
    static_idx = torch.empty(local_batch, dtype=torch.int64, device=dev)

    def step(i):
        s = (i % nb) * local_batch
        static_idx.copy_(order[s:s + local_batch], non_blocking=True)
        return i

    def body():
        x, y = loader.batch(static_idx, 0, local_batch)
        opt.zero_grad()
        out = model(x)
        if sync is not None:
            sync.prepare(out)
        loss = crit(out, y)
        loss.backward()
        if world > 1 and args.strategy == "allreduce_blocking":
            cdp.parallel.average_gradients_allreduce(model)
        elif world > 1 and args.strategy == "gather_scatter":
            cdp.parallel.average_gradients_gather_scatter(model)
        opt.step()
        return loss

    # warmup (eager; includes bucket rebuild in ready order after iteration 1)
    n_eager_warm = max(3, args.warmup)
    for i in range(n_eager_warm):
        step(i)
        body()
    torch.cuda.synchronize()
    _dbg("eager warmup done")

    graph = None
    use_graph = (not args.no_graph and args.strategy in ("ddp", "bucketed_overlap")
                 and (world == 1 or args.graph))
    if use_graph:
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    body()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            _dbg("side-stream warmup done")
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                static_loss = body()
            torch.cuda.synchronize()
            _dbg("captured")
            for i in range(2):  # warm replays
                step(i)
                graph.replay()
            torch.cuda.synchronize()
        except Exception as e:  # pragma: no cover - depends on the runtime
            print(f"[bench] hipGraph capture failed ({e!r}); timing eager steps", file=sys.stderr)
            graph = None
            torch.cuda.synchronize()

    def run_one(i):
        step(i)
        if graph is not None:
            graph.replay()
        else:
            body()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        run_one(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    el_t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el_t, "max")
    el = float(el_t.item())
    ms = el / args.steps * 1e3
    img_s = global_batch * args.steps / el
    if rank == 0:
        rec = {
            "metric": METRIC if not imagenet else
            "images/sec (whole node) ResNet-50 ImageNet-shaped synthetic, bucketed DDP (BASELINE.json config #5)",
            "value": round(img_s, 1),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None if imagenet else round(img_s / BASELINE_IMG_S, 2),
            "dtype": "fp32" if args.precision == "fp32" else "bf16",
            "data": ("synthetic (random uint8 ImageNet-shaped 224x224x3, GPU-resident, on-GPU flip/normalize); "
                     if imagenet else
                     "synthetic (random uint8 CIFAR-10-shaped 32x32x3, GPU-resident, on-GPU crop/flip/normalize); ")
                    + "random-init weights",
            "config": {
                "model": {"vgg11": "VGG-11", "resnet50": "ResNet-50"}.get(args.model, args.model),
                "global_batch": global_batch,
                "local_batch": local_batch,
                "seq_len": None,
                "image_shape": [3, 224, 224] if imagenet else [3, 32, 32],
                "parallelism": f"dp{world}",
                "strategy": args.strategy if world > 1 else "single",
                "backend": args.backend,
                "hipgraph": graph is not None,
                "optimizer": "SGD(lr=0.1, momentum=0.9, wd=1e-4)",
                # conv GEMM numerics, all with fp32 operands and fp32 accumulation: "f16x2" =
                # power-of-two-scaled operands split into two fp16 terms, three products on the
                # fp16 MFMA; "x3" = 3-term bf16 split, six products on the bf16 MFMA (both: error vs
                # fp64 <= the exact fp32 MFMA's, tests/test_kernels_gpu.py, docs/PERF.md); "f32" =
                # exact fp32-input MFMA
                "conv_gemm": _conv_gemm_engine(args.backend),
            },
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()
    faulthandler.cancel_dump_traceback_later()


def _conv_gemm_engine(backend):
    if backend != "native":
        return "miopen"
    try:
        from cs744_distributed_data_parallel_amd import _native

        return _native.lib().get_conv_gemm()
    except Exception:  # pragma: no cover - CPU-only environments
        return "reference"


if __name__ == "__main__":
    main()
