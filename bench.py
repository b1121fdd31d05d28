#!/usr/bin/env python
"""Headline benchmark: VGG-11 training throughput (images/sec, whole node) on CIFAR-shaped data.

Metric/config from BASELINE.json: "images/sec (whole node) VGG-11 CIFAR-shaped at 1/2/4/8 MI355X".
One step = the reference's full training iteration (``/root/reference/src/Part 3/main.py:88-97``):
batch fetch + RandomCrop/Flip/Normalize (on-GPU kernel), zero_grad, forward, CrossEntropy, backward
with the gradient sync of ``--strategy`` (DDP wrapper by default: bucketed RCCL all-reduce
overlapped with backward), SGD(momentum 0.9, wd 1e-4) step. fp32 numerics (the reference's
precision), random-init weights, synthetic uint8 CIFAR-10-shaped images resident on the GPU. The
whole step is captured once as a hipGraph and replayed (eager fallback if capture fails).

Scaling: ``value`` is for ``--scaling`` (weak by default: 256 images per GPU per step, the
reference's per-process batch at W=1). For N > 1 the line also carries ``strong``: the reference's
own rule -- a fixed global batch of 256 split ``int(256/W)`` per rank
(``/root/reference/src/Part 2a/main.py:22``) -- and ``exposed_comm_ms``: ms/step with sync minus
ms/step of the same step without gradient sync (the part of the all-reduce backward did not hide).

Launch:
  python bench.py --gpus N ...            N > 1 without WORLD_SIZE: this process starts N rank
                                          processes itself (one per GPU) and never touches a GPU
  torchrun --nproc-per-node N bench.py --gpus N ...   the driver's way; same result
  python bench.py --gpus 2 --device cpu   gloo/CPU smoke of the multi-process path (no GPU)
Rank 0 prints ONE JSON line; any failing rank makes the launcher exit non-zero.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

BASELINE_IMG_S = 322.9  # reference Part 1, single process, B=256 (measured, CPU)
METRIC = "images/sec (whole node) VGG-11 CIFAR-shaped at 1/2/4/8 MI355X; scaling eff"
REF_GLOBAL_BATCH = 256
_GRAPH_FALLBACKS = []  # measurements that timed eager steps because a capture failed (see _Run._note_fallback)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--model", default="vgg11")
    p.add_argument("--local-batch", type=int, default=256, help="per-rank batch for weak scaling")
    p.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    p.add_argument("--strategy", default="ddp", choices=["ddp", "bucketed_overlap", "allreduce_blocking",
                                                          "gather_scatter"])
    p.add_argument("--no-graph", action="store_true", help="eager steps instead of one hipGraph replay per step")
    p.add_argument("--no-extra", action="store_true",
                   help="skip the secondary measurements (strong-scaling point, no-sync step for exposed comm)")
    p.add_argument("--backend", default="native", choices=["native", "torch"],
                   help="torch = stock PyTorch-ROCm ops + torch DDP (comparison only)")
    p.add_argument("--precision", default="fp32", choices=["fp32", "bf16"],
                   help="fp32 (default, the reference's precision; conv GEMMs fp32-accurate via the f16x2 "
                        "split, or CDP_CONV_GEMM=x3|f32) or bf16 (conv GEMM operands rounded to bf16, fp32 "
                        "accumulation: the non-parity fast mode)")
    p.add_argument("--global-batch", type=int, default=REF_GLOBAL_BATCH,
                   help="global batch of the strong-scaling rule, int(global/N) per rank (the reference's 256, "
                        "/root/reference/src/Part 2a/main.py:22)")
    p.add_argument("--bucket-cap-mb", type=float, default=None)
    p.add_argument("--dataset-size", type=int, default=50000)
    p.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                   help="cpu = gloo smoke mode of the multi-process path (reference ops, tiny sizes)")
    p.add_argument("--dist-backend", default="auto", choices=["auto", "gloo"],
                   help="gloo: rehearse the multi-rank GPU path on ONE GPU (all ranks share cuda:0, gradients "
                        "over gloo; not a performance mode)")
    return p.parse_args(argv)


# ---------------------------------------------------------------------------------- launcher
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(args) -> int:
    """Start ``--gpus`` rank processes (this process imports no GPU code and never execs)."""
    n = args.gpus
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if args.device == "cpu":
            env.setdefault("OMP_NUM_THREADS", "1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    try:
        alive = list(procs)
        while alive:
            for p in list(alive):
                r = p.poll()
                if r is None:
                    continue
                alive.remove(p)
                if r != 0 and rc == 0:
                    rc = r
                    print(f"[bench] rank {procs.index(p)} exited with {r}; stopping the others", file=sys.stderr)
                    for q in alive:
                        q.terminate()
            time.sleep(0.05)
    except KeyboardInterrupt:
        for p in procs:
            p.terminate()
        rc = 130
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
    return rc if rc >= 0 else 128 - rc


# ---------------------------------------------------------------------------------- one rank
class _Run:
    """Builds model/optimizer/data for one (local batch, sync on/off) point and times it."""

    def __init__(self, args, world, rank, dev, local_batch, sync_grads=True, model_name=None, strategy=None,
                 image_size=224):
        import torch

        import cs744_distributed_data_parallel_amd as cdp
        from cs744_distributed_data_parallel_amd.data import (
            DeviceLoader,
            DistributedSampler,
            synthetic_cifar10,
            synthetic_imagenet,
        )

        self.torch, self.cdp = torch, cdp
        self.args, self.world, self.dev, self.local_batch = args, world, dev, local_batch
        # diagnostic hook: CDP_BENCH_DDP_W1=1 wraps the model in DDP at one rank too (with
        # CDP_REDUCER_TEST_POSTOP the bucket all-reduces then run real RCCL kernels)
        self.ddp_w1 = os.environ.get("CDP_BENCH_DDP_W1") == "1" and world == 1
        self.sync_grads = sync_grads and (world > 1 or self.ddp_w1)
        cdp.utils.seed_everything(0)
        self.model_name = model_name = model_name or args.model
        self.imagenet = model_name.startswith("resnet")
        size = args.dataset_size if dev.type == "cuda" else min(args.dataset_size, 8 * local_batch)
        size = max(size, local_batch * world)  # at least one batch per rank
        if self.imagenet:  # BASELINE.json config #5: ResNet-50, ImageNet-shaped synthetic
            ds = synthetic_imagenet(min(size, 4 * local_batch * world), seed=0, device=dev, size=image_size)
        else:
            ds = synthetic_cifar10(size, seed=0, device=dev)
        sampler = DistributedSampler(ds, num_replicas=world, rank=rank) if world > 1 else None
        self.loader = DeviceLoader(ds, local_batch, sampler=sampler, shuffle=(world == 1), train=True)
        self.strategy = strategy = strategy or args.strategy
        self.sync = None
        if args.backend == "native":
            model = cdp.get_model(model_name).to(dev)
            if (world > 1 or self.ddp_w1) and strategy == "ddp":
                model = cdp.DistributedDataParallel(model, bucket_cap_mb=args.bucket_cap_mb)
            if world > 1 and strategy == "bucketed_overlap":
                self.sync = cdp.parallel.BucketedOverlap(model, bucket_cap_mb=args.bucket_cap_mb)
            self.opt = cdp.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
            # A/B hook: the optimizer step without the next forward's weight preparation (a separate
            # weight_prep launch per forward, as before round 4)
            self.opt.fused_prep = os.environ.get("CDP_BENCH_NO_FUSED_PREP") != "1"
            # one batch per step: the SGD kernel advances the loader's step counter
            self.loader.advance_with(self.opt)
            self.crit = cdp.CrossEntropyLoss()
        else:
            os.environ["CDP_FORCE_REFERENCE"] = "1"
            model = cdp.get_model(model_name).to(dev).to(memory_format=torch.channels_last)
            if world > 1:
                model = torch.nn.parallel.DistributedDataParallel(
                    model, device_ids=[dev.index] if dev.type == "cuda" else None)
            self.opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
            self.crit = torch.nn.CrossEntropyLoss()
        self.model = model
        self.order = self.loader._order()
        self.nb = max(1, self.order.numel() // local_batch)
        self.graph = None
        self.seed = None
        self.graph_collectives = None  # native-communicator collectives recorded in the captured step
        # test hooks: CDP_BENCH_BREAK_CAPTURE=1 (every rank) or =r (rank r only) invalidates the capture;
        # CDP_BENCH_CORRUPT_RANK=r perturbs rank r's gradient after the sync (replicas then diverge)
        bc = os.environ.get("CDP_BENCH_BREAK_CAPTURE")
        self.break_capture = bc == "1" if world == 1 else bc in ("all", str(rank))
        self.corrupt = os.environ.get("CDP_BENCH_CORRUPT_RANK") == str(rank) and world > 1

    def body(self):
        import contextlib

        cdp, strategy = self.cdp, self.strategy
        x, y = self.loader.batch(self.order, 0, self.local_batch, nbatches=self.nb)
        self.opt.zero_grad()
        nosync = (not self.sync_grads and self.world > 1 and hasattr(self.model, "no_sync"))
        with (self.model.no_sync() if nosync else contextlib.nullcontext()):
            out = self.model(x)
            if self.sync is not None and self.sync_grads:
                self.sync.prepare(out)
            loss = self.crit(out, y)
            if self.seed is None:  # persistent d(loss)/d(loss): no fill kernel in the captured step
                self.seed = self.torch.ones_like(loss)
            loss.backward(self.seed)
        if self.sync_grads and strategy == "allreduce_blocking":
            cdp.parallel.average_gradients_allreduce(self.model)
        elif self.sync_grads and strategy == "gather_scatter":
            cdp.parallel.average_gradients_gather_scatter(self.model)
        if self.corrupt:
            next(self.model.parameters()).grad.narrow(0, 0, 1).add_(1e-3)
        self.opt.step()
        if self.break_capture and self.torch.cuda.is_current_stream_capturing():
            loss.item()  # test hook: a host read of a captured value invalidates the capture
        return loss

    def prepare(self, warmup, dbg):
        torch = self.torch
        cuda = self.dev.type == "cuda"
        # eager warmup (includes the bucket rebuild in ready order after iteration 1)
        for i in range(max(3, warmup)):
            self.body()
        if cuda:
            torch.cuda.synchronize()
        dbg("eager warmup done")
        # gloo executes its collectives on the host, which no stream capture survives (and a rank
        # failing mid-capture would leave its peer blocked in the collective): eager steps
        # (a no-sync step of the per-tensor strategies has no collective in it: those are captured
        # under gloo too, which lets the one-GPU rehearsal exercise the capture agreement)
        no_coll = not self.sync_grads and self.strategy in ("allreduce_blocking", "gather_scatter")
        if self.args.no_graph or not cuda or (self.args.dist_backend == "gloo" and not no_coll):
            return
        from cs744_distributed_data_parallel_amd import distributed as D

        ok = True
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    self.body()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            cs = torch.cuda.Stream()
            cs.wait_stream(torch.cuda.current_stream())
            n0 = D.collective_counts()
            with torch.cuda.stream(cs):
                # thread-local capture mode: a failing rank's other threads (watchdog, autograd
                # workers) cannot invalidate it, and ending it below always leaves capture mode
                g.capture_begin(capture_error_mode="thread_local")
                try:
                    self.body()
                finally:
                    g.capture_end()
            torch.cuda.current_stream().wait_stream(cs)
            torch.cuda.synchronize()
            n1 = D.collective_counts()
            if n0 is not None and n1 is not None:
                self.graph_collectives = n1["captured"] - n0["captured"]
            self.graph = g
            dbg("captured")
        except Exception as e:  # pragma: no cover - depends on the runtime
            print(f"[bench] hipGraph capture failed ({str(e)[:200]!r}); timing eager steps", file=sys.stderr)
            self._note_fallback(f"capture failed on this rank: {str(e)[:160]}")
            ok = False
            self.graph = None
            self._recover_from_failed_capture()
        if self.world > 1:
            # all ranks replay graphs or all run eager. Agreed BEFORE any replay: a replay runs the
            # recorded collectives, which a rank that could not capture would never join (capture
            # itself records them without running them, so dropping every graph keeps the order)
            import torch.distributed as tdist

            store = tdist.distributed_c10d._get_default_store()
            _Run._gen = getattr(_Run, "_gen", 0) + 1
            keys = [f"cdp_bench_graph/{_Run._gen}/{r}" for r in range(self.world)]
            store.set(keys[tdist.get_rank()], "1" if ok else "0")
            store.wait(keys)
            if any(store.get(k) != b"1" for k in keys) and self.graph is not None:
                print("[bench] another rank could not capture; all ranks time eager steps", file=sys.stderr)
                self._note_fallback("another rank could not capture")
                self.graph.reset()
                self.graph = None
                self.graph_collectives = None
                self.opt.zero_grad()
        if self.graph is not None:
            # the W warmup steps again, as replays of the graph that is timed next: the eager warmup
            # above ran before the (host-side, GPU-idle) capture, and a timed region that starts
            # right after that idle gap pays the clock's ramp back up in its first steps
            for i in range(max(2, warmup)):
                self.graph.replay()
            torch.cuda.synchronize()

    def _note_fallback(self, reason):
        """Record which measurement times eager steps instead of graph replays, and why (the record's
        ``graph_fallbacks`` list; each entry's own ``hipgraph`` flag only says that it fell back)."""
        _GRAPH_FALLBACKS.append({"model": self.model_name, "strategy": self.strategy, "local_batch": self.local_batch,
                                 "sync_grads": self.sync_grads, "reason": reason})

    def _recover_from_failed_capture(self):
        """An invalidated capture leaves the thread's last HIP error set (the next launch would report
        it) and may leave a reducer armed mid-backward: clear both so eager steps can run."""
        torch = self.torch
        if self.args.backend == "native":
            self.cdp._native.lib().clear_hip_error()
        for r in (getattr(self.model, "reducer", None), getattr(self.sync, "reducer", None)):
            if isinstance(r, self.cdp.parallel.reducer.GradReducer):
                r.disarm()
        torch.cuda.synchronize()
        if self.args.backend == "native":
            self.cdp._native.lib().clear_hip_error()
        self.opt.zero_grad()

    def time(self, steps, dist):
        torch = self.torch
        cuda = self.dev.type == "cuda"
        if self.world > 1:
            dist.barrier()
        if cuda:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            if self.graph is not None:
                self.graph.replay()
            else:
                self.body()
        if cuda:
            torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        el_t = torch.tensor([el], dtype=torch.float64, device=self.dev)
        if self.world > 1:
            dist.all_reduce(el_t, "max")  # the slowest rank defines the step
        return float(el_t.item()) / steps * 1e3

    def replicas_identical(self, dist):
        """True when every rank's parameters + momentum are bit-identical (None at one rank)."""
        if self.world == 1:
            return None
        torch = self.torch
        dg = self.replica_digest()
        allg = [torch.empty_like(dg) for _ in range(self.world)]
        dist.all_gather(allg, dg)
        return all(torch.equal(allg[0].cpu(), a.cpu()) for a in allg)

    def bucket_plan(self):
        """The gradient buckets of this point's reducer in launch order (None without one)."""
        red = getattr(self.model, "reducer", None) or getattr(self.sync, "reducer", None)
        if red is None or not hasattr(red, "plan_summary"):
            return None
        mod = getattr(self.model, "module", self.model)
        return red.plan_summary({id(p): n for n, p in mod.named_parameters()})

    def replica_digest(self):
        """Exact digest of this replica's training state: the int64 sum of the parameters' and the
        momentum buffers' fp32 bit patterns (order-independent, bit-exact) and their fp64 sum. DDP's
        invariant (``/root/reference/src/Part 3/main.py:61,96-97``) is that every rank holds the same
        parameters after every step; BN running statistics are per-rank between forwards (DDP
        broadcasts them from rank 0 at the next forward) and are not part of the digest."""
        torch = self.torch
        ts = [p.detach() for p in self.model.parameters()]
        for p in self.model.parameters():
            st = self.opt.state.get(p) if hasattr(self.opt, "state") else None
            if st and st.get("momentum_buffer") is not None:
                ts.append(st["momentum_buffer"].detach())
        bits = torch.zeros((), dtype=torch.int64, device=self.dev)
        val = torch.zeros((), dtype=torch.float64, device=self.dev)
        for t in ts:
            t = t.contiguous().reshape(-1)
            bits += t.view(torch.int32).to(torch.int64).sum()
            val += t.to(torch.float64).sum()
        return torch.stack([bits, val.view(torch.int64)])

    def release(self):
        if self.graph is not None:
            self.graph.reset()
        self.graph = None
        # drop the autograd hooks of this point's reducer before the next point builds its own
        if isinstance(getattr(self.model, "reducer", None), self.cdp.parallel.reducer.GradReducer):
            self.model.reducer.remove()
        if self.sync is not None:
            self.sync.remove()
            self.sync = None


def _measure(args, world, rank, dev, lb, dbg, dist, steps=None, warmup=None, full=False, **kw):
    """ms/step of one more (local batch, model, sync) point, measured like the headline. With
    ``full``: (ms, hipgraph, replicas_identical, bucket plan)."""
    r = _Run(args, world, rank, dev, lb, **kw)
    r.prepare(args.warmup if warmup is None else warmup, dbg)
    ms = r.time(args.steps if steps is None else steps, dist)
    hg = r.graph is not None
    rep = r.replicas_identical(dist) if full else None
    plan = r.bucket_plan() if full else None
    r.release()
    del r
    return (ms, hg, rep, plan) if full else (ms, hg)


# The reference's three multi-process stages and the hook-driven bucketed strategy, in the order
# BASELINE.md lists them (its per-strategy rows map one-to-one onto these keys)
STRATEGY_REF = {
    "gather_scatter": "Part 2a: rank-0 gather -> mean -> scatter per parameter (src/Part 2a/main.py:117-127)",
    "allreduce_blocking": "Part 2b: blocking per-tensor all_reduce(SUM) / W after backward (src/Part 2b/main.py:116-119)",
    "bucketed_overlap": "backward-hook bucketed all-reduce overlapped with backward (BASELINE.json config #3)",
    "ddp": "Part 3: DistributedDataParallel wrapper (src/Part 3/main.py:61)",
}


def _strategies_block(args, world, rank, dev, dbg, dist, lb, known=None):
    """Every gradient-sync strategy at the reference's strong-scaling point (``lb`` = int(256 / W)
    images per rank): ms/step, the sync time the step exposes (vs the same step without gradient
    sync), ``scaling_eff`` = ms_no_sync / ms (1.0 = communication fully hidden) and whether the
    replicas stayed bit-identical. ``known`` = {strategy: (ms, hg, rep, plan)} already measured."""
    known = known or {}
    ms0, hg0 = _measure(args, world, rank, dev, lb, dbg, dist, sync_grads=False)
    out = {"local_batch": lb, "global_batch": lb * world,
           "no_sync": {"ms_per_step": round(ms0, 4), "value": round(lb * world / ms0 * 1e3, 1), "hipgraph": hg0}}
    for strat in STRATEGY_REF:
        if strat in known:
            ms, hg, rep, plan = known[strat]
        else:
            ms, hg, rep, plan = _measure(args, world, rank, dev, lb, dbg, dist, full=True, strategy=strat)
        ent = {"reference": STRATEGY_REF[strat], "ms_per_step": round(ms, 4), "value": round(lb * world / ms * 1e3, 1),
               "exposed_sync_ms": round(max(0.0, ms - ms0), 4), "scaling_eff": round(min(1.0, ms0 / ms), 4),
               "replicas_identical": rep, "hipgraph": hg}
        if plan is not None:
            ent["buckets"] = plan
        out[strat] = ent
    return out


def _resnet_ddp_block(args, world, rank, dev, dbg, dist, cpu):
    """BASELINE.json config #5 at N > 1: ResNet-50 (25.6M parameters in 161 tensors, ImageNet-shaped
    synthetic) under the DDP wrapper at 64 images per GPU (weak scaling), its buckets designed by the
    timed planner from the measured backward (the larger-model bucket-sizing stress; the reference's
    DDP bucketing is the one inside ``/root/reference/src/Part 3/main.py:61``). ms/step with and
    without gradient sync, the exposed communication, the bucket plan in launch order and the
    bit-identical-replicas check. CPU smoke mode: 2 images of 32x32 per rank."""
    lb, size = (2, 32) if cpu else (64, 224)
    steps, warm = min(args.steps, 10), 3
    kw = dict(model_name="resnet50", strategy="ddp", image_size=size)
    ms, hg, rep, plan = _measure(args, world, rank, dev, lb, dbg, dist, steps=steps, warmup=warm, full=True, **kw)
    ms0, _ = _measure(args, world, rank, dev, lb, dbg, dist, steps=steps, warmup=warm, sync_grads=False, **kw)
    out = {"local_batch": lb, "global_batch": lb * world, "image_shape": [3, size, size], "strategy": "ddp",
           "ms_per_step": round(ms, 4), "value": round(lb * world / ms * 1e3, 1), "unit": "images/sec",
           "ms_per_step_no_sync": round(ms0, 4), "exposed_comm_ms": round(max(0.0, ms - ms0), 4),
           "scaling_eff": round(min(1.0, ms0 / ms), 4), "replicas_identical": rep, "hipgraph": hg,
           "conv_gemm": "reference" if cpu else _conv_gemm_engine(args.backend)}
    if plan is not None:
        out["buckets"] = plan
    return out


def rank_main(args) -> int:
    import faulthandler

    faulthandler.enable()
    # hang guard: a stuck collective or kernel ends the process (with every thread's traceback)
    # instead of holding the node; generous against the ~1 min a run takes
    faulthandler.dump_traceback_later(float(os.environ.get("CDP_BENCH_TIMEOUT_S", "1200")), exit=True)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # native RCCL communicator unavailable on some rank -> all ranks agree to use torch's nccl (=RCCL)
    # process group instead of failing the run (distributed._init_native_rccl); "comm" in the JSON
    # says which one ran
    os.environ.setdefault("CDP_RCCL_FALLBACK", "1")
    if os.environ.get("CDP_BENCH_FAIL_RANK") == str(rank):  # launcher test hook
        raise SystemExit(f"[bench] rank {rank}: CDP_BENCH_FAIL_RANK")
    if world != args.gpus:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)

    import torch

    import cs744_distributed_data_parallel_amd as cdp
    from cs744_distributed_data_parallel_amd import distributed as dist

    def dbg(msg):
        if os.environ.get("CDP_BENCH_DEBUG"):
            print(f"[bench r{rank}] {msg}", file=sys.stderr, flush=True)

    cpu = args.device == "cpu"
    if cpu:
        dev = torch.device("cpu")
        torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "1")))
        if world > 1:
            dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        if args.dist_backend == "gloo":
            local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if world > 1 and args.dist_backend == "gloo":
            dist.init_process_group("gloo", rank=rank, world_size=world)
        elif world > 1 or os.environ.get("CDP_BENCH_DDP_W1") == "1":
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29561")
            # collectives that stall longer than 5 minutes are aborted by the communicator's watchdog
            dist.init_process_group("rccl" if args.backend == "native" else "nccl", rank=rank, world_size=world,
                                    comm_timeout_s=300.0)
        if args.backend == "native":
            cdp._native.lib()  # fail loudly if the HIP extension is missing
            if args.precision == "bf16":
                cdp._native.lib().set_conv_gemm("bf16")
    ranks_seen = dist.ranks_seen() if world > 1 else 1
    comm_kind = ("rccl-native" if dist.native_communicator() is not None else
                 ("gloo" if (cpu or args.dist_backend == "gloo") else "torch-nccl")) if world > 1 else "none"

    strong_lb = max(1, args.global_batch // world)
    main_lb = args.local_batch if args.scaling == "weak" else strong_lb

    run = _Run(args, world, rank, dev, main_lb, sync_grads=True)
    run.prepare(args.warmup, dbg)
    ms = run.time(args.steps, dist)
    hipgraph = run.graph is not None
    graph_collectives = run.graph_collectives
    # every rank's parameters + momentum after the timed steps must be bit-identical
    replicas_identical = run.replicas_identical(dist)
    bucket_plan = run.bucket_plan()
    run.release()
    del run

    extra = {}
    if bucket_plan is not None:
        extra["buckets"] = bucket_plan
    if world > 1 and not args.no_extra:
        ms_nosync, _ = _measure(args, world, rank, dev, main_lb, dbg, dist, sync_grads=False)
        extra["ms_per_step_no_sync"] = round(ms_nosync, 4)
        extra["exposed_comm_ms"] = round(max(0.0, ms - ms_nosync), 4)
        # the reference's whole multi-process experiment: its four sync strategies at its own
        # strong-scaling rule (global batch 256 split int(256 / W) per rank)
        known = {args.strategy: (ms, hipgraph, replicas_identical, bucket_plan)} if main_lb == strong_lb else None
        blk = _strategies_block(args, world, rank, dev, dbg, dist, strong_lb, known)
        extra["strategies"] = blk
        d = blk[args.strategy]
        eff = {args.scaling: round(min(1.0, ms_nosync / ms), 4)}
        if args.scaling == "weak":
            extra["strong"] = {"value": d["value"], "ms_per_step": d["ms_per_step"], "global_batch": strong_lb * world,
                               "local_batch": strong_lb, "strategy": args.strategy}
            eff["strong"] = d["scaling_eff"]
        # ms/step without gradient sync over ms/step with it (1.0 = communication fully hidden); the
        # driver computes the across-N scaling efficiency from the per-N values itself
        extra["scaling_eff"] = eff
        if args.model == "vgg11" and os.environ.get("CDP_BENCH_RESNET", "1") != "0":
            extra["resnet50"] = _resnet_ddp_block(args, world, rank, dev, dbg, dist, cpu)

    engine = "reference" if cpu else _conv_gemm_engine(args.backend)
    headline = (world == 1 and not args.no_extra and not cpu and args.backend == "native" and args.precision == "fp32"
                and args.model == "vgg11")
    if headline and engine == "f16x2":
        # the same step on the strict engine (3-term bf16 split: every conv GEMM output within the
        # fp32 per-element error bound, tests/test_accuracy_gpu.py), so both numbers are measured here
        C = cdp._native.lib()
        C.set_conv_gemm("x3")
        try:
            ms_x3, _ = _measure(args, world, rank, dev, main_lb, dbg, dist)
        finally:
            C.set_conv_gemm(engine)
        extra["strict_fp32"] = {"conv_gemm": "x3", "value": round(main_lb * world / ms_x3 * 1e3, 1),
                                "ms_per_step": round(ms_x3, 4)}
    if headline and args.local_batch == REF_GLOBAL_BATCH:
        # the reference's strong-scaling rule (int(256 / W) images per rank,
        # /root/reference/src/Part 2a/main.py:22): the per-GPU step of its W = 2 / 4 / 8 points,
        # measured here on one GPU (no gradient sync: what the W-rank run costs before communication)
        pts = []
        for w_ref in (2, 4, 8):
            lb = REF_GLOBAL_BATCH // w_ref
            ms_s, hg = _measure(args, 1, rank, dev, lb, dbg, dist, steps=max(args.steps, 20))
            pts.append({"reference_world_size": w_ref, "local_batch": lb, "ms_per_step": round(ms_s, 4),
                        "img_s_per_gpu": round(lb / ms_s * 1e3, 1), "hipgraph": hg})
        extra["per_gpu_strong"] = pts
        # BASELINE.json config #5 (ResNet-50, ImageNet-shaped, 64 images per GPU), one GPU
        ms_r, hg = _measure(args, 1, rank, dev, 64, dbg, dist, steps=min(args.steps, 10), warmup=3,
                            model_name="resnet50")
        extra["resnet50"] = {"local_batch": 64, "image_shape": [3, 224, 224], "ms_per_step": round(ms_r, 3),
                             "value": round(64 / ms_r * 1e3, 1), "unit": "images/sec", "hipgraph": hg,
                             "conv_gemm": engine}

    global_batch = main_lb * world
    img_s = global_batch / ms * 1e3
    imagenet = args.model.startswith("resnet")
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
            # fp32 operands and accumulation everywhere; every conv GEMM engine meets the fp32
            # per-element error bound on Gaussian, heavy-tailed, whole-image and whole-channel
            # dynamic range (tests/test_accuracy_gpu.py; f16x2 scales each GEMM row by its own image /
            # channel maximum). "strict_fp32" carries the x3 engine's number too.
            "dtype": _dtype_label(args.precision, engine),
            "data": ("synthetic (random uint8 ImageNet-shaped 224x224x3, GPU-resident, on-GPU flip/normalize); "
                     if imagenet else
                     "synthetic (random uint8 CIFAR-10-shaped 32x32x3, GPU-resident, on-GPU crop/flip/normalize); ")
                    + "random-init weights",
            "ranks_seen": ranks_seen,
            "replicas_identical": replicas_identical,
            "config": {
                "model": {"vgg11": "VGG-11", "resnet50": "ResNet-50"}.get(args.model, args.model),
                "global_batch": global_batch,
                "local_batch": main_lb,
                "seq_len": None,
                "image_shape": [3, 224, 224] if imagenet else [3, 32, 32],
                "parallelism": f"dp{world}",
                "strategy": args.strategy if world > 1 else "single",
                "comm": comm_kind,
                "comm_fallback_reason": dist.comm_fallback_reason() if world > 1 else None,
                "graph_fallbacks": _GRAPH_FALLBACKS,
                # native-communicator collectives recorded inside the captured step (replayed every
                # step); null when the step is not captured or collectives go through torch
                "graph_collectives": graph_collectives if hipgraph else None,
                "backend": args.backend,
                "device": "cpu" if cpu else "mi355x",
                "hipgraph": hipgraph,
                "optimizer": "SGD(lr=0.1, momentum=0.9, wd=1e-4)",
                # conv GEMM numerics, all with fp32 operands and fp32 accumulation: "f16x2" =
                # power-of-two-scaled operands split into two fp16 terms, three products on the
                # fp16 MFMA; "x3" = 3-term bf16 split, six products on the bf16 MFMA; "f32" =
                # exact fp32-input MFMA (docs/PERF.md, tests/test_kernels_gpu.py)
                "conv_gemm": engine,
            },
        }
        rec.update(extra)
        print(json.dumps(rec), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    faulthandler.cancel_dump_traceback_later()
    if replicas_identical is False:
        print(f"[bench] rank {rank}: replicas diverged after the timed steps", file=sys.stderr)
        return 3
    return 0


def _dtype_label(precision, engine):
    return "fp32" if precision == "fp32" else "bf16"


def _conv_gemm_engine(backend):
    if backend != "native":
        return "miopen"
    try:
        from cs744_distributed_data_parallel_amd import _native

        return _native.lib().get_conv_gemm()
    except Exception:  # pragma: no cover - CPU-only environments
        return "reference"


def main(argv=None) -> int:
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch(args)
    return rank_main(args)


if __name__ == "__main__":
    sys.exit(main())
