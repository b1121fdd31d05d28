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
Rank 0 prints ONE JSON line. For N > 1 every measurement is a phase run by fresh per-rank worker
processes under a supervisor (see ``supervise``): the headline first, then the secondary points in
order of risk, each with its own time limit; a secondary point that fails, crashes or hangs on any
rank becomes ``{"error": ...}`` in its block and the run still exits 0 with the headline. Only a
failed headline (no measurement) or diverged replicas make the run exit non-zero.
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
_LAST_GRAPH_COLLECTIVES = [None]  # native collectives recorded in the last measured captured step
# profiling aid (CDP_GEMM_LOG=1 CDP_GEMM_LOG_OUT=path, eager runs): the last step's GEMM launches as
# JSON (kind, M, N, K, tile, splits), to label a rocprofv3 trace's dispatches (scripts/pmc_resnet_layers.py)
_GEMM_LOG_OUT = os.environ.get("CDP_GEMM_LOG_OUT")


def _dump_gemm_log(cdp):
    if not _GEMM_LOG_OUT:
        return
    rows = [dict(zip(("kind", "M", "N", "K", "bm", "bn", "splits"), r)) for r in cdp._native.lib().gemm_log(False)]
    with open(_GEMM_LOG_OUT, "w") as f:
        json.dump(rows, f)


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
    p.add_argument("--extras", default="all",
                   help="N > 1: comma list of the secondary phases to run (no_sync, strong_ddp, strong_no_sync, "
                        "strong_allreduce_blocking, strong_bucketed_overlap, resnet50_ddp, resnet50_no_sync, "
                        "strong_gather_scatter), default all")
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
    p.add_argument("--overlap-step", action="store_true",
                   help="DDP: run the SGD step bucket by bucket right after each bucket's all-reduce "
                        "(DistributedDataParallel.overlap_optimizer); recorded as config.optimizer_overlap")
    p.add_argument("--early-bcast", action="store_true",
                   help="DDP: broadcast the BN buffers at the end of backward behind the last bucket, joined "
                        "after the SGD (DistributedDataParallel.early_buffer_broadcast); recorded as "
                        "config.early_buffer_broadcast")
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
            if args.overlap_step and isinstance(model, cdp.DistributedDataParallel):
                model.overlap_optimizer(self.opt)
            if args.early_bcast and isinstance(model, cdp.DistributedDataParallel) and self.dev.type == "cuda":
                model.early_buffer_broadcast(self.opt)
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
        if _GEMM_LOG_OUT and self.args.backend == "native" and not self.torch.cuda.is_current_stream_capturing():
            cdp._native.lib().gemm_log(True)  # keep only the latest step's GEMM launches (_dump_gemm_log)
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
    _maybe_fault(r)
    ms = r.time(args.steps if steps is None else steps, dist)
    hg = r.graph is not None
    _LAST_GRAPH_COLLECTIVES[0] = r.graph_collectives if hg else None
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


# ---------------------------------------------------------------------------------- phases (N > 1)
# A multi-rank run is a list of PHASES. Each phase is one measurement point run by a fresh worker
# process per rank (its own process group on its own port, its own RCCL communicator); the rank
# process the launcher started is a SUPERVISOR that never touches the GPU: it starts the phase's
# worker, enforces the phase's time limit, and agrees the phase's outcome with the other supervisors
# through the launcher's TCP store (no collective). A phase that raises, crashes or hangs on any rank
# -- including a hang inside a captured RCCL kernel, which no in-process watchdog can interrupt --
# ends in every rank's worker being stopped and becomes {"error": ...} in its block; the next phase
# starts from clean processes. The headline runs first and is kept; extras follow in order of risk
# (the never-before-run paths last) while the time budget lasts, and rank 0's supervisor always
# prints exactly one JSON line (unless the headline itself failed: then there is no measurement).
# The experiment being measured: /root/reference/src/Part 2a/main.py:148-175, Part 3/main.py:135-162.
def _phase_plan(args, world):
    strong_lb = max(1, args.global_batch // world)
    main_lb = args.local_batch if args.scaling == "weak" else strong_lb
    plan = [{"name": "headline", "lb": main_lb, "strategy": args.strategy, "sync": True, "full": True,
             "headline": True}]
    if args.no_extra:
        return plan
    def need(s):  # the headline already is the strong point of its own strategy under strong scaling
        return not (s == args.strategy and main_lb == strong_lb)

    plan.append({"name": "no_sync", "lb": main_lb, "strategy": args.strategy, "sync": False})
    if need("ddp"):  # the DDP strong point first (least risky: the headline's own path)
        plan.append({"name": "strong_ddp", "lb": strong_lb, "strategy": "ddp", "sync": True, "full": True})
    if main_lb != strong_lb:
        plan.append({"name": "strong_no_sync", "lb": strong_lb, "strategy": args.strategy, "sync": False})
    for s in ("allreduce_blocking", "bucketed_overlap"):
        if need(s):
            plan.append({"name": f"strong_{s}", "lb": strong_lb, "strategy": s, "sync": True, "full": True})
    if args.model == "vgg11" and os.environ.get("CDP_BENCH_RESNET", "1") != "0":
        cpu = args.device == "cpu"
        lb, size = (2, 32) if cpu else (64, 224)
        rn = dict(lb=lb, model="resnet50", strategy="ddp", image_size=size, steps=min(args.steps, 10), warmup=3)
        plan.append(dict(rn, name="resnet50_ddp", sync=True, full=True))
        plan.append(dict(rn, name="resnet50_no_sync", sync=False))
    if need("gather_scatter"):  # the grouped point-to-point path: never run with a peer before, last
        plan.append({"name": "strong_gather_scatter", "lb": strong_lb, "strategy": "gather_scatter", "sync": True,
                     "full": True})
    if args.extras != "all":
        keep = {"headline"} | {e.strip() for e in args.extras.split(",") if e.strip()}
        plan = [p for p in plan if p["name"] in keep]
    return plan


def _maybe_fault(run):
    """Test hook ``CDP_BENCH_FAULT=phase:rank:kind[,...]`` (kind = raise | hang | crash): make this
    rank's worker fail the named phase after its warm-up, i.e. while its peers are about to enter the
    timed region's collectives (how a real failure in a never-run path would meet them)."""
    spec = os.environ.get("CDP_BENCH_FAULT")
    phase = os.environ.get("CDP_BENCH_PHASE")
    if not spec or not phase:
        return
    rank = os.environ.get("RANK", "0")
    for item in spec.split(","):
        p, r, kind = item.split(":")
        if p != phase or r != rank:
            continue
        print(f"[bench] rank {rank}: injected fault '{kind}' in phase {phase}", file=sys.stderr, flush=True)
        if kind == "raise":
            raise RuntimeError(f"injected fault in phase {phase}")
        if kind == "hang":
            time.sleep(3600)
        if kind == "crash":
            import signal

            os.kill(os.getpid(), signal.SIGKILL)


def _write_json(path, obj):
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f)
    os.replace(tmp, path)


class _Ctx:
    """One rank's process-level state: device, process group, communicator kind."""

    def __init__(self, args, comm_timeout_s=300.0):
        import torch

        import cs744_distributed_data_parallel_amd as cdp
        from cs744_distributed_data_parallel_amd import distributed as dist

        self.torch, self.cdp, self.dist, self.args = torch, cdp, dist, args
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        world = self.world
        # native RCCL communicator unavailable on some rank -> all ranks agree to use torch's nccl (=RCCL)
        # process group instead of failing the run (distributed._init_native_rccl); "comm" in the JSON
        # says which one ran
        os.environ.setdefault("CDP_RCCL_FALLBACK", "1")
        self.cpu = args.device == "cpu"
        if self.cpu:
            self.dev = torch.device("cpu")
            torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "1")))
            if world > 1:
                dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            if args.dist_backend == "gloo":
                local = local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(local)
            self.dev = torch.device("cuda", local)
            if world > 1 and args.dist_backend == "gloo":
                dist.init_process_group("gloo", rank=rank, world_size=world)
            elif world > 1 or os.environ.get("CDP_BENCH_DDP_W1") == "1":
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                os.environ.setdefault("MASTER_PORT", "29561")
                # a collective that stalls past the phase's limit is aborted by the communicator's watchdog
                dist.init_process_group("rccl" if args.backend == "native" else "nccl", rank=rank, world_size=world,
                                        comm_timeout_s=comm_timeout_s)
            if args.backend == "native":
                cdp._native.lib()  # fail loudly if the HIP extension is missing
                if args.precision == "bf16":
                    cdp._native.lib().set_conv_gemm("bf16")

    def dbg(self, msg):
        if os.environ.get("CDP_BENCH_DEBUG"):
            print(f"[bench r{self.rank}] {msg}", file=sys.stderr, flush=True)

    def comm_kind(self):
        if self.world == 1:
            return "none"
        if self.dist.native_communicator() is not None:
            return "rccl-native"
        return "gloo" if (self.cpu or self.args.dist_backend == "gloo") else "torch-nccl"

    def point(self, spec):
        """Measure one phase spec; returns its data dict."""
        args = self.args
        kw = dict(sync_grads=spec["sync"], strategy=spec.get("strategy"), model_name=spec.get("model"))
        if "image_size" in spec:
            kw["image_size"] = spec["image_size"]
        res = _measure(args, self.world, self.rank, self.dev, spec["lb"], self.dbg, self.dist, steps=spec.get("steps"),
                       warmup=spec.get("warmup"), full=bool(spec.get("full")), **kw)
        out = {"ms": res[0], "hipgraph": res[1]}
        if spec.get("full"):
            out["replicas_identical"], out["buckets"] = res[2], res[3]
        return out

    def close(self):
        if self.dist.is_initialized():
            self.dist.destroy_process_group()


def worker_main(args) -> int:
    """One phase on one rank (started by that rank's supervisor): writes {"ok", "data" | "error"}."""
    import faulthandler

    spec = json.loads(os.environ["CDP_BENCH_SPEC"])
    out_path = os.environ["CDP_BENCH_RESULT"]
    limit = float(os.environ.get("CDP_BENCH_PHASE_LIMIT_S", "300"))
    faulthandler.enable()
    faulthandler.dump_traceback_later(limit + 30.0, exit=True)  # the supervisor kills us first
    _orphan_guard()
    rank = os.environ.get("RANK", "0")
    try:
        if spec.get("headline") and os.environ.get("CDP_BENCH_FAIL_RANK") == rank:  # launcher test hook
            raise SystemExit(f"[bench] rank {rank}: CDP_BENCH_FAIL_RANK")
        ctx = _Ctx(args, comm_timeout_s=limit)
        data = ctx.point(spec)
        if spec.get("headline"):
            data.update(ranks_seen=ctx.dist.ranks_seen() if ctx.world > 1 else 1, comm=ctx.comm_kind(),
                        comm_fallback_reason=ctx.dist.comm_fallback_reason() if ctx.world > 1 else None,
                        engine="reference" if ctx.cpu else _conv_gemm_engine(args.backend))
        data["graph_fallbacks"] = list(_GRAPH_FALLBACKS)
        data["graph_collectives"] = _LAST_GRAPH_COLLECTIVES[0]
        _write_json(out_path, {"ok": True, "data": data})
    except BaseException as e:  # noqa: BLE001 - every failure becomes the phase's error
        msg = f"{type(e).__name__}: {str(e)[:400]}"
        print(f"[bench] rank {rank} phase {spec['name']} failed: {msg}", file=sys.stderr, flush=True)
        _write_json(out_path, {"ok": False, "error": msg})
        return 1
    try:
        ctx.close()
    finally:
        faulthandler.cancel_dump_traceback_later()
    return 0


def _orphan_guard():
    """Die with the supervisor: a worker whose supervisor was killed must not hold the GPU."""
    ppid = int(os.environ.get("CDP_BENCH_SUPERVISOR_PID", "0"))
    if not ppid:
        return
    try:
        import ctypes
        import signal

        ctypes.CDLL(None).prctl(1, int(signal.SIGKILL))  # PR_SET_PDEATHSIG
    except Exception:  # pragma: no cover - non-Linux
        return
    if os.getppid() != ppid:  # the supervisor died before the guard was set
        os._exit(1)


def _supervisor_store(world, rank):
    import datetime

    import torch.distributed as tdist

    store, _, _ = next(tdist.rendezvous("env://", rank=rank, world_size=world,
                                        timeout=datetime.timedelta(seconds=600)))
    return tdist.PrefixStore("cdp_bench_sup", store)


def supervise(args) -> int:
    """The rank process of a multi-rank run (see the phase notes above)."""
    import signal
    import tempfile

    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    if world != args.gpus:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    store = _supervisor_store(world, rank)
    plan = _phase_plan(args, world)
    head_limit = float(os.environ.get("CDP_BENCH_HEADLINE_LIMIT_S", "300"))
    extra_limit = float(os.environ.get("CDP_BENCH_PHASE_LIMIT_S", "90"))
    budget = float(os.environ.get("CDP_BENCH_BUDGET_S", "500"))
    grace = float(os.environ.get("CDP_BENCH_PEER_GRACE_S", "5"))
    tmp = tempfile.mkdtemp(prefix=f"cdp_bench_r{rank}_")
    child = {"p": None}

    def _stop(p):
        if p is None or p.poll() is not None:
            return
        try:
            os.killpg(p.pid, signal.SIGTERM)
            p.wait(timeout=10)
        except (subprocess.TimeoutExpired, ProcessLookupError, PermissionError):
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
            p.wait()

    def _on_term(signum, frame):  # the launcher stops us: take the worker down too
        _stop(child["p"])
        os._exit(128 + signum)

    signal.signal(signal.SIGTERM, _on_term)
    t_start = time.monotonic()
    results, phases = {}, []
    for i, spec in enumerate(plan):
        name, limit = spec["name"], (head_limit if i == 0 else extra_limit)
        # rank 0 decides whether the phase runs (time budget) and on which port; everyone follows
        if rank == 0:
            go = str(_free_port())
            if i > 0 and time.monotonic() - t_start + limit > budget:
                go = f"skipped: time budget ({budget:.0f} s) spent"
            store.set(f"{i}/go", go)
        store.wait([f"{i}/go"])
        go = store.get(f"{i}/go").decode()
        if not go.isdigit():
            results[name] = {"ok": False, "error": go}
            phases.append({"name": name, "status": go})
            continue
        res_path = os.path.join(tmp, f"{name}.json")
        env = dict(os.environ)
        env.update(CDP_BENCH_WORKER="1", CDP_BENCH_PHASE=name, CDP_BENCH_SPEC=json.dumps(spec),
                   CDP_BENCH_RESULT=res_path, CDP_BENCH_PHASE_LIMIT_S=str(limit), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=go, TORCHELASTIC_USE_AGENT_STORE="False", CDP_BENCH_SUPERVISOR_PID=str(os.getpid()))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        t0 = time.monotonic()
        p = subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                             stdout=sys.stderr.fileno(), start_new_session=True)
        child["p"] = p
        reason, peer_t = None, None
        fail_key = f"{i}/failed"
        while p.poll() is None:
            if time.monotonic() - t0 > limit:
                reason = f"timeout: no result within {limit:.0f} s"
                break
            if peer_t is None and store.check([fail_key]):
                peer_t = time.monotonic()
            if peer_t is not None and time.monotonic() - peer_t > grace:
                reason = "stopped: " + store.get(fail_key).decode()
                break
            time.sleep(0.05)
        _stop(p)
        child["p"] = None
        got = None
        if os.path.exists(res_path):
            with open(res_path) as f:
                got = json.load(f)
        if got is not None and got.get("ok"):
            st = "ok"  # (a worker killed after writing its result, e.g. stuck in teardown, still measured)
        else:
            st = (got or {}).get("error") or reason or f"worker exited with {p.returncode}"
            if not st.startswith("stopped:"):
                store.set(fail_key, f"rank {rank}: {st}")
        store.set(f"{i}/st/{rank}", st)
        keys = [f"{i}/st/{r}" for r in range(world)]
        import datetime

        try:
            store.wait(keys, datetime.timedelta(seconds=limit + 120.0))
        except Exception:  # noqa: BLE001 - a supervisor that never reports counts as failed
            pass
        sts = [store.get(k).decode() if store.check([k]) else "no status from this rank's supervisor" for k in keys]
        bad = [(r, s) for r, s in enumerate(sts) if s != "ok"]
        if bad:
            # every rank's own failure (ranks stopped because of a peer's are implied by it)
            own = [(r, s) for r, s in bad if not s.startswith("stopped:")] or bad
            err = " | ".join(f"rank {r}: {s}" for r, s in own)
            results[name] = {"ok": False, "error": err}
            phases.append({"name": name, "status": "error", "error": err, "seconds": round(time.monotonic() - t0, 1)})
            print(f"[bench] phase {name} failed ({err})", file=sys.stderr, flush=True)
        else:
            results[name] = got
            phases.append({"name": name, "status": "ok", "seconds": round(time.monotonic() - t0, 1)})
        if i == 0 and bad:
            break  # no headline, no record
    rc = 0
    head = results.get("headline") or {"ok": False, "error": "not run"}
    if not head.get("ok"):
        print(f"[bench] rank {rank}: the headline measurement failed ({head.get('error')}); no record",
              file=sys.stderr)
        rc = 1
    elif rank == 0:
        rec = _assemble_multi(args, world, plan, results, phases)
        print(json.dumps(rec), flush=True)
    if head.get("ok") and head["data"].get("replicas_identical") is False:
        print(f"[bench] rank {rank}: replicas diverged after the timed steps", file=sys.stderr)
        rc = 3
    # the phases' outcome is agreed; leave together (rank 0 may host the store)
    store.set(f"done/{rank}", "1")
    try:
        import datetime

        store.wait([f"done/{r}" for r in range(world)], datetime.timedelta(seconds=60))
    except Exception:  # noqa: BLE001
        pass
    return rc


def _assemble_multi(args, world, plan, results, phases):
    """Rank 0's record of a multi-rank run from the phases' results (failed extras become errors)."""
    head = results["headline"]["data"]
    strong_lb = max(1, args.global_batch // world)
    main_lb = args.local_batch if args.scaling == "weak" else strong_lb
    ms = head["ms"]

    def get(name):
        r = results.get(name)
        if r is None:
            return None, None
        return (r["data"], None) if r.get("ok") else (None, r.get("error"))

    extra = {}
    if head.get("buckets") is not None:
        extra["buckets"] = head["buckets"]
    fallbacks = list(head.get("graph_fallbacks", []))
    if not args.no_extra:
        ns, ns_err = get("no_sync")
        if ns is not None:
            extra["ms_per_step_no_sync"] = round(ns["ms"], 4)
            extra["exposed_comm_ms"] = round(max(0.0, ms - ns["ms"]), 4)
        elif ns_err:
            extra["no_sync"] = {"error": ns_err}
        # the reference's whole multi-process experiment: its four sync strategies at its own
        # strong-scaling rule (global batch 256 split int(256 / W) per rank)
        blk = {"local_batch": strong_lb, "global_batch": strong_lb * world}
        s0, s0_err = get("strong_no_sync" if main_lb != strong_lb else "no_sync")
        blk["no_sync"] = ({"ms_per_step": round(s0["ms"], 4), "value": round(strong_lb * world / s0["ms"] * 1e3, 1),
                           "hipgraph": s0["hipgraph"]} if s0 is not None else {"error": s0_err or "not run"})
        for strat in STRATEGY_REF:
            if strat == args.strategy and main_lb == strong_lb:
                d, err = head, None
            else:
                d, err = get(f"strong_{strat}")
            if d is None:
                if err is not None or f"strong_{strat}" in {p["name"] for p in plan}:
                    blk[strat] = {"reference": STRATEGY_REF[strat], "error": err or "not run"}
                continue
            if d is not head:
                fallbacks += d.get("graph_fallbacks", [])
            ent = {"reference": STRATEGY_REF[strat], "ms_per_step": round(d["ms"], 4),
                   "value": round(strong_lb * world / d["ms"] * 1e3, 1), "replicas_identical": d.get("replicas_identical"),
                   "hipgraph": d["hipgraph"]}
            if s0 is not None:
                ent["exposed_sync_ms"] = round(max(0.0, d["ms"] - s0["ms"]), 4)
                ent["scaling_eff"] = round(min(1.0, s0["ms"] / d["ms"]), 4)
            if d.get("buckets") is not None:
                ent["buckets"] = d["buckets"]
            blk[strat] = ent
        extra["strategies"] = blk
        eff = {}
        if ns is not None:
            eff[args.scaling] = round(min(1.0, ns["ms"] / ms), 4)
        d = blk.get(args.strategy, {})
        if args.scaling == "weak" and "ms_per_step" in d:
            extra["strong"] = {"value": d["value"], "ms_per_step": d["ms_per_step"], "global_batch": strong_lb * world,
                               "local_batch": strong_lb, "strategy": args.strategy}
            if "scaling_eff" in d:
                eff["strong"] = d["scaling_eff"]
        elif args.scaling == "weak" and "error" in d:
            extra["strong"] = {"error": d["error"]}
        # ms/step without gradient sync over ms/step with it (1.0 = communication fully hidden); the
        # driver computes the across-N scaling efficiency from the per-N values itself
        extra["scaling_eff"] = eff
        names = {p["name"] for p in plan}
        if "resnet50_ddp" in names:
            rd, rerr = get("resnet50_ddp")
            rn0, rn0_err = get("resnet50_no_sync")
            cpu = args.device == "cpu"
            lb, size = (2, 32) if cpu else (64, 224)
            rn = {"local_batch": lb, "global_batch": lb * world, "image_shape": [3, size, size], "strategy": "ddp",
                  "unit": "images/sec", "conv_gemm": head.get("engine")}
            if rd is not None:
                rn.update(ms_per_step=round(rd["ms"], 4), value=round(lb * world / rd["ms"] * 1e3, 1),
                          replicas_identical=rd.get("replicas_identical"), hipgraph=rd["hipgraph"])
                if rd.get("buckets") is not None:
                    rn["buckets"] = rd["buckets"]
                fallbacks += rd.get("graph_fallbacks", [])
            else:
                rn["error"] = rerr or "not run"
            if rn0 is not None:
                rn["ms_per_step_no_sync"] = round(rn0["ms"], 4)
                if rd is not None:
                    rn["exposed_comm_ms"] = round(max(0.0, rd["ms"] - rn0["ms"]), 4)
                    rn["scaling_eff"] = round(min(1.0, rn0["ms"] / rd["ms"]), 4)
            elif rn0_err:
                rn["no_sync_error"] = rn0_err
            extra["resnet50"] = rn
        for nm in ("no_sync", "strong_no_sync", "resnet50_no_sync"):
            d2, _ = get(nm)
            if d2 is not None:
                fallbacks += d2.get("graph_fallbacks", [])
    extra["phases"] = phases
    return _record(args, world, main_lb, ms, head, fallbacks, extra)


def _record(args, world, main_lb, ms, head, fallbacks, extra):
    cpu = args.device == "cpu"
    engine = head.get("engine") or ("reference" if cpu else _conv_gemm_engine(args.backend))
    hipgraph = head["hipgraph"]
    global_batch = main_lb * world
    img_s = global_batch / ms * 1e3
    imagenet = args.model.startswith("resnet")
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
        # fp32 operands, fp32 accumulation. The conv GEMM engine is named in config.conv_gemm and its
        # numerics (with the one documented limit of the f16x2 split) in "numerics" below.
        "dtype": _dtype_label(args.precision, engine),
        "numerics": _numerics_note(args.precision, engine),
        "data": ("synthetic (random uint8 ImageNet-shaped 224x224x3, GPU-resident, on-GPU flip/normalize); "
                 if imagenet else
                 "synthetic (random uint8 CIFAR-10-shaped 32x32x3, GPU-resident, on-GPU crop/flip/normalize); ")
                + "random-init weights",
        "ranks_seen": head.get("ranks_seen", 1),
        "replicas_identical": head.get("replicas_identical"),
        "config": {
            "model": {"vgg11": "VGG-11", "resnet50": "ResNet-50"}.get(args.model, args.model),
            "global_batch": global_batch,
            "local_batch": main_lb,
            "seq_len": None,
            "image_shape": [3, 224, 224] if imagenet else [3, 32, 32],
            "parallelism": f"dp{world}",
            "strategy": args.strategy if world > 1 else "single",
            "comm": head.get("comm", "none"),
            "comm_fallback_reason": head.get("comm_fallback_reason"),
            "graph_fallbacks": fallbacks,
            # native-communicator collectives recorded inside the captured step (replayed every
            # step); null when the step is not captured or collectives go through torch
            "graph_collectives": head.get("graph_collectives") if hipgraph else None,
            "backend": args.backend,
            "device": "cpu" if cpu else "mi355x",
            "hipgraph": hipgraph,
            "optimizer": "SGD(lr=0.1, momentum=0.9, wd=1e-4)",
            # the step split per gradient bucket and run behind each bucket's all-reduce (--overlap-step)
            "optimizer_overlap": bool(args.overlap_step) and args.strategy == "ddp" and (world > 1 or os.environ.get("CDP_BENCH_DDP_W1") == "1"),
            "early_buffer_broadcast": bool(args.early_bcast) and args.strategy == "ddp" and not cpu and (world > 1 or os.environ.get("CDP_BENCH_DDP_W1") == "1"),
            # conv GEMM numerics, all with fp32 operands and fp32 accumulation: "f16x2" =
            # power-of-two-scaled operands split into two fp16 terms, three products on the
            # fp16 MFMA; "x3" = 3-term bf16 split, six products on the bf16 MFMA; "f32" =
            # exact fp32-input MFMA (docs/PERF.md, tests/test_kernels_gpu.py)
            "conv_gemm": engine,
        },
    }
    rec.update(extra)
    return rec


def single_main(args) -> int:
    """N = 1: the headline in this process, then every secondary point, each isolated by try/except
    (no collective can strand a peer at one rank): a failing extra becomes {"error": ...}."""
    import faulthandler

    faulthandler.enable()
    # hang guard: a stuck kernel ends the process (with every thread's traceback) instead of holding the box
    faulthandler.dump_traceback_later(float(os.environ.get("CDP_BENCH_TIMEOUT_S", "1200")), exit=True)
    if os.environ.get("CDP_BENCH_FAIL_RANK") == "0":
        raise SystemExit("[bench] rank 0: CDP_BENCH_FAIL_RANK")
    ctx = _Ctx(args)
    cdp, dist, dev, dbg = ctx.cdp, ctx.dist, ctx.dev, ctx.dbg
    main_lb = args.local_batch if args.scaling == "weak" else max(1, args.global_batch)
    os.environ["CDP_BENCH_PHASE"] = "headline"
    head = ctx.point({"lb": main_lb, "sync": True, "full": True, "strategy": args.strategy})
    if args.backend == "native" and not ctx.cpu:
        _dump_gemm_log(cdp)
    head.update(ranks_seen=1, comm="none", engine="reference" if ctx.cpu else _conv_gemm_engine(args.backend),
                graph_collectives=_LAST_GRAPH_COLLECTIVES[0])
    ms = head["ms"]
    engine = head["engine"]
    extra = {}
    if head.get("buckets") is not None:
        extra["buckets"] = head["buckets"]
    full = not args.no_extra and not ctx.cpu and args.backend == "native" and args.precision == "fp32" \
        and args.model == "vgg11"

    def guarded(key, fn):
        os.environ["CDP_BENCH_PHASE"] = key
        try:
            extra[key] = fn()
        except Exception as e:  # noqa: BLE001 - recorded, the headline stands
            print(f"[bench] extra {key} failed: {e!r}", file=sys.stderr, flush=True)
            extra[key] = {"error": f"{type(e).__name__}: {str(e)[:400]}"}
            try:
                cdp._native.lib().clear_hip_error()
                ctx.torch.cuda.synchronize()
            except Exception:  # noqa: BLE001
                pass

    if full and engine == "f16x2":
        # the same step on the strict engine (3-term bf16 split: every conv GEMM output within the
        # fp32 per-element error bound with no range limit, tests/test_accuracy_gpu.py)
        def _x3():
            C = cdp._native.lib()
            C.set_conv_gemm("x3")
            try:
                ms_x3, _ = _measure(args, 1, 0, dev, main_lb, dbg, dist)
            finally:
                C.set_conv_gemm(engine)
            return {"conv_gemm": "x3", "value": round(main_lb / ms_x3 * 1e3, 1), "ms_per_step": round(ms_x3, 4)}

        guarded("strict_fp32", _x3)
    if full and args.local_batch == REF_GLOBAL_BATCH:
        # the reference's strong-scaling rule (int(256 / W) images per rank,
        # /root/reference/src/Part 2a/main.py:22): the per-GPU step of its W = 2 / 4 / 8 points,
        # measured here on one GPU (no gradient sync: what the W-rank run costs before communication)
        def _strong():
            pts = []
            for w_ref in (2, 4, 8):
                lb = REF_GLOBAL_BATCH // w_ref
                ms_s, hg = _measure(args, 1, 0, dev, lb, dbg, dist, steps=max(args.steps, 20))
                pts.append({"reference_world_size": w_ref, "local_batch": lb, "ms_per_step": round(ms_s, 4),
                            "img_s_per_gpu": round(lb / ms_s * 1e3, 1), "hipgraph": hg})
            return pts

        guarded("per_gpu_strong", _strong)

        # BASELINE.json config #5 (ResNet-50, ImageNet-shaped, 64 images per GPU), one GPU
        def _resnet():
            ms_r, hg = _measure(args, 1, 0, dev, 64, dbg, dist, steps=min(args.steps, 10), warmup=3,
                                model_name="resnet50")
            return {"local_batch": 64, "image_shape": [3, 224, 224], "ms_per_step": round(ms_r, 3),
                    "value": round(64 / ms_r * 1e3, 1), "unit": "images/sec", "hipgraph": hg, "conv_gemm": engine}

        guarded("resnet50", _resnet)
    rec = _record(args, 1, main_lb, ms, head, list(_GRAPH_FALLBACKS), extra)
    print(json.dumps(rec), flush=True)
    ctx.close()
    faulthandler.cancel_dump_traceback_later()
    return 0


def _dtype_label(precision, engine):
    return "fp32" if precision == "fp32" else "bf16"


def _numerics_note(precision, engine):
    if precision != "fp32":
        return "bf16 conv GEMM operands, fp32 accumulation (non-parity fast mode)"
    if engine == "f16x2":
        return ("fp32 per-element error bound met on Gaussian, heavy-tailed, whole-image and whole-channel "
                "dynamic range (per-row power-of-two scales); limit: more than ~2^17 of dynamic range inside "
                "ONE image row exceeds it (tests/test_accuracy_gpu.py::test_f16x2_intra_image_range_limit)")
    if engine == "x3":
        return "fp32 per-element error bound, no range limit (3-term bf16 split)"
    if engine == "f32":
        return "exact fp32-input MFMA"
    return "fp32 (reference ops)"


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
    if os.environ.get("CDP_BENCH_WORKER") == "1":
        return worker_main(args)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return supervise(args)
    return single_main(args)


if __name__ == "__main__":
    sys.exit(main())
