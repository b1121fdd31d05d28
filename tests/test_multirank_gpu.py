"""Multi-process training on the GPU: two ranks share the test box's one MI355X.

RCCL refuses two ranks on one device ("Duplicate GPU detected"), so the ranks talk over gloo with
device tensors. Everything else is the production multi-GPU path: the native HIP kernels, the
C++ reducer's autograd hooks and bucket launches on real streams, DDP's construction broadcast
and per-forward buffer sync, and the four sync strategies of the reference
(``/root/reference/src/Part 2a/main.py:117-127``, ``src/Part 2b/main.py:116-119``,
``src/Part 3/main.py:61``). The SURVEY.md §4 oracle applies: all strategies end at the same
parameters, and both ranks agree.
"""
import numpy as np
import pytest
import torch

from _dist_util import run_ranks

pytestmark = pytest.mark.gpu


def _batch(rank, step, B=16):
    g = torch.Generator().manual_seed(1000 * step + rank)
    return torch.randn(B, 3, 32, 32, generator=g), torch.randint(0, 10, (B,), generator=g)


def _train_gpu(rank, world, strategy, steps=3):
    import cs744_distributed_data_parallel_amd as cdp
    from cs744_distributed_data_parallel_amd import _native
    from cs744_distributed_data_parallel_amd.parallel import (
        BucketedOverlap,
        DistributedDataParallel,
        average_gradients_allreduce,
        average_gradients_gather_scatter,
    )

    _native.lib()  # the HIP path, not a fallback
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    cdp.utils.seed_everything(0)
    model = cdp.VGG11().to(dev)
    sync = None
    if strategy == "ddp":
        model = DistributedDataParallel(model, bucket_cap_mb=4.0)
    elif strategy == "bucketed_overlap":
        sync = BucketedOverlap(model, bucket_cap_mb=4.0)
    opt = cdp.SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    crit = cdp.CrossEntropyLoss()
    losses = []
    m = getattr(model, "module", model)
    flat1 = None
    for step in range(steps):
        x, y = _batch(rank, step)
        x = x.to(dev).contiguous(memory_format=torch.channels_last)
        y = y.to(dev)
        opt.zero_grad()
        out = model(x)
        if sync is not None:
            sync.prepare(out)
        loss = crit(out, y)
        loss.backward()
        if strategy == "gather_scatter":
            average_gradients_gather_scatter(model, rank)
        elif strategy == "allreduce_blocking":
            average_gradients_allreduce(model)
        opt.step()
        losses.append(float(loss))
        if step == 0:
            torch.cuda.synchronize()
            flat1 = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy()
    torch.cuda.synchronize()
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy()
    info = model._get_ddp_logging_data() if strategy == "ddp" else {}
    return (flat1, flat), losses, info


def test_two_ranks_on_one_gpu_strategy_equivalence():
    outs = {s: run_ranks(_train_gpu, 2, (s,), timeout=300)
            for s in ["allreduce_blocking", "gather_scatter", "bucketed_overlap", "ddp"]}
    (ref1, ref_flat), ref_losses, _ = outs["allreduce_blocking"][0]
    for s, per_rank in outs.items():
        ((a1, f0), l0, _), ((b1, f1), l1, _) = per_rank
        # the DDP invariant: both ranks hold bit-identical parameters after every step
        np.testing.assert_array_equal(a1, b1, err_msg=f"{s}: ranks diverged after step 1")
        np.testing.assert_array_equal(f0, f1, err_msg=f"{s}: ranks diverged after step 3")
        # strategies average in different orders (per-tensor SUM then /W, bucketed ncclAvg-style,
        # gather + stack_mean), so their gradients may differ in the last ulp; after ONE step that
        # is at most lr * ulp(grad) per parameter: tight elementwise agreement
        np.testing.assert_allclose(a1, ref1, rtol=0, atol=2e-5, err_msg=f"{s} != allreduce_blocking after step 1")
        # after three steps such 1-ulp differences pass through ReLU masks and max-pool argmaxes; the
        # model-level check is a relative L2 norm, the losses must agree tightly
        rel = float(np.linalg.norm(f0 - ref_flat) / np.linalg.norm(ref_flat))
        assert rel < 1e-5, (s, rel)
        np.testing.assert_allclose(l0, ref_losses, rtol=1e-4, err_msg=f"{s} losses")
    info = outs["ddp"][0][2]
    assert info["native_reducer"], info
    assert info["rebuilt_buckets"], info


def test_capture_failure_on_one_rank_makes_every_rank_eager():
    """Two ranks on the one GPU (gloo): in the collective-free no-sync step that bench.py also times,
    rank 1's hipGraph capture is broken on purpose (CDP_BENCH_BREAK_CAPTURE=1), rank 0's succeeds.
    The ranks agree BEFORE any replay, so both time eager steps, nobody replays a graph the other
    cannot match, and the run finishes with one record and identical replicas."""
    import json
    import os
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=repo, CDP_BENCH_BREAK_CAPTURE="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--strategy", "allreduce_blocking", "--steps", "2", "--warmup", "1", "--local-batch", "8",
                        "--dataset-size", "64", "--extras", "no_sync,strong_no_sync"],
                       env=env, capture_output=True, text=True, timeout=240, cwd=repo)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "hipGraph capture failed" in r.stderr, r.stderr[-3000:]
    assert "another rank could not capture; all ranks time eager steps" in r.stderr, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["replicas_identical"] is True and rec["ranks_seen"] == 2
    # the record names the measurement that fell back (rank 0 captured, its peer did not)
    fb = rec["config"]["graph_fallbacks"]
    assert fb and all(f["reason"] == "another rank could not capture" for f in fb), fb
    assert {f["sync_grads"] for f in fb} == {False}, fb
