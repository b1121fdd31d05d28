"""Multi-process (gloo, world 2/4) tests: collectives, the four sync strategies, reducer and DDP.

The strategy-equivalence test is the SURVEY.md §4 oracle: with identical seeds, Part 2a
(gather/scatter), Part 2b (blocking all-reduce), the hook-bucketed reducer, our DDP wrapper and
torch's own DDP all produce the same parameters after k SGD steps.
"""
import os

import numpy as np
import pytest
import torch

from _dist_util import run_ranks


# ----------------------------------------------------------------------------- workers
def _collectives(rank, world):
    from cs744_distributed_data_parallel_amd import distributed as dist

    t = torch.full((5,), float(rank + 1))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    s = float(t[0])
    t = torch.full((3,), float(rank + 1))
    dist.all_reduce(t, op=dist.reduce_op.MAX)  # deprecated alias used by the reference
    mx = float(t[0])
    b = torch.full((4,), float(rank))
    dist.broadcast(b, src=world - 1)
    g = torch.full((2,), float(rank * 10))
    outs = [torch.empty(2) for _ in range(world)] if rank == 0 else None
    dist.gather(g, outs, dst=0)
    gathered = [float(o[0]) for o in outs] if rank == 0 else None
    sc = torch.empty(3)
    ins = [torch.full((3,), float(100 + r)) for r in range(world)] if rank == 0 else None
    dist.scatter(sc, ins, src=0)
    lst = [torch.empty(2) for _ in range(world)]
    dist.all_gather(lst, torch.full((2,), float(rank)))
    avg = torch.full((2,), float(rank))
    dist.communicator_for(avg).all_reduce(avg, "avg")
    dist.barrier()
    return dict(s=s, mx=mx, b=float(b[0]), gathered=gathered, sc=float(sc[0]),
                ag=[float(x[0]) for x in lst], avg=float(avg[0]), world=dist.get_world_size(), rank=dist.get_rank())


def _make_batch(rank, step, B=8):
    g = torch.Generator().manual_seed(1000 * step + rank)
    return torch.randn(B, 3, 32, 32, generator=g), torch.randint(0, 10, (B,), generator=g)


def _train(rank, world, strategy, steps=3):
    import cs744_distributed_data_parallel_amd as cdp
    from cs744_distributed_data_parallel_amd.parallel import (
        BucketedOverlap,
        DistributedDataParallel,
        average_gradients_allreduce,
        average_gradients_gather_scatter,
    )

    cdp.utils.seed_everything(0)
    model = cdp.VGG11(channels_last=False)
    sync = None
    if strategy == "ddp":
        model = DistributedDataParallel(model, bucket_cap_mb=4.0)
    elif strategy == "torch_ddp":
        model = torch.nn.parallel.DistributedDataParallel(model)
    elif strategy == "bucketed_overlap":
        sync = BucketedOverlap(model, bucket_cap_mb=4.0)
    if strategy == "torch_ddp":
        opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    else:
        opt = cdp.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    crit = cdp.CrossEntropyLoss()
    losses = []
    for step in range(steps):
        x, y = _make_batch(rank, step)
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
    m = getattr(model, "module", model)
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).numpy()
    bufs = torch.cat([b.detach().float().reshape(-1) for b in m.buffers()]).numpy()
    info = {}
    if strategy == "ddp":
        info = model._get_ddp_logging_data()
    return flat, bufs, losses, info


def _reducer_unused(rank, world, find_unused):
    import cs744_distributed_data_parallel_amd as cdp

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Linear(4, 4)
            self.b = torch.nn.Linear(4, 4)  # unused in forward

        def forward(self, x):
            return self.a(x)

    torch.manual_seed(0)
    net = cdp.DistributedDataParallel(Net(), find_unused_parameters=find_unused)
    err = None
    try:
        for _ in range(2):
            out = net(torch.randn(2, 4))
            out.sum().backward()
    except RuntimeError as e:
        err = str(e)
    return err, float(net.module.a.weight.grad.abs().sum()) if net.module.a.weight.grad is not None else None


def _unused_output_head(rank, world, py_reducer=False):
    """find_unused_parameters with an output that stays out of the loss (its parameters are reached
    from the outputs, so only the end-of-backward callback can mark them), in the first -- timed,
    launch-deferred -- iteration of the default bucket planner."""
    import copy

    import cs744_distributed_data_parallel_amd as cdp

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Linear(4, 4)
            self.b = torch.nn.Linear(4, 4)

        def forward(self, x):
            return self.a(x), self.b(x)

    if py_reducer:
        os.environ["CDP_PY_REDUCER"] = "1"
    torch.manual_seed(0)
    module = Net()
    ref = copy.deepcopy(module)
    net = cdp.DistributedDataParallel(module, find_unused_parameters=True)
    x = torch.randn(3, 4, generator=torch.Generator().manual_seed(100 + rank))
    out_a, _ = net(x)
    out_a.pow(2).sum().backward()
    ref(x)[0].pow(2).sum().backward()
    return (net.module.a.weight.grad.clone().numpy(), ref.a.weight.grad.clone().numpy(), net.reducer.iterations,
            net.reducer.native)


def _no_sync(rank, world):
    import cs744_distributed_data_parallel_amd as cdp

    torch.manual_seed(0)
    net = cdp.DistributedDataParallel(torch.nn.Linear(3, 2, bias=False))
    x = torch.full((1, 3), float(rank + 1))
    with net.no_sync():
        net(x).sum().backward()
    local = net.module.weight.grad.clone()
    net(x).sum().backward()  # synced: accumulated local grads (2x) averaged across ranks
    return local.numpy(), net.module.weight.grad.numpy()


def _buffers_broadcast(rank, world):
    import cs744_distributed_data_parallel_amd as cdp

    torch.manual_seed(rank)  # different init per rank: DDP must broadcast rank 0's state
    m = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 3), torch.nn.BatchNorm2d(4))
    with torch.no_grad():
        m[1].running_mean.fill_(float(rank))
    net = cdp.DistributedDataParallel(m)
    w0 = m[0].weight.detach().clone().numpy()
    rm0 = m[1].running_mean.clone().numpy()
    net(torch.randn(2, 3, 8, 8))
    # per-forward sync: rank 1 drifts its fp32 and int64 buffers, the next forward restores
    # rank 0's (both dtypes travel in one byte broadcast, see utils/arena.py BufferArena)
    with torch.no_grad():
        if rank == 1:
            m[1].running_var.fill_(7.0)
            m[1].num_batches_tracked.fill_(100)
    net(torch.randn(2, 3, 8, 8, generator=torch.Generator().manual_seed(0)))  # same batch on both
    extra = (m[1].running_var.clone().numpy(), int(m[1].num_batches_tracked))
    return w0, rm0, net.state_dict().keys().__iter__().__next__(), extra


def _rebuild_ready_order(rank, world):
    import cs744_distributed_data_parallel_amd as cdp

    cdp.utils.seed_everything(0)
    model = cdp.VGG11(channels_last=False)
    net = cdp.DistributedDataParallel(model, bucket_cap_mb=8.0)
    before = net.bucket_sizes_bytes()
    crit = cdp.CrossEntropyLoss()
    for step in range(2):
        x, y = _make_batch(rank, step, B=4)
        net.zero_grad(set_to_none=True)
        crit(net(x), y).backward()
    after = net.bucket_sizes_bytes()
    return before, after, net._get_ddp_logging_data()["rebuilt_buckets"]


# ----------------------------------------------------------------------------- tests
@pytest.mark.parametrize("world", [2, 4])
def test_collectives(world):
    res = run_ranks(_collectives, world)
    tot = sum(range(1, world + 1))
    for r, d in enumerate(res):
        assert d["s"] == tot
        assert d["mx"] == world
        assert d["b"] == world - 1
        assert d["sc"] == 100 + r
        assert d["ag"] == [float(i) for i in range(world)]
        assert abs(d["avg"] - (world - 1) / 2) < 1e-6
        assert d["world"] == world and d["rank"] == r
    assert res[0]["gathered"] == [10.0 * i for i in range(world)]


def test_strategy_equivalence_oracle():
    """Parts 2a / 2b / bucketed / DDP / torch-DDP agree after 3 steps (SURVEY.md §4 oracle 1)."""
    outs = {s: run_ranks(_train, 2, (s,)) for s in
            ["gather_scatter", "allreduce_blocking", "bucketed_overlap", "ddp", "torch_ddp"]}
    ref_flat, _, ref_losses, _ = outs["torch_ddp"][0]
    for s, per_rank in outs.items():
        f0, _, l0, _ = per_rank[0]
        f1, _, l1, _ = per_rank[1]
        np.testing.assert_allclose(f0, f1, rtol=0, atol=1e-6, err_msg=f"{s}: ranks diverged")
        np.testing.assert_allclose(f0, ref_flat, rtol=1e-4, atol=1e-5, err_msg=f"{s} != torch DDP")
        np.testing.assert_allclose(l0, ref_losses, rtol=1e-4, err_msg=f"{s} losses")


def test_ddp_uses_native_reducer_and_buckets():
    res = run_ranks(_train, 2, ("ddp", 2))
    info = res[0][3]
    import cs744_distributed_data_parallel_amd as cdp

    assert info["native_reducer"] == cdp.native_available()
    assert info["num_buckets"] >= 3
    assert sum(info["bucket_sizes"]) >= 9231114 * 4


def test_unused_parameters_error_and_find_unused():
    errs = run_ranks(_reducer_unused, 2, (False,))
    assert errs[0][0] is not None and "did not receive gradients" in errs[0][0]
    ok = run_ranks(_reducer_unused, 2, (True,))
    assert ok[0][0] is None and ok[0][1] > 0


@pytest.mark.parametrize("py_reducer", [False, True])
def test_find_unused_with_an_output_left_out_of_the_loss(py_reducer):
    """Every bucket is all-reduced when an output's parameters get no gradient: the
    synced gradient equals the mean of the ranks' local gradients on both ranks, with the C++
    reducer and with its Python twin."""
    import cs744_distributed_data_parallel_amd as cdp

    (g0, l0, it0, nat), (g1, l1, it1, _) = run_ranks(_unused_output_head, 2, (py_reducer,))
    assert nat == (cdp.native_available() and not py_reducer)
    assert not np.allclose(l0, l1)
    np.testing.assert_allclose(g0, g1, rtol=0, atol=1e-7)
    np.testing.assert_allclose(g0, (l0 + l1) / 2, rtol=1e-6, atol=1e-7)
    assert it0 == it1 == 1


def test_no_sync_accumulates_locally():
    res = run_ranks(_no_sync, 2)
    (l0, g0), (l1, g1) = res
    assert not np.allclose(l0, l1)  # local grads differ across ranks
    np.testing.assert_allclose(g0, g1, atol=1e-6)
    np.testing.assert_allclose(g0, (2 * l0 + 2 * l1) / 2, atol=1e-5)


def test_ddp_broadcasts_rank0_state():
    res = run_ranks(_buffers_broadcast, 2)
    np.testing.assert_allclose(res[0][0], res[1][0])
    np.testing.assert_allclose(res[1][1], 0.0)  # rank 1's running_mean replaced by rank 0's
    assert res[0][2].startswith("module.")
    np.testing.assert_allclose(res[0][3][0], res[1][3][0])
    assert res[0][3][1] == res[1][3][1] == 2


def test_bucket_rebuild_in_ready_order():
    res = run_ranks(_rebuild_ready_order, 2)
    before, after, rebuilt = res[0]
    assert rebuilt
    assert sum(before) == sum(after)
    assert res[0][1] == res[1][1]  # identical plan on all ranks


def _dead_peer(rank, world):
    import time

    from cs744_distributed_data_parallel_amd import distributed as dist

    if rank == 1:
        time.sleep(6)  # never enters the collective within the group timeout
        return ("slept", 0.0)
    t0 = time.time()
    try:
        dist.all_reduce(torch.ones(4))
    except Exception:  # failure detection: the collective times out instead of hanging
        return ("raised", time.time() - t0)
    return ("completed", time.time() - t0)


def test_dead_peer_is_detected_by_timeout():
    import datetime

    res = run_ranks(_dead_peer, 2, init_kwargs={"timeout": datetime.timedelta(seconds=2)}, timeout=120)
    status, dt = res[0]
    assert status == "raised", res
    assert dt < 6.0, res


# ----------------------------------------------------------------------------- overlap
def _overlap_trace(rank, world, strategy):
    import cs744_distributed_data_parallel_amd as cdp
    from cs744_distributed_data_parallel_amd.parallel import BucketedOverlap, DistributedDataParallel

    cdp.utils.seed_everything(0)
    model = cdp.VGG11(channels_last=False)
    sync = None
    if strategy == "ddp":
        model = DistributedDataParallel(model, bucket_cap_mb=2.0)
        reducer = model.reducer
    else:
        sync = BucketedOverlap(model, bucket_cap_mb=2.0)
        reducer = sync.reducer
    crit = cdp.CrossEntropyLoss()
    logs = []
    for step in range(3):  # step 0 records the ready order, step 1 runs on the rebuilt buckets
        reducer.set_trace(True)
        x, y = _make_batch(rank, step, B=4)
        out = model(x)
        if sync is not None:
            sync.prepare(out)
        crit(out, y).backward()
        logs.append(reducer.trace_log())
    return logs, reducer.num_buckets


@pytest.mark.parametrize("strategy", ["ddp", "bucketed_overlap"])
def test_bucket_allreduce_overlaps_backward(strategy):
    """Part 2b/3 semantics: bucket all-reduces are launched from the autograd hooks WHILE backward
    is still producing gradients -- not after it. Bucket 0 launches before the last gradient-ready
    hook, more than one bucket is in flight before backward ends, launches are in bucket order, and
    the end-of-backward callback comes last."""
    res = run_ranks(_overlap_trace, 2, (strategy,))
    for logs, nb in res:
        assert nb >= 4
        for log in logs[1:]:
            kinds = [k for k, _, _ in log]
            launches = [i for k, i, _ in log if k == "l"]
            assert launches == list(range(nb)), launches
            first_launch = kinds.index("l")
            last_hook = len(kinds) - 1 - kinds[::-1].index("h")
            assert first_launch < last_hook, kinds
            assert sum(1 for k in kinds[:last_hook] if k == "l") >= 2, kinds
            assert kinds[-1] == "f"
            ts = [t for _, _, t in log]
            assert ts == sorted(ts)


# ----------------------------------------------------------------------------- resume agreement
def _agreed_resume(rank, world, root, shared):
    import os

    from cs744_distributed_data_parallel_amd import distributed as dist
    from cs744_distributed_data_parallel_amd.train import _agreed_checkpoint

    d = root if shared else os.path.join(root, f"rank{rank}")
    os.makedirs(d, exist_ok=True)
    if rank == 0:  # only rank 0 writes checkpoints (utils/checkpoint.py)
        for e in (1, 2):
            with open(os.path.join(d, f"ckpt_{e}.pt"), "wb") as fh:
                fh.write(b"x")
    dist.barrier()
    if not shared:  # this rank's filesystem shows only its own directory (no shared storage)
        real = os.path.isfile
        os.path.isfile = lambda q: q.startswith(d) and real(q)
    try:
        return ("ok", _agreed_checkpoint(d, world))
    except RuntimeError as e:
        return ("error", str(e))


def test_resume_checkpoint_is_chosen_by_rank0_and_checked_on_every_rank(tmp_path):
    """--resume: every rank loads the checkpoint rank 0 picked (shared dir), and a checkpoint that
    some rank cannot read fails on every rank instead of silently diverging the replicas."""
    ok = run_ranks(_agreed_resume, 2, (str(tmp_path / "shared"), True))
    assert ok[0][0] == ok[1][0] == "ok"
    assert ok[0][1] == ok[1][1] and ok[0][1].endswith("ckpt_2.pt")
    bad = run_ranks(_agreed_resume, 2, (str(tmp_path / "private"), False))
    assert bad[0][0] == bad[1][0] == "error", bad
    assert "not readable on every rank" in bad[1][1]
