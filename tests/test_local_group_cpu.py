"""In-process multi-rank tests on the thread/shared-memory communicator double:
collectives at W=8 over odd sizes and the VGG-11 message sizes of SURVEY §2.5, the four sync
strategies' equivalence at W=4, reducer bucket order / unused parameters, and fail-fast behaviour."""
import copy

import pytest
import torch

import cs744_distributed_data_parallel_amd as cdp
from cs744_distributed_data_parallel_amd.parallel import (
    BucketedOverlap,
    DistributedDataParallel,
    LocalGroup,
    average_gradients_allreduce,
    average_gradients_gather_scatter,
)

# fp32 element counts of the VGG-11 gradients plus odd sizes
SIZES = [1, 3, 10, 64, 1728, 73728, 294912, 589824, 1179648, 2359296]


def _coll(rank, world, comm):
    out = {}
    for n in SIZES:
        t = torch.arange(n, dtype=torch.float32) * 1e-3 + rank
        comm.all_reduce(t, "sum")
        exp = torch.arange(n, dtype=torch.float64) * 1e-3 * world + sum(range(world))
        out[("sum", n)] = float((t.double() - exp).abs().max())
        a = torch.full((n,), float(rank))
        comm.all_reduce(a, "avg")
        out[("avg", n)] = float((a - (world - 1) / 2).abs().max())
    b = torch.full((5,), float(rank))
    comm.broadcast(b, src=world - 1)
    out["bcast"] = b.tolist()
    g = [torch.empty(7) for _ in range(world)] if rank == 0 else None
    comm.gather(torch.full((7,), 10.0 * rank), g, 0)
    out["gather"] = [float(x[0]) for x in g] if g else None
    s = torch.empty(3)
    comm.scatter(s, [torch.full((3,), 100.0 + r) for r in range(world)] if rank == 1 else None, 1)
    out["scatter"] = float(s[0])
    ag = torch.empty(world * 2)
    comm.all_gather(ag, torch.full((2,), float(rank)))
    out["ag"] = ag.tolist()
    rs = torch.empty(2)
    comm.reduce_scatter(rs, torch.arange(world * 2, dtype=torch.float32), "sum")
    out["rs"] = rs.tolist()
    mx = torch.tensor([float(rank)])
    comm.all_reduce(mx, "max")
    out["max"] = float(mx)
    comm.barrier()
    return out


def test_collectives_w8_message_sizes():
    world = 8
    res = LocalGroup(world).run(_coll)
    for r, d in enumerate(res):
        for n in SIZES:
            assert d[("sum", n)] < 1e-3 * max(1.0, n * 1e-3), (r, n)
            assert d[("avg", n)] == 0.0
        assert d["bcast"] == [float(world - 1)] * 5
        assert d["scatter"] == 100.0 + r
        assert d["ag"] == [float(i) for i in range(world) for _ in range(2)]
        assert d["rs"] == [float(world * (2 * r)), float(world * (2 * r + 1))]
        assert d["max"] == world - 1
    assert res[0]["gather"] == [10.0 * i for i in range(world)]


def _batch(rank, step, B=4):
    g = torch.Generator().manual_seed(1000 * step + rank)
    return torch.randn(B, 3, 32, 32, generator=g), torch.randint(0, 10, (B,), generator=g)


def _train(rank, world, comm, base, strategy, steps):
    model = copy.deepcopy(base)  # identical init on every rank (2a/2b have no broadcast)
    sync = None
    if strategy == "ddp":
        model = DistributedDataParallel(model, bucket_cap_mb=1.0, comm=comm)
    elif strategy == "bucketed_overlap":
        sync = BucketedOverlap(model, comm=comm, bucket_cap_mb=1.0)
    opt = cdp.SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    crit = cdp.CrossEntropyLoss()
    for step in range(steps):
        x, y = _batch(rank, step)
        opt.zero_grad()
        out = model(x)
        if sync is not None:
            sync.prepare(out)
        loss = crit(out, y)
        loss.backward()
        if strategy == "gather_scatter":
            average_gradients_gather_scatter(model, rank, comm=comm)
        elif strategy == "allreduce_blocking":
            average_gradients_allreduce(model, comm=comm)
        opt.step()
    m = getattr(model, "module", model)
    return torch.cat([p.detach().reshape(-1) for p in m.parameters()])


@pytest.mark.parametrize("world", [4])
def test_four_strategies_equivalent_in_process(world):
    torch.manual_seed(0)
    base = cdp.VGG11(channels_last=False)
    flats = {}
    for strategy in ("gather_scatter", "allreduce_blocking", "bucketed_overlap", "ddp"):
        res = LocalGroup(world).run(_train, base, strategy, 2)
        for r in range(1, world):  # every rank holds the same model
            assert torch.allclose(res[r], res[0], atol=1e-6), (strategy, r)
        flats[strategy] = res[0]
    ref = flats["allreduce_blocking"]
    for s, f in flats.items():
        assert torch.allclose(f, ref, atol=2e-5, rtol=1e-5), s


def _unused(rank, world, comm, find_unused):
    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Linear(4, 4)
            self.b = torch.nn.Linear(4, 4)  # never used

        def forward(self, x):
            return self.a(x)

    torch.manual_seed(0)
    m = DistributedDataParallel(Net(), comm=comm, find_unused_parameters=find_unused)
    out = m(torch.randn(2, 4) + rank)
    out.sum().backward()
    return m.module.b.weight.grad is not None and float(m.module.b.weight.grad.abs().sum()) == 0.0


def test_unused_parameters_w8():
    assert all(LocalGroup(8).run(_unused, True))
    with pytest.raises(RuntimeError):
        LocalGroup(2, timeout_s=10).run(_unused, False)


def _fail(rank, world, comm):
    if rank == 2:
        raise ValueError("rank 2 dies")
    comm.all_reduce(torch.ones(3))  # the others must not hang
    return True


def test_dead_rank_fails_fast():
    import time

    t0 = time.time()
    with pytest.raises(RuntimeError, match="rank 2 dies"):
        LocalGroup(4, timeout_s=30).run(_fail)
    assert time.time() - t0 < 20
