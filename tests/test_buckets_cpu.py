"""The bucket planner (parallel/buckets.py): the timed plan the reducer designs at its ready-order
rebuild, pinned for VGG-11 and ResNet-50, checked optimal against brute force, and never worse
than the fixed-cap plan under the same model. Reference: the bucketing inside ``DDP(model)``
(/root/reference/src/Part 3/main.py:61)."""
import itertools
import random

import pytest

from cs744_distributed_data_parallel_amd.parallel.buckets import (
    fit_comm_model,
    plan_buckets,
    plan_buckets_timed,
)

# VGG-11 at the reference's 8-rank strong-scaling point (32 images per GPU): when each block's
# gradients are ready after backward starts (us; the reducer's timed calibration backward measured on
# MI355X, profiles/vgg11_b32_ddp_overlap_r4.md), and the block's tensors in ready order (BN weight /
# bias, conv bias, conv weight; bytes)
VGG11_B32 = [
    (0, [40, 20480]),  # fc1
    (33, [2048, 2048, 2048, 9437184]),  # block 7 (layers.25/26)
    (59, [2048, 2048, 2048, 9437184]),
    (101, [2048, 2048, 2048, 9437184]),
    (133, [2048, 2048, 2048, 4718592]),
    (179, [1024, 1024, 1024, 2359296]),
    (214, [1024, 1024, 1024, 1179648]),
    (252, [512, 512, 512, 294912]),
    (267, [256, 256, 256, 6912]),  # block 0 (the stem), ready last
]
ALPHA = 15e-6  # RCCL all-reduce latency at W = 8 (assumed for the pin)
BETA = 1.75 / 300e9  # ring: 2 (W-1) / W bytes per byte at 300 GB/s bus bandwidth


def _vgg():
    nb, rd = [], []
    for t, sizes in VGG11_B32:
        for b in sizes:
            nb.append(b)
            rd.append(t * 1e-6)
    return nb, rd


def _end(groups, nb, rd, alpha, beta):
    end = float("-inf")
    for g in groups:
        end = max(end, max(rd[: g[-1] + 1])) + alpha + beta * sum(nb[i] for i in g)
    return end


def test_vgg11_strong_scaling_plan_is_pinned():
    nb, rd = _vgg()
    groups, info = plan_buckets_timed(nb, rd, ALPHA, BETA)
    assert [sum(nb[i] for i in g) for g in groups] == [9_463_848, 9_443_328, 14_168_064, 3_849_216]
    # the tail (blocks 0-3, ready last) stays small: its all-reduce is the only exposed one
    assert info["exposed_us"] < 45.0
    assert info["backward_end_us"] == 267.0
    # the fixed 8 MiB / 1 MiB plan ends later under the same model
    greedy = plan_buckets(nb, 8.0, 1.0)
    assert _end(groups, nb, rd, ALPHA, BETA) < _end(greedy, nb, rd, ALPHA, BETA) - 20e-6


@pytest.mark.parametrize("bwd_ms,expect", [(8.0, [148, 13]), (1.0, [56, 78, 23, 4])])
def test_resnet50_plan_is_pinned(bwd_ms, expect):
    import cs744_distributed_data_parallel_amd as cdp

    ps = list(cdp.get_model("resnet50").parameters())[::-1]  # launch order: reverse definition
    assert len(ps) == 161
    nb = [p.numel() * 4 for p in ps]
    rd = [bwd_ms * 1e-3 * (i + 1) / len(nb) for i in range(len(nb))]  # uniform timeline
    groups, info = plan_buckets_timed(nb, rd, ALPHA, BETA)
    assert [len(g) for g in groups] == expect
    assert info["exposed_us"] < 20.0


def test_timed_plan_is_optimal_by_brute_force():
    rnd = random.Random(5)
    for _ in range(60):
        n = rnd.randint(1, 8)
        nb = [rnd.choice([256, 4096, 2 ** 20, 9 * 2 ** 20]) for _ in range(n)]
        rd = sorted(rnd.uniform(0, 300e-6) for _ in range(n))
        alpha, beta, pen = rnd.uniform(2e-6, 30e-6), 1.75 / rnd.uniform(50e9, 500e9), 3e-6
        groups, _ = plan_buckets_timed(nb, rd, alpha, beta, pen)
        assert sorted(i for g in groups for i in g) == list(range(n))
        got = _end(groups, nb, rd, alpha, beta) + pen * len(groups)
        best = float("inf")
        for cuts in itertools.product([0, 1], repeat=n - 1):
            gs, cur = [], [0]
            for i, c in enumerate(cuts, start=1):
                if c:
                    gs.append(cur)
                    cur = []
                cur.append(i)
            gs.append(cur)
            best = min(best, _end(gs, nb, rd, alpha, beta) + pen * len(gs))
        assert got <= best + 1e-12, (got, best)


def test_comm_model_fit_recovers_alpha_beta():
    sizes = [2 ** 18, 2 ** 21, 2 ** 23]
    a, b = fit_comm_model(sizes, [12e-6 + s * 4e-12 for s in sizes])
    assert abs(a - 12e-6) < 1e-9 and abs(b - 4e-12) < 1e-15


class _FakeLib:
    @staticmethod
    def gpu_wall_clock_khz():
        return 100_000.0  # 100 MHz: 100 ticks per us


def _timed_reducer(monkeypatch, stamp_cost_us):
    """A GradReducer over a small CPU model whose last timed backward is faked as a GPU record:
    parameters ready 10 us apart in reverse order, and the two back-to-back reference stamps
    stamp_cost_us apart."""
    import torch

    from cs744_distributed_data_parallel_amd.parallel import reducer as R
    from cs744_distributed_data_parallel_amd.parallel.local import LocalGroup
    from cs744_distributed_data_parallel_amd.utils.arena import arena_for

    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    params = list(model.parameters())
    red = R.GradReducer(arena_for(params), LocalGroup(1).communicator(0), timed_plan=True)
    n = len(params)
    ticks = [1000 + 1000 * (n - 1 - i) for i in range(n)] + [0, int(stamp_cost_us * 100)]
    red.stop_ready_timing()
    red._timing = ({i: i for i in range(n)}, [], True, params, [True], torch.tensor(ticks, dtype=torch.int64))
    monkeypatch.setattr(R._native, "lib", lambda: _FakeLib)
    monkeypatch.setattr(R.torch.cuda, "synchronize", lambda *a, **k: None)
    monkeypatch.setattr(R.GradReducer, "_measure_comm", lambda self, *a, **k: (20e-6, 1e-12))
    return red, params


def test_calibration_stamps_give_the_ready_timeline(monkeypatch):
    red, params = _timed_reducer(monkeypatch, 2.0)
    rt = red._ready_times()
    assert rt is not None and abs(red.stamp_cost_us - 2.0) < 1e-9
    # ready 10 us apart, minus the 2 us each preceding stamp adds: 8 us apart
    got = sorted(rt[id(p)] for p in params)
    assert all(abs((b - a) - 8e-6) < 1e-12 for a, b in zip(got, got[1:]))
    assert red.rebuild_in_ready_order(list(range(len(params)))[::-1])
    assert red.plan_info["planner"] == "timed"


def test_distorted_calibration_timeline_keeps_the_cap_plan(monkeypatch):
    """Dispatches ~50 us apart during the timed backward (the stream was held back): no plan is
    designed from that timeline; the reducer keeps the fixed-cap plan and says why."""
    red, params = _timed_reducer(monkeypatch, 50.0)
    assert red._ready_times() is None
    red.rebuild_in_ready_order(list(range(len(params)))[::-1])
    assert red.plan_info["planner"] == "cap"
    assert "distorted" in red.plan_info["fallback"]
