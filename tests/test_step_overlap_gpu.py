"""Overlapped optimizer step (``DistributedDataParallel.overlap_optimizer``) on the GPU.

The SGD of each gradient bucket runs on the reducer's step stream right after that bucket's RCCL
all-reduce, instead of once after the last bucket (the DDP step of ``/root/reference/src/Part
3/main.py:61,96-97``). One rank on the test box's one GPU, with every all-reduce followed by the
modelled ring time of an 8-rank xGMI node (``CDP_REDUCER_TEST_POSTOP=xgmi:alpha:GBps:W``), so the
buckets finish late and out of step with backward, as they would with peers. The result must be
bitwise the end-of-step SGD's, eager and replayed from a hipGraph, and the step counter must advance
exactly once per step.
"""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

SCRIPT = textwrap.dedent(
    r"""
    import os, torch
    os.environ["CDP_REDUCER_TEST_POSTOP"] = "xgmi:20:100:8"
    import cs744_distributed_data_parallel_amd as cdp
    from cs744_distributed_data_parallel_amd import distributed as dist
    dist.init_process_group("rccl", rank=0, world_size=1)
    assert dist.native_communicator() is not None
    crit = cdp.CrossEntropyLoss()
    g = torch.Generator(device="cuda").manual_seed(1)
    xs = [torch.randn(32, 3, 32, 32, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
          for _ in range(5)]
    ys = [torch.randint(0, 10, (32,), device="cuda", generator=g) for _ in range(5)]

    MODE = os.environ["CDP_TEST_MODE"]  # the variant run: "overlap", "early" or "both"

    def make(variant):
        torch.manual_seed(0)
        model = cdp.DistributedDataParallel(cdp.VGG11().cuda())
        opt = cdp.SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
        ctr = torch.zeros(1, dtype=torch.int64, device="cuda")
        opt.advance_each_step(ctr)
        if variant and MODE in ("overlap", "both"):
            model.overlap_optimizer(opt)
        if variant and MODE in ("early", "both"):
            model.early_buffer_broadcast(opt)
        return model, opt, ctr

    runs = {k: make(k) for k in (False, True)}
    xb = torch.empty_like(xs[0]); yb = torch.empty_like(ys[0])

    def body(model, opt):
        opt.zero_grad()
        loss = crit(model(xb), yb)
        loss.backward()
        opt.step()
        return loss

    def state(model, opt):
        ps = [p.detach().clone() for p in model.parameters()] + [b.detach().clone() for b in model.buffers()]
        ms = [opt.state[p]["momentum_buffer"].detach().clone() for p in model.parameters()]
        return ps, ms

    def same(a, b, what):
        for u, v in zip(a[0] + a[1], b[0] + b[1]):
            assert torch.equal(u, v), what

    # eager: 20 steps each, compared after every step
    for step in range(20):
        xb.copy_(xs[step % 5]); yb.copy_(ys[step % 5])
        losses = {}
        for k, (m, o, c) in runs.items():
            losses[k] = body(m, o).item()
        assert losses[False] == losses[True], (step, losses)
        same(state(*runs[False][:2]), state(*runs[True][:2]), f"eager step {step}")
    m1 = runs[True][0]
    nb = m1.reducer.num_buckets
    if MODE in ("overlap", "both"):
        assert m1._get_ddp_logging_data()["overlapped_step_buckets"] == nb >= 2, (nb, m1._get_ddp_logging_data())
    if MODE in ("early", "both"):
        # every synced backward issued the broadcast (the next forward took it instead of its own)
        assert m1._get_ddp_logging_data()["early_buffer_broadcast"]
        assert m1.reducer.take_post_issued() == len(list(m1._buffers_arena.flats())) > 0
    assert runs[True][0]._get_ddp_logging_data()["rebuilt_buckets"]
    assert int(runs[False][2]) == 20 and int(runs[True][2]) == 20

    # captured: one graph per run, 20 replays, compared after every replay
    graphs = {}
    for k, (m, o, c) in runs.items():
        s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            body(m, o)
        torch.cuda.current_stream().wait_stream(s)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            lo = body(m, o)
        graphs[k] = (gr, lo)
    torch.cuda.synchronize()
    same(state(*runs[False][:2]), state(*runs[True][:2]), "after capture")
    for step in range(20):
        xb.copy_(xs[step % 5]); yb.copy_(ys[step % 5])
        for k, (gr, lo) in graphs.items():
            gr.replay()
        torch.cuda.synchronize()
        assert graphs[False][1].item() == graphs[True][1].item(), step
        same(state(*runs[False][:2]), state(*runs[True][:2]), f"replay {step}")
    assert int(runs[False][2]) == int(runs[True][2]) == 41
    dist.destroy_process_group()
    print("OVERLAP_OK", nb)
    """
)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode", ["overlap", "early", "both"])
def test_overlapped_step_is_bitwise_the_end_of_step_sgd(mode):
    """mode: the variant run overlaps the SGD with the buckets (overlap), broadcasts the BN buffers
    behind the last bucket joined after the SGD (early: DistributedDataParallel.early_buffer_broadcast;
    in the modelled mode the one rank's broadcasts are timed delays on the comm stream), or both."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", CDP_TEST_MODE=mode)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = repo + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True, timeout=300)
    assert "OVERLAP_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-5000:]
