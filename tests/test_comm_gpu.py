"""Native RCCL communicator + reducer on the GPU (single-rank world on the 1-GPU test box; the
multi-rank logic is covered by the gloo tests and the driver's 8-GPU scaling run)."""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

SCRIPT = textwrap.dedent(
    r"""
    import os, torch
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    import cs744_distributed_data_parallel_amd as cdp
    from cs744_distributed_data_parallel_amd import distributed as dist
    dist.init_process_group("rccl", rank=0, world_size=1)
    comm = dist.native_communicator()
    assert comm is not None and comm.kind == "rccl"
    t = torch.arange(8, dtype=torch.float32, device="cuda")
    dist.all_reduce(t)                       # 1 rank: identity
    assert torch.equal(t, torch.arange(8, dtype=torch.float32, device="cuda"))
    w = comm.all_reduce(t, "avg", async_op=True); w.wait()
    dist.broadcast(t, 0)
    outs = [torch.empty(8, device="cuda")]
    dist.gather(t, outs, 0); assert torch.equal(outs[0], t)
    sc = torch.empty(8, device="cuda"); dist.scatter(sc, [t], 0); assert torch.equal(sc, t)
    ag = [torch.empty(8, device="cuda")]; dist.all_gather(ag, t); assert torch.equal(ag[0], t)
    dist.barrier()
    assert comm.healthy()

    # DDP on the native reducer, eager then captured in a hipGraph
    torch.manual_seed(0)
    model = cdp.DistributedDataParallel(cdp.VGG11().cuda(), bucket_cap_mb=4.0)
    info = model._get_ddp_logging_data()
    assert info["native_reducer"] and info["comm"] == "rccl", info
    opt = cdp.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    crit = cdp.CrossEntropyLoss()
    x = torch.randn(32, 3, 32, 32, device="cuda"); y = torch.randint(0, 10, (32,), device="cuda")
    def body():
        opt.zero_grad()
        loss = crit(model(x), y)
        loss.backward()
        opt.step()
        return loss
    for _ in range(3):
        body()
    assert model._get_ddp_logging_data()["rebuilt_buckets"]
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        sl = body()
    vals = []
    for _ in range(4):
        g.replay(); vals.append(sl.item())
    assert vals[-1] < vals[0], vals
    # every parameter's gradient is its arena view (zero-copy buckets)
    ar = model.arena
    for p in model.parameters():
        assert p.grad is not None
        v = ar.grad_views()[p._cdp_index]
        assert p.grad.data_ptr() == v.data_ptr()
    dist.destroy_process_group()
    print("COMM_OK")
    """
)


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_single_rank_ddp_and_graph():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = repo + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True, timeout=300)
    assert "COMM_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-5000:]


ORDER_SCRIPT = textwrap.dedent(
    r"""
    import os, torch
    # every all_reduce on the native communicator is followed, on the comm stream and inside its
    # completion event, by a ~3 ms idle wait and then grad *= 2 (RcclComm::set_test_postop)
    os.environ["CDP_REDUCER_TEST_POSTOP"] = "3000:2"
    import cs744_distributed_data_parallel_amd as cdp
    from cs744_distributed_data_parallel_amd import distributed as dist
    dist.init_process_group("rccl", rank=0, world_size=1)
    assert dist.native_communicator() is not None
    crit = cdp.CrossEntropyLoss()
    x = torch.randn(64, 3, 32, 32, device="cuda"); y = torch.randint(0, 10, (64,), device="cuda")

    def fresh():
        torch.manual_seed(0)
        return cdp.VGG11().cuda()

    m0 = fresh()
    crit(m0(x), y).backward()
    ref = [p.grad.detach().clone() for p in m0.parameters()]
    snap = [p.detach().clone() for p in m0.parameters()]
    torch.cuda.synchronize()

    # tensors whose gradient is numerically zero (conv biases ahead of BatchNorm: analytically 0,
    # rounding noise in practice) carry no ordering signal and are skipped
    rms = [float(v.pow(2).mean().sqrt()) for v in ref]
    keep = [r > 1e-3 * max(rms) for r in rms]

    def ratios(a, b):
        return [float((u * v).sum() / (v * v).sum()) for u, v, k in zip(a, b, keep) if k]

    for kind in ("ddp", "bucketed_overlap"):
        for graph in (False, True):
            base = fresh()
            model, sync = base, None
            if kind == "ddp":
                model = cdp.DistributedDataParallel(base, bucket_cap_mb=2.0)
            else:
                sync = cdp.parallel.BucketedOverlap(base, bucket_cap_mb=2.0)
            opt = cdp.SGD(base.parameters(), lr=1.0, momentum=0.0, weight_decay=0.0)

            def body():
                opt.zero_grad()
                out = model(x)
                if sync is not None:
                    sync.prepare(out)
                crit(out, y).backward()
                opt.step()

            for _ in range(3):  # includes the bucket rebuild in ready order
                body()
            g = None
            if graph:
                s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    body()
                torch.cuda.current_stream().wait_stream(s)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    body()
            torch.cuda.synchronize()
            with torch.no_grad():
                for p, v in zip(base.parameters(), snap):
                    p.copy_(v)
            # weights edited outside the captured step: re-derive what its forward reads from the
            # last step (the fused SGD + weight preparation, SGD.refresh_weight_prep)
            opt.refresh_weight_prep()
            if g is not None:
                g.replay()
            else:
                body()
            # read the update on the compute stream right away: SGD (p -= 1.0 * grad) must have run
            # after the delayed post-op, i.e. consumed exactly 2x the gradient
            delta = [v - p.detach() for p, v in zip(base.parameters(), snap)]
            torch.cuda.synchronize()
            final = [p.grad.detach() for p in base.parameters()]
            r_step = ratios(delta, final)  # 1.0: SGD consumed the post-op'd gradient
            r_grad = ratios(final, ref)    # 2.0: the post-op ran on every bucket
            assert all(abs(r - 1.0) < 2e-3 for r in r_step), (kind, graph, "SGD saw", r_step)
            assert all(abs(r - 2.0) < 2e-3 for r in r_grad), (kind, graph, r_grad)
            print("ORDER_OK", kind, "graph" if graph else "eager", len(r_step), flush=True)
            if g is not None:
                g.reset()
            if kind == "ddp":
                model.reducer.remove()
            else:
                sync.remove()
    dist.destroy_process_group()
    print("ORDER_ALL_OK")
    """
)


def test_reducer_comm_to_compute_ordering_with_delayed_postop():
    """Proves the comm->compute event edge on ONE GPU: each bucket's collective is followed on the
    communicator stream by a delay and a scale-by-2; SGD must see exactly 2x the gradient, eager and
    under hipGraph capture, for DDP and BucketedOverlap (csrc/runtime/reducer.cpp finalize ->
    RcclWork::wait)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = repo + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-c", ORDER_SCRIPT], env=env, capture_output=True, text=True, timeout=300)
    assert "ORDER_ALL_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-5000:]
    assert r.stdout.count("ORDER_OK") == 4


WATCHDOG_SCRIPT = textwrap.dedent(
    r"""
    import os, time, torch
    # every all_reduce is followed, on the comm stream and inside its completion event, by a 1.5 s
    # idle wait (RcclComm::set_test_postop): to the watchdog that is a collective that never finishes
    os.environ["CDP_REDUCER_TEST_POSTOP"] = "1500000:1"
    from cs744_distributed_data_parallel_amd import distributed as dist
    dist.init_process_group("rccl", rank=0, world_size=1)
    comm = dist.native_communicator()
    assert comm is not None and comm.healthy()
    comm.set_timeout(0.2)
    t = torch.ones(1024, device="cuda")
    w = comm.all_reduce(t, "sum", async_op=True)
    t0 = time.time()
    try:
        w.synchronize()
        raise SystemExit("synchronize returned although the collective outlived the timeout")
    except RuntimeError as e:
        msg = str(e)
    waited = time.time() - t0
    assert "did not complete within" in msg and "all_reduce" in msg, msg
    assert waited < 1.2, waited  # the watchdog's abort ended the wait, not the collective finishing
    assert not comm.healthy() and not dist.healthy()
    assert "all_reduce" in comm.error()
    try:  # every later collective fails fast instead of hanging on the aborted communicator
        dist.all_reduce(t)
        raise SystemExit("a collective ran on the aborted communicator")
    except RuntimeError as e:
        assert "RCCL communicator failed" in str(e), str(e)
    torch.cuda.synchronize()  # the delay kernel drains
    dist.destroy_process_group()
    print("WATCHDOG_OK", round(waited, 3))
    """
)


def test_watchdog_aborts_a_stuck_collective():
    """A collective that outlives set_timeout: the communicator's watchdog aborts it, the waiting
    host call raises instead of hanging, healthy() goes false and the next collective raises
    (csrc/runtime/rccl_comm.cpp watchdog_loop / abort / check)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = repo + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-c", WATCHDOG_SCRIPT], env=env, capture_output=True, text=True, timeout=200)
    assert "WATCHDOG_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-5000:]


OVERLAP_SCRIPT = textwrap.dedent(
    r"""
    import os, torch
    # every collective is followed on the comm stream by a ~300 us kernel (RcclComm test post-op)
    os.environ["CDP_REDUCER_TEST_POSTOP"] = "300:1"
    import cs744_distributed_data_parallel_amd as cdp
    from cs744_distributed_data_parallel_amd import distributed as dist
    dist.init_process_group("rccl", rank=0, world_size=1)
    comm = dist.native_communicator()
    C = cdp._native.lib()
    hz = C.gpu_wall_clock_khz() * 1e3
    buf = torch.zeros(1024, device="cuda")  # one workgroup of post-op: no CU starvation, only the streams
    ts = torch.zeros(8, dtype=torch.int64, device="cuda")
    worst = []
    for rep in range(5):
        torch.cuda.synchronize()
        C.gpu_sleep(2000.0)                 # the host enqueues everything below ahead of the GPU
        C.gpu_timestamp(ts, 0)
        w = comm.all_reduce(buf, "sum", True)
        for i in range(1, 7):
            C.gpu_timestamp(ts, i)          # compute-stream dispatches while the comm stream works
        w.wait()
        C.gpu_timestamp(ts, 7)              # ordered after the collective and its post-op
        torch.cuda.synchronize()
        r = ts.cpu().tolist()
        gaps = [(r[i + 1] - r[i]) / hz * 1e6 for i in range(1, 6)]
        worst.append(max(gaps))
        assert (r[7] - r[0]) / hz * 1e6 >= 250.0, r
    print("GAPS", worst)
    # the comm stream runs beside the compute stream without holding its dispatches back, in every
    # repetition (a stream at the device's least priority held every compute dispatch 40-57 us;
    # profiles/comm_stream_priority_r5.md)
    assert max(worst) < 25.0, worst
    dist.destroy_process_group()
    print("OVERLAP_OK")
    """
)


def test_comm_stream_work_does_not_hold_back_compute_dispatches():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = repo + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-c", OVERLAP_SCRIPT], env=env, capture_output=True, text=True, timeout=300)
    assert "OVERLAP_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-5000:]


PRIVATE_STREAM_SCRIPT = textwrap.dedent(
    r"""
    import torch
    import cs744_distributed_data_parallel_amd as cdp
    from cs744_distributed_data_parallel_amd import distributed as dist
    dist.init_process_group("rccl", rank=0, world_size=1)
    c = dist.native_communicator().native
    assert c.stream_kind == "own", c.stream_kind
    ptr = c.stream_ptr
    # PyTorch's pool hands its 32 streams per priority out round-robin: none of them, nor a capture
    # stream, may be the communicator's
    seen = {torch.cuda.Stream().cuda_stream for _ in range(100)}
    seen |= {torch.cuda.Stream(priority=-1).cuda_stream for _ in range(100)}
    assert ptr not in seen and ptr != torch.cuda.current_stream().cuda_stream
    # a collective issued FROM the comm stream is refused instead of ordering it behind itself
    buf = torch.ones(16, device="cuda")
    with torch.cuda.stream(torch.cuda.ExternalStream(ptr)):
        try:
            c.all_reduce(buf, "sum", False)
            raise SystemExit("collective from the comm stream was accepted")
        except RuntimeError as e:
            assert "communicator's own stream" in str(e), str(e)
    dist.destroy_process_group()
    print("PRIVATE_OK")
    """
)


def test_comm_stream_is_private_to_the_communicator():
    """The communicator's stream is its own (normal priority, never one PyTorch's stream pool can hand
    out again) and a collective issued from it is refused."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    env.pop("CDP_COMM_STREAM", None)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = repo + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-c", PRIVATE_STREAM_SCRIPT], env=env, capture_output=True, text=True,
                       timeout=200)
    assert "PRIVATE_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-5000:]
