"""The optimizer step that also prepares the next forward's weights (csrc sgd_prep_kernel): one pass
over the parameter arena instead of SGD (sgd_kernel) + a separate weight_prep_kernel at the next
forward.

* 20 VGG-11 steps with the fused step and 20 with the two-kernel path from the same init give
  bitwise-identical parameters and momentum buffers (the update is the same sgd_one per element),
  and the forwards after the first really take the fused products (PREP_HITS).
* The prepared |max| partials and W^T equal what the standalone weight_prep_kernel makes from the
  stepped weights.
* A weight edited in place between steps (``torch.no_grad(): w.add_``, load_state_dict) bumps its
  version: the next forward prepares the weights itself and its output matches a model that never
  used the fused path.
* A captured hipGraph step cannot re-check weights on the host: after editing them between replays,
  SGD.refresh_weight_prep() re-derives the products in place and the replay equals an eager step.
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(seed=0):
    import cs744_distributed_data_parallel_amd as cdp

    torch.manual_seed(seed)
    model = cdp.VGG11().cuda()
    opt = cdp.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    return cdp, model, opt


def _batch(step, B=64):
    g = torch.Generator(device="cuda").manual_seed(1000 + step)
    x = torch.randn(B, 3, 32, 32, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (B,), device="cuda", generator=g)
    return x, y


def _train(fused, steps=20):
    from cs744_distributed_data_parallel_amd.ops import functional as CF

    cdp, model, opt = _setup()
    opt.fused_prep = fused
    crit = cdp.CrossEntropyLoss()
    h0 = CF.PREP_HITS[0]
    for i in range(steps):
        x, y = _batch(i)
        opt.zero_grad()
        crit(model(x), y).backward()
        opt.step()
    torch.cuda.synchronize()
    params = [p.detach().clone() for p in model.parameters()]
    moms = [opt.state[p]["momentum_buffer"].clone() for p in model.parameters()]
    return params, moms, CF.PREP_HITS[0] - h0, model, opt


def test_fused_step_is_bitwise_the_two_kernel_path():
    p_f, m_f, hits_f, _, _ = _train(True)
    p_s, m_s, hits_s, _, _ = _train(False)
    assert hits_f == 19 and hits_s == 0, (hits_f, hits_s)
    for a, b in zip(p_f + m_f, p_s + m_s):
        assert torch.equal(a, b)


def test_fused_products_equal_standalone_weight_prep():
    from cs744_distributed_data_parallel_amd.ops import functional as CF

    _, _, _, model, opt = _train(True, steps=3)
    weights = [model.layers[ci].weight for ci, _, _ in model._plan]
    want = [k > 0 for k in range(len(weights))]
    hit = model.layers[0].weight._cdp_arena.prep_lookup(weights, want)
    assert hit is not None
    amax_f, wts_f = hit
    C = __import__("cs744_distributed_data_parallel_amd")._native.lib()
    amax_s, wts_s = C.weight_prep(weights, want)
    for k in range(len(weights)):
        assert torch.equal(amax_f[k], amax_s[k]), k
        if want[k]:
            assert torch.equal(wts_f[k], wts_s[k]), k
        else:
            assert wts_f[k] is None


@pytest.mark.parametrize("edit", ["inplace", "load_state_dict"])
def test_weight_edited_between_steps_is_seen_by_the_gemms(edit):
    from cs744_distributed_data_parallel_amd.ops import functional as CF

    cdp, model, opt = _setup()
    crit = cdp.CrossEntropyLoss()
    for i in range(3):
        x, y = _batch(i)
        opt.zero_grad()
        crit(model(x), y).backward()
        opt.step()
    w = model.layers[8].weight  # block 2's conv: its W^T and |max| come from the fused step
    if edit == "inplace":
        with torch.no_grad():
            w.mul_(3.0)  # the |max| and W^T the step wrote are now stale
    else:
        sd = {k: v.clone() for k, v in model.state_dict().items()}
        sd["layers.8.weight"] = sd["layers.8.weight"] * 3.0
        model.load_state_dict(sd)
    h0 = CF.PREP_HITS[0]
    x, y = _batch(99)
    model.train()
    out = model(x)
    if edit == "inplace":
        assert CF.PREP_HITS[0] == h0  # the forward prepared the edited weights itself
    else:
        # load_state_dict's post-hook re-derived the products from the loaded weights
        assert CF.PREP_HITS[0] == h0 + 1
    # a fresh model holding the same (edited) weights, never touched by a fused step
    _, ref, _ = _setup()
    ref.load_state_dict(model.state_dict())
    ref.train()
    out_ref = ref(x)
    torch.cuda.synchronize()
    assert torch.equal(out, out_ref)
    # and backward uses the edited W^T: same input gradient as the fresh model
    xa = x.clone().requires_grad_()
    xb = x.clone().requires_grad_()
    crit(model(xa), y).backward()
    crit(ref(xb), y).backward()
    assert torch.equal(xa.grad, xb.grad)


def test_captured_step_sees_weights_edited_between_replays_after_refresh():
    """A replayed hipGraph step reads the |max| / W^T its previous replay's optimizer step wrote; after
    weights are edited outside the graph, SGD.refresh_weight_prep() re-derives them in place, and the
    replay then equals an eager step from the edited weights."""
    cdp, model, opt = _setup()
    crit = cdp.CrossEntropyLoss()
    x, y = _batch(0)

    def body():
        opt.zero_grad()
        crit(model(x), y).backward()
        opt.step()

    for _ in range(3):
        body()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    torch.cuda.synchronize()
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    sd["layers.11.weight"] = sd["layers.11.weight"] * 0.5
    mom = {id(p): opt.state[p]["momentum_buffer"].clone() for p in model.parameters()}
    model.load_state_dict(sd)
    assert opt.refresh_weight_prep()
    g.replay()
    torch.cuda.synchronize()
    got = [p.detach().clone() for p in model.parameters()]
    # eager twin: a fresh model + optimizer with the same weights and momentum, one step
    _, ref, ropt = _setup()
    ref.load_state_dict(sd)
    ropt.fused_prep = False
    for p in ref.parameters():
        ropt.state[p]["momentum_buffer"] = None
    rp = list(ref.parameters())
    for p, q in zip(rp, model.parameters()):
        ropt.state[p]["momentum_buffer"] = mom[id(q)].clone()
    ropt.zero_grad()
    crit(ref(x), y).backward()
    ropt.step()
    torch.cuda.synchronize()
    for a, b in zip(got, rp):
        assert torch.equal(a, b.detach())


@pytest.mark.parametrize("what", ["model", "model+optimizer"])
def test_captured_step_after_load_state_dict_matches_eager(what):
    """No manual refresh: ``model.load_state_dict`` (its post-hook re-derives the fused-step products
    from the loaded weights) and ``opt.load_state_dict`` (the loaded momentum moves into the arena
    the graph reads) between replays of a captured step, and the next replay equals an eager step
    of a fresh model + optimizer loaded from the same state."""
    cdp, model, opt = _setup()
    crit = cdp.CrossEntropyLoss()
    x, y = _batch(0)

    def body():
        opt.zero_grad()
        crit(model(x), y).backward()
        opt.step()

    for _ in range(3):
        body()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    torch.cuda.synchronize()
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    for k in ("layers.8.weight", "layers.11.weight", "layers.25.weight"):
        sd[k] = sd[k] * 0.5
    osd = copy.deepcopy(opt.state_dict())  # (state_dict() returns the live arena views)
    if what == "model+optimizer":
        for st in osd["state"].values():
            st["momentum_buffer"] = st["momentum_buffer"] * 0.25
    model.load_state_dict(sd)
    if what == "model+optimizer":
        opt.load_state_dict(osd)
    g.replay()
    torch.cuda.synchronize()
    got = [p.detach().clone() for p in model.parameters()]
    _, ref, ropt = _setup()
    ref.load_state_dict(sd)
    ropt.load_state_dict(osd)
    ropt.fused_prep = False
    ropt.zero_grad()
    crit(ref(x), y).backward()
    ropt.step()
    torch.cuda.synchronize()
    for a, b in zip(got, ref.parameters()):
        assert torch.equal(a, b.detach())


def test_loader_counter_advanced_by_the_optimizer_step():
    """DeviceLoader.advance_with(opt): the SGD kernel advances the loader's step counter (no
    counter_inc launch); the batch sequence and the trained parameters are those of the default
    path, eager and in a replayed hipGraph."""
    import cs744_distributed_data_parallel_amd as cdp
    from cs744_distributed_data_parallel_amd.data import DeviceLoader, synthetic_cifar10

    def run(external, graph):
        torch.manual_seed(0)
        model = cdp.VGG11().cuda()
        opt = cdp.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        crit = cdp.CrossEntropyLoss()
        loader = DeviceLoader(synthetic_cifar10(256, seed=0, device=torch.device("cuda")), 32, shuffle=True)
        if external:
            assert loader.advance_with(opt)
        order = loader._order()
        labels = []

        def body():
            x, y = loader.batch(order, 0, 32, nbatches=8)
            labels.append(y)
            opt.zero_grad()
            crit(model(x), y).backward()
            opt.step()

        for _ in range(3):
            body()
        if graph:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                body()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                body()
            for _ in range(3):
                g.replay()
                labels.append(labels[-1].clone())
        torch.cuda.synchronize()
        return [p.detach().clone() for p in model.parameters()], int(loader._counter.item()), labels

    for graph in (False, True):
        p_ext, c_ext, l_ext = run(True, graph)
        p_def, c_def, l_def = run(False, graph)
        assert c_ext == c_def == (3 if not graph else 7)
        for a, b in zip(l_ext, l_def):
            assert torch.equal(a, b)
        for a, b in zip(p_ext, p_def):
            assert torch.equal(a, b)


def test_loader_advance_with_detaches_and_warns_on_reuse():
    """advance_with(None) hands the step counter back to the loader: batches then
    advance it themselves; a second eager batch without an optimizer step in between warns."""
    import cs744_distributed_data_parallel_amd as cdp
    from cs744_distributed_data_parallel_amd.data import DeviceLoader, synthetic_cifar10

    model = cdp.VGG11().cuda()
    opt = cdp.SGD(model.parameters(), lr=0.1, momentum=0.9)
    loader = DeviceLoader(synthetic_cifar10(256, seed=0, device=torch.device("cuda")), 32, shuffle=True)
    order = loader._order()
    assert loader.advance_with(opt)
    loader.batch(order, 0, 32, nbatches=8)
    with pytest.warns(UserWarning, match="two batches without an optimizer step"):
        loader.batch(order, 0, 32, nbatches=8)
    c0 = int(loader._counter.item())
    assert loader.advance_with(None) and opt._step_counter is None
    loader.batch(order, 0, 32, nbatches=8)
    loader.batch(order, 0, 32, nbatches=8)
    assert int(loader._counter.item()) == c0 + 2
