"""Numerics of every HIP kernel against a plain PyTorch fp32/fp64 reference of the same op.

Shapes follow the VGG-11 launch inventory at reduced batch, plus the ResNet-50
cases (stride 2, 1x1, 7x7 stem) and awkward tails (K = 27, M not a multiple of the tile).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def C():
    import cs744_distributed_data_parallel_amd as cdp

    return cdp._native.lib()


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


CONV_CASES = [
    # N, C, H, W, Co, k, s, p
    (8, 3, 32, 32, 64, 3, 1, 1),      # VGG layer 0 (K = 27 generic gather)
    (8, 64, 16, 16, 128, 3, 1, 1),    # VGG layer 1
    (4, 128, 8, 8, 256, 3, 1, 1),
    (4, 256, 8, 8, 256, 3, 1, 1),
    (4, 256, 4, 4, 512, 3, 1, 1),
    (4, 512, 2, 2, 512, 3, 1, 1),     # split-K regime
    (3, 64, 14, 14, 64, 1, 1, 0),     # 1x1, M tail
    (2, 64, 15, 15, 128, 3, 2, 1),    # strided 3x3, odd size
    (2, 128, 14, 14, 256, 1, 2, 0),   # 1x1 stride-2 downsample
    (2, 3, 64, 64, 64, 7, 2, 3),      # ResNet stem
]


@pytest.mark.parametrize("N,Ci,H,W,Co,k,s,p", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(N, Ci, H, W, Co, k, s, p):
    torch.manual_seed(0)
    dev = "cuda"
    x = torch.randn(N, Ci, H, W, device=dev)
    w = torch.randn(Co, Ci, k, k, device=dev) * (1.0 / (Ci * k * k) ** 0.5)
    b = torch.randn(Co, device=dev)
    y = C().conv2d_fwd(cl(x), cl(w), b, s, p, False)[0]
    ref = F.conv2d(x.double().cpu(), w.double().cpu(), b.double().cpu(), s, p)
    assert y.shape == ref.shape
    assert rel_err(y, ref) < 2e-5
    gy = torch.randn_like(y)
    xr = x.double().cpu().requires_grad_()
    wr = w.double().cpu().requires_grad_()
    F.conv2d(xr, wr, None, s, p).backward(gy.double().cpu())
    dx = C().conv2d_dgrad(cl(gy), cl(w), list(x.shape), s, p)
    assert rel_err(dx, xr.grad) < 2e-5
    dw = C().conv2d_wgrad(cl(gy), cl(x), list(w.shape), s, p)
    assert rel_err(dw, wr.grad) < 2e-5


@pytest.mark.parametrize("N,Ci,H,W,Co,k,s,p", [
    (4, 64, 28, 28, 256, 1, 1, 0),   # full tiles and an M tail through the wide epilogue loads
    (2, 64, 56, 56, 64, 3, 1, 1),
    (2, 128, 14, 14, 256, 1, 2, 0),  # stride 2: sub-pixel classes, tap-less ones skipped
    (3, 64, 14, 14, 64, 1, 1, 0),
])
def test_conv_dgrad_accumulates_into_addend(N, Ci, H, W, Co, k, s, p):
    """dX += dgrad in place (the parked residual gradient of a ResNet block): the epilogue's addend
    loads (16-B rows through LDS on full tiles, per element on edge tiles) before any store."""
    torch.manual_seed(3)
    dev = "cuda"
    x = torch.randn(N, Ci, H, W, device=dev)
    w = torch.randn(Co, Ci, k, k, device=dev) * (1.0 / (Ci * k * k) ** 0.5)
    xr = x.double().cpu().requires_grad_()
    y = F.conv2d(xr, w.double().cpu(), None, s, p)
    gy = torch.randn(y.shape, dtype=torch.float64)
    y.backward(gy)
    base = cl(torch.randn(N, Ci, H, W, device=dev))
    ref = xr.grad + base.double().cpu()
    acc = base.clone()
    dx = C().conv2d_dgrad(cl(gy.float().to(dev)), cl(w), list(x.shape), s, p, acc)
    assert dx.data_ptr() == acc.data_ptr()
    assert rel_err(dx, ref) < 2e-5


def test_conv_bn_stats_match_batchnorm():
    torch.manual_seed(1)
    x = torch.randn(16, 64, 16, 16, device="cuda")
    w = torch.randn(128, 64, 3, 3, device="cuda") * 0.05
    b = torch.randn(128, device="cuda")
    y, part, rpp = C().conv2d_fwd(cl(x), cl(w), b, 1, 1, True)
    ref = F.conv2d(x.double(), w.double(), b.double(), 1, 1)
    mean_ref = ref.mean((0, 2, 3))
    var_ref = ref.var((0, 2, 3), unbiased=False)
    # merge partials on the host (Chan)
    n = int(rpp.item())
    M = y.shape[0] * y.shape[2] * y.shape[3]
    cnt = torch.tensor([min(n, M - i * n) for i in range(part.shape[0])], dtype=torch.float64, device="cuda")
    pm, pq = part[..., 0].double(), part[..., 1].double()
    mean = (cnt[:, None] * pm).sum(0) / M
    m2 = pq.sum(0) + (cnt[:, None] * (pm - mean) ** 2).sum(0)
    assert torch.allclose(mean, mean_ref, rtol=1e-5, atol=1e-6)
    assert torch.allclose(m2 / M, var_ref, rtol=1e-5, atol=1e-6)


BLOCK_CASES = [
    (8, 3, 32, 32, 64, True),
    (8, 64, 16, 16, 128, True),
    (4, 128, 8, 8, 256, False),
    (4, 512, 2, 2, 512, True),
    (4, 512, 4, 4, 512, False),
    (2, 64, 7, 7, 64, True),  # odd map under pooling: separate conv-bias partial pass
]


@pytest.mark.parametrize("N,Ci,H,W,Co,pool", BLOCK_CASES)
@pytest.mark.parametrize("training", [True, False])
def test_fused_block_matches_torch(N, Ci, H, W, Co, pool, training):
    import cs744_distributed_data_parallel_amd as cdp
    from cs744_distributed_data_parallel_amd.ops import functional as CF

    torch.manual_seed(2)
    conv = torch.nn.Conv2d(Ci, Co, 3, 1, 1).cuda()
    bn = torch.nn.BatchNorm2d(Co).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.1, 0.1)
        bn.running_var.uniform_(0.5, 1.5)
    conv_r = torch.nn.Conv2d(Ci, Co, 3, 1, 1).double()
    bn_r = torch.nn.BatchNorm2d(Co).double()
    conv_r.load_state_dict(conv.state_dict())
    bn_r.load_state_dict(bn.state_dict())
    conv.weight.data = cl(conv.weight.data)
    bn.train(training)
    bn_r.train(training)
    x = torch.randn(N, Ci, H, W, device="cuda")
    xn = cl(x).requires_grad_()
    out = CF.conv_bn_act(xn, conv, bn, relu=True, pool=pool)
    xr = x.double().cpu().requires_grad_()
    ref = F.relu(bn_r(conv_r(xr)))
    if pool:
        ref = F.max_pool2d(ref, 2, 2)
    assert rel_err(out, ref) < 5e-5
    g = torch.randn_like(out)
    out.backward(g)
    ref.backward(g.double().cpu())
    assert rel_err(xn.grad, xr.grad) < 5e-4
    assert rel_err(conv.weight.grad, conv_r.weight.grad) < 5e-4
    assert rel_err(bn.weight.grad, bn_r.weight.grad) < 5e-4
    assert rel_err(bn.bias.grad, bn_r.bias.grad) < 5e-4
    assert (conv.bias.grad.double().cpu() - conv_r.bias.grad).abs().max().item() < 1e-3 * (
        conv_r.bias.grad.abs().max().item() + g.abs().mean().item())
    if training:
        assert rel_err(bn.running_mean, bn_r.running_mean) < 1e-5
        assert rel_err(bn.running_var, bn_r.running_var) < 1e-5
        assert int(bn.num_batches_tracked) == int(bn_r.num_batches_tracked) == 1


@pytest.mark.parametrize("N,H,W,x_grad", [(8, 32, 32, False), (3, 10, 6, False), (4, 8, 8, True)])
def test_rgb_stem_block_matches_torch(N, H, W, x_grad):
    """VGG layer 0 (Cin = 3): exact-fp32 stem forward (stem_fwd_kernel) and, without an input
    gradient, the weight gradient with the BN/ReLU/pool backward applied on the fly
    (stem_wgrad_kernel) against fp64 torch."""
    from cs744_distributed_data_parallel_amd.ops import functional as CF

    torch.manual_seed(5)
    conv = torch.nn.Conv2d(3, 64, 3, 1, 1).cuda()
    bn = torch.nn.BatchNorm2d(64).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    conv_r = torch.nn.Conv2d(3, 64, 3, 1, 1).double()
    bn_r = torch.nn.BatchNorm2d(64).double()
    conv_r.load_state_dict(conv.state_dict())
    bn_r.load_state_dict(bn.state_dict())
    conv.weight.data = cl(conv.weight.data)
    x = torch.randn(N, 3, H, W, device="cuda")
    xn = cl(x).requires_grad_(x_grad)
    out = CF.conv_bn_act(xn, conv, bn, relu=True, pool=True)
    xr = x.double().cpu().requires_grad_(x_grad)
    ref = F.max_pool2d(F.relu(bn_r(conv_r(xr))), 2, 2)
    assert rel_err(out, ref) < 1e-5
    g = torch.randn_like(out)
    out.backward(g)
    ref.backward(g.double().cpu())
    if x_grad:
        assert rel_err(xn.grad, xr.grad) < 5e-4
    assert rel_err(conv.weight.grad, conv_r.weight.grad) < 5e-5
    assert rel_err(bn.weight.grad, bn_r.weight.grad) < 5e-5
    assert rel_err(bn.bias.grad, bn_r.bias.grad) < 5e-5
    assert (conv.bias.grad.double().cpu() - conv_r.bias.grad).abs().max().item() < 1e-3 * (
        conv_r.bias.grad.abs().max().item() + g.abs().mean().item())
    assert rel_err(bn.running_mean, bn_r.running_mean) < 1e-5
    assert rel_err(bn.running_var, bn_r.running_var) < 1e-5


def test_residual_block_no_pool():
    from cs744_distributed_data_parallel_amd.ops import functional as CF

    torch.manual_seed(3)
    conv = torch.nn.Conv2d(64, 64, 1, 1, 0, bias=False).cuda()
    bn = torch.nn.BatchNorm2d(64).cuda()
    conv.weight.data = cl(conv.weight.data)
    x = torch.randn(4, 64, 8, 8, device="cuda")
    r = torch.randn(4, 64, 8, 8, device="cuda")
    xn, rn = cl(x).requires_grad_(), cl(r).requires_grad_()
    out = CF.conv_bn_act(xn, conv, bn, relu=True, residual=rn)
    conv_r = torch.nn.Conv2d(64, 64, 1, 1, 0, bias=False).double()
    conv_r.weight.data = conv.weight.data.double().cpu().contiguous()
    bn_r = torch.nn.BatchNorm2d(64).double()
    xr, rr = x.double().cpu().requires_grad_(), r.double().cpu().requires_grad_()
    ref = F.relu(bn_r(conv_r(xr)) + rr)
    assert rel_err(out, ref) < 5e-5
    g = torch.randn_like(out)
    out.backward(g)
    ref.backward(g.double().cpu())
    assert rel_err(rn.grad, rr.grad) < 1e-5
    assert rel_err(xn.grad, xr.grad) < 5e-4


@pytest.mark.parametrize("B,I,O", [(256, 512, 10), (33, 2048, 1000)])
def test_linear(B, I, O):
    from cs744_distributed_data_parallel_amd.ops import functional as CF

    torch.manual_seed(4)
    x = torch.randn(B, I, device="cuda", requires_grad=True)
    w = (torch.randn(O, I, device="cuda") * 0.05).requires_grad_()
    b = torch.randn(O, device="cuda", requires_grad=True)
    y = CF.linear(x, w, b)
    xr, wr, br = (t.detach().double().cpu().requires_grad_() for t in (x, w, b))
    ref = F.linear(xr, wr, br)
    assert rel_err(y, ref) < 2e-5
    g = torch.randn_like(y)
    y.backward(g)
    ref.backward(g.double().cpu())
    for a, r in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert rel_err(a, r) < 2e-5


@pytest.mark.parametrize("B,K", [(256, 10), (64, 1000), (37, 1000), (5, 100), (3, 2000)])
def test_cross_entropy_and_accuracy(B, K):
    """Softmax cross-entropy (one thread per row for <= 64 classes, four rows per wave for <= 1024,
    one row per wave beyond) and the correct count, against torch in fp64."""
    from cs744_distributed_data_parallel_amd.ops import functional as CF

    torch.manual_seed(5)
    logits = (3 * torch.randn(B, K, device="cuda")).requires_grad_()
    t = torch.randint(0, K, (B,), device="cuda")
    loss = CF.cross_entropy(logits, t)
    lr = logits.detach().double().cpu().requires_grad_()
    ref = F.cross_entropy(lr, t.cpu())
    assert abs(loss.item() - ref.item()) < 1e-5
    loss.backward()
    ref.backward()
    assert rel_err(logits.grad, lr.grad) < 1e-5
    c = CF.count_correct(logits.detach(), t)
    assert int(c.item()) == int(logits.detach().max(1)[1].eq(t).sum().item())


def test_sgd_matches_torch():
    import cs744_distributed_data_parallel_amd as cdp

    torch.manual_seed(6)
    m1 = cdp.VGG11().cuda()
    m2 = cdp.VGG11(channels_last=False)
    m2.load_state_dict({k: v.cpu() for k, v in m1.state_dict().items()})
    o1 = cdp.SGD(m1.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    o2 = torch.optim.SGD(m2.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    for step in range(3):
        for p1, p2 in zip(m1.parameters(), m2.parameters()):
            g = torch.randn(p2.shape)
            p2.grad = g.clone()
            p1.grad.copy_(g.to(p1.device))
        o1.step()
        o2.step()
        for p1, p2 in zip(m1.parameters(), m2.parameters()):
            assert torch.allclose(p1.detach().cpu(), p2.detach(), rtol=1e-6, atol=1e-7)
    # torch-compatible optimizer state layout
    sd = o1.state_dict()
    assert set(sd["state"][0].keys()) == {"momentum_buffer"}


def test_augment_normalize_and_determinism():
    import cs744_distributed_data_parallel_amd as cdp
    from cs744_distributed_data_parallel_amd.data import DeviceLoader, synthetic_cifar10

    ds = synthetic_cifar10(64, device="cuda")
    ld = DeviceLoader(ds, 16, train=False)
    x, y = next(iter(ld))
    ref = (ds.images[:16].permute(0, 3, 1, 2).float() / 255.0 - torch.tensor(ds.mean, device="cuda").view(1, 3, 1, 1)) \
        / torch.tensor(ds.std, device="cuda").view(1, 3, 1, 1)
    assert torch.allclose(x, ref, atol=1e-5)
    assert torch.equal(y, ds.labels[:16])
    lt = DeviceLoader(ds, 16, train=True, seed=3)
    a, _ = next(iter(lt))
    lt2 = DeviceLoader(ds, 16, train=True, seed=3)
    b, _ = next(iter(lt2))
    assert torch.equal(a, b)
    # every augmented image is a shifted / flipped copy: value range preserved
    assert a.shape == (16, 3, 32, 32) and a.is_contiguous(memory_format=torch.channels_last)


def test_augment_counter_driven_batches_in_graph():
    """nbatches > 0: one captured graph walks the epoch order by the on-device step counter, and the
    fused label gather matches labels[idx]."""
    from cs744_distributed_data_parallel_amd.data import DeviceLoader, synthetic_cifar10

    ds = synthetic_cifar10(64, device="cuda")
    ld = DeviceLoader(ds, 16, train=False)
    order = torch.randperm(64, generator=torch.Generator().manual_seed(1)).cuda()
    xs = torch.empty(16, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    ys = torch.empty(16, dtype=torch.int64, device="cuda")

    def body():
        x, y = ld.batch(order, 0, 16, out=xs, nbatches=4)
        ys.copy_(y)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()  # step 0
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()  # captured (not run): the first replay reads counter 1, each replay advances it
    mean = torch.tensor(ds.mean, device="cuda").view(1, 3, 1, 1)
    std = torch.tensor(ds.std, device="cuda").view(1, 3, 1, 1)
    for step in range(1, 7):
        g.replay()
        torch.cuda.synchronize()
        sel = order[(step % 4) * 16:(step % 4) * 16 + 16]
        ref = (ds.images[sel].permute(0, 3, 1, 2).float() / 255.0 - mean) / std
        assert torch.allclose(xs, ref, atol=1e-5), step
        assert torch.equal(ys, ds.labels[sel]), step


def test_pooling_ops():
    from cs744_distributed_data_parallel_amd.ops import functional as CF

    x = torch.randn(2, 64, 15, 15, device="cuda")
    xn = cl(x).requires_grad_()
    y = CF.max_pool2d(xn, 3, 2, 1)
    xr = x.double().cpu().requires_grad_()
    ref = F.max_pool2d(xr, 3, 2, 1)
    assert rel_err(y, ref) < 1e-6
    g = torch.randn_like(y)
    y.backward(g)
    ref.backward(g.double().cpu())
    assert rel_err(xn.grad, xr.grad) < 1e-6
    # ties (all-zero windows after a ReLU): the first max in scan order takes the gradient, as in ATen
    xt = torch.randn(2, 32, 16, 16, device="cuda").clamp_min(0.5) - 0.5
    xtn = cl(xt).requires_grad_()
    yt = CF.max_pool2d(xtn, 3, 2, 1)
    xtr = xt.double().cpu().requires_grad_()
    reft = F.max_pool2d(xtr, 3, 2, 1)
    gt = torch.randn_like(yt)
    yt.backward(gt)
    reft.backward(gt.double().cpu())
    assert rel_err(yt, reft) < 1e-6 and rel_err(xtn.grad, xtr.grad) < 1e-6
    # the backward's <= 2x2-window path (k <= 2s) and its general loop (k = 3, s = 1)
    for k, s, p in [(2, 2, 0), (3, 1, 1), (3, 2, 0)]:
        xk = torch.randn(2, 32, 9, 11, device="cuda")
        xkn = cl(xk).requires_grad_()
        yk = CF.max_pool2d(xkn, k, s, p)
        xkr = xk.double().cpu().requires_grad_()
        refk = F.max_pool2d(xkr, k, s, p)
        gk = torch.randn_like(yk)
        yk.backward(gk)
        refk.backward(gk.double().cpu())
        assert rel_err(yk, refk) < 1e-6 and rel_err(xkn.grad, xkr.grad) < 1e-6, (k, s, p)
    x2 = cl(torch.randn(4, 128, 7, 7, device="cuda")).requires_grad_()
    p = CF.global_avg_pool(x2)
    x2r = x2.detach().double().cpu().requires_grad_()
    pr = torch.flatten(F.adaptive_avg_pool2d(x2r, 1), 1)
    assert rel_err(p, pr) < 1e-6


def test_stack_mean_and_scale():
    srcs = [torch.randn(1000, device="cuda") for _ in range(4)]
    out = torch.empty(1000, device="cuda")
    C().stack_mean(srcs, out)
    assert torch.allclose(out, torch.stack(srcs).mean(0), atol=1e-6)
    C().scale_(out, 0.5)
    assert torch.allclose(out, torch.stack(srcs).mean(0) * 0.5, atol=1e-6)


def _rms_rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _heavy(shape, scale):
    """Wide-dynamic-range data (log-normal magnitudes spanning ~6 decades, random signs)."""
    return torch.randn(shape, device="cuda") * torch.exp(2.0 * torch.randn(shape, device="cuda")) * scale


@pytest.mark.parametrize("mode", ["x3", "f16x2"])
@pytest.mark.parametrize("N,Ci,H,W,Co,k,s,p", [CONV_CASES[i] for i in (0, 1, 3, 5, 7, 9)])
def test_split_engines_are_as_accurate_as_fp32_mfma(N, Ci, H, W, Co, k, s, p, mode):
    """The split engines (3-term bf16 "x3", scaled 2-term fp16 "f16x2") must match the exact
    fp32-input MFMA engine's error against fp64, for the forward, data- and weight-gradient GEMMs."""
    _engine_vs_f32(mode, N, Ci, H, W, Co, k, s, p, torch.randn)


@pytest.mark.parametrize("scale", [1e-12, 1e9])
def test_f16x2_scaling_wide_and_extreme_ranges(scale):
    """f16x2 operand scales: heavy-tailed magnitudes and values far outside fp16's range (tiny
    gradients, huge activations) keep fp32-level accuracy -- the power-of-two scales map every
    operand's max into fp16 range, and what falls below 2^-18 of it contributes only below the
    dot products' own fp32 rounding."""
    N, Ci, H, W, Co, k, s, p = CONV_CASES[3]
    _engine_vs_f32("f16x2", N, Ci, H, W, Co, k, s, p, lambda *sh, device: _heavy(sh, scale))


def _engine_vs_f32(mode, N, Ci, H, W, Co, k, s, p, gen):
    torch.manual_seed(1)
    x = gen(N, Ci, H, W, device="cuda")
    w = torch.randn(Co, Ci, k, k, device="cuda") * (1.0 / (Ci * k * k) ** 0.5)
    xr = x.double().cpu().requires_grad_()
    wr = w.double().cpu().requires_grad_()
    ref = F.conv2d(xr, wr, None, s, p)
    gy = gen(*ref.shape, device="cuda")
    ref.backward(gy.double().cpu())
    orig = C().get_conv_gemm()
    errs = {}
    try:
        for m in ("f32", mode):
            C().set_conv_gemm(m)
            y = C().conv2d_fwd(cl(x), cl(w), None, s, p, False)[0]
            dx = C().conv2d_dgrad(cl(gy), cl(w), list(x.shape), s, p)
            dw = C().conv2d_wgrad(cl(gy), cl(x), list(w.shape), s, p)
            errs[m] = (_rms_rel(y, ref.detach()), _rms_rel(dx, xr.grad), rel_err(y, ref.detach()),
                       _rms_rel(dw, wr.grad))
    finally:
        C().set_conv_gemm(orig)
    print(f"conv errs {mode} (rms fwd, rms dgrad, max fwd, rms wgrad)", errs)
    for i in range(4):
        assert errs[mode][i] <= 2.0 * errs["f32"][i] + 1e-9, errs
    assert max(errs[mode][0], errs[mode][1], errs[mode][3]) < 1e-6, errs


def test_bf16_engine_runs_at_bf16_accuracy():
    """CDP_CONV_GEMM=bf16 (non-parity fast mode): one bf16 product per MAC, fp32 accumulation."""
    torch.manual_seed(2)
    N, Ci, H, W, Co = 4, 128, 8, 8, 256
    x = torch.randn(N, Ci, H, W, device="cuda")
    w = torch.randn(Co, Ci, 3, 3, device="cuda") * (1.0 / (Ci * 9) ** 0.5)
    ref = F.conv2d(x.double().cpu(), w.double().cpu(), None, 1, 1)
    orig = C().get_conv_gemm()
    try:
        C().set_conv_gemm("bf16")
        assert C().get_conv_gemm() == "bf16"
        y = C().conv2d_fwd(cl(x), cl(w), None, 1, 1, False)[0]
        gy = torch.randn_like(y)
        dw = C().conv2d_wgrad(cl(gy), cl(x), list(w.shape), 1, 1)
    finally:
        C().set_conv_gemm(orig)
    e = _rms_rel(y, ref)
    assert 1e-5 < e < 1e-2, e  # bf16-level, clearly not fp32-level
    xr = x.double().cpu()
    wr = w.double().cpu().requires_grad_()
    F.conv2d(xr, wr, None, 1, 1).backward(gy.double().cpu())
    assert _rms_rel(dw, wr.grad) < 1e-2


def test_torch_custom_ops_with_autograd():
    """torch.ops.cdp.* (TORCH_LIBRARY registration) dispatch to the gfx950 kernels; conv2d and
    linear carry C++ autograd formulas."""
    C()  # loads the extension, which registers the ops
    torch.manual_seed(3)
    x = cl(torch.randn(4, 64, 8, 8, device="cuda")).requires_grad_()
    w = cl(torch.randn(128, 64, 3, 3, device="cuda") * 0.05).requires_grad_()
    b = torch.randn(128, device="cuda", requires_grad=True)
    y = torch.ops.cdp.conv2d(x, w, b, 1, 1)
    gy = torch.randn_like(y)
    y.backward(gy)
    xr, wr, br = (t.detach().double().cpu().requires_grad_() for t in (x, w, b))
    yr = F.conv2d(xr, wr, br, 1, 1)
    yr.backward(gy.double().cpu())
    assert rel_err(y, yr) < 2e-5
    for g, gr in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert rel_err(g, gr) < 2e-5
    xl = torch.randn(16, 512, device="cuda", requires_grad=True)
    wl = (torch.randn(10, 512, device="cuda") * 0.05).requires_grad_()
    yl = torch.ops.cdp.linear(xl, wl, None)
    yl.sum().backward()
    assert rel_err(yl, xl.detach().double().cpu() @ wl.detach().double().cpu().t()) < 2e-5
    assert rel_err(xl.grad, wl.detach().double().cpu().sum(0).expand(16, 512)) < 2e-5
    logits = torch.randn(32, 10, device="cuda")
    tgt = torch.randint(0, 10, (32,), device="cuda")
    assert abs(torch.ops.cdp.cross_entropy(logits, tgt).item() - F.cross_entropy(logits, tgt).item()) < 1e-5
    yp, arg = torch.ops.cdp.max_pool2d(cl(torch.randn(2, 32, 8, 8, device="cuda")), 2, 2, 0)
    assert yp.shape == (2, 32, 4, 4) and arg.dtype == torch.uint8


@pytest.mark.parametrize("N,Ci,H,W,Co,k,s,p", [CONV_CASES[i] for i in (4, 5, 7)])
def test_split_k_conv_is_deterministic_and_exact_order(N, Ci, H, W, Co, k, s, p):
    """Split-K shapes (in-kernel fixup: the last split of each tile sums the partial slabs in split
    order): repeated launches are bitwise identical, BN partials included, and match fp64."""
    torch.manual_seed(3)
    x = torch.randn(N, Ci, H, W, device="cuda")
    w = torch.randn(Co, Ci, k, k, device="cuda") * (1.0 / (Ci * k * k) ** 0.5)
    b = torch.randn(Co, device="cuda")
    outs = [C().conv2d_fwd(cl(x), cl(w), b, s, p, True) for _ in range(3)]
    gy = torch.randn_like(outs[0][0])
    dxs = [C().conv2d_dgrad(cl(gy), cl(w), list(x.shape), s, p) for _ in range(3)]
    for o in outs[1:]:
        assert torch.equal(o[0], outs[0][0]) and torch.equal(o[1], outs[0][1])
    for d in dxs[1:]:
        assert torch.equal(d, dxs[0])
    ref = F.conv2d(x.double().cpu(), w.double().cpu(), b.double().cpu(), s, p)
    assert rel_err(outs[0][0], ref) < 2e-5
    xr = x.double().cpu().requires_grad_()
    F.conv2d(xr, w.double().cpu(), None, s, p).backward(gy.double().cpu())
    assert rel_err(dxs[0], xr.grad) < 2e-5


def test_weight_prep_transposes_and_maxima():
    """One launch for all conv weights: W^T [Ci, KH*KW*Co] where asked, and (f16x2) the per-output-
    and per-input-channel |max| partials; dgrad with the prepared W^T equals dgrad without."""
    torch.manual_seed(4)
    ws = [cl(torch.randn(co, ci, k, k, device="cuda")) for co, ci, k in
          [(64, 3, 3), (128, 64, 3), (512, 512, 3), (256, 64, 1), (10, 7, 3), (64, 3, 7), (40, 36, 5)]]
    want = [False, True, True, True, True, True, True]  # 7x7 / 5x5: taps past one 9-tap load batch
    amax, wts = C().weight_prep(ws, want)
    for w, wt, f in zip(ws, wts, want):
        if not f:
            continue
        co, ci, kh, kw = w.shape
        ref = w.permute(1, 2, 3, 0).reshape(ci, kh * kw * co)  # [ci][kh][kw][co]
        assert torch.equal(wt, ref)
    if C().get_conv_gemm() == "f16x2":
        # per weight: the per-co partials of every 32-wide ci block, then the per-ci partials of
        # every 32-wide co block (csrc weight_max_elems), exact
        assert len(amax) == len(ws)
        for w, a in zip(ws, amax):
            co, ci = w.shape[:2]
            nci, nco = (ci + 31) // 32, (co + 31) // 32
            wa = w.abs()
            ref_co = torch.stack([wa[:, 32 * j:32 * (j + 1)].amax(dim=(1, 2, 3)) for j in range(nci)])
            ref_ci = torch.stack([wa[32 * j:32 * (j + 1)].amax(dim=(0, 2, 3)) for j in range(nco)])
            assert a.numel() == nci * co + nco * ci
            assert torch.equal(a[:nci * co].view(nci, co), ref_co)
            assert torch.equal(a[nci * co:].view(nco, ci), ref_ci)
    x = torch.randn(2, 128, 8, 8, device="cuda")
    gy = torch.randn(2, 512, 8, 8, device="cuda")
    w = ws[2]
    a = C().conv2d_dgrad(cl(gy), w, [2, 512, 8, 8], 1, 1)
    b = C().conv2d_dgrad(cl(gy), w, [2, 512, 8, 8], 1, 1, None, None, None, wts[2])
    assert torch.equal(a, b)
    del x
