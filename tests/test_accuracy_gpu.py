"""fp32-class accuracy of the conv GEMM engines, per element and over a training run.

1. Per element: every output of the forward, data-gradient and weight-gradient GEMMs must satisfy
   the fp32 dot-product error bound

       |y - y_fp64| <= c * (2^-22 + K * 2^-24) * sum_i |a_i| |b_i|        (c = 4)

   where K is the reduction length (Ci*k*k forward, Co*k*k dgrad, N*P*Q wgrad). Global RMS or
   max-normalised errors (tests/test_kernels_gpu.py) are dominated by the large outputs and cannot
   see an output whose inputs all sit far below the tensor maximum; this bound can. Data: Gaussian,
   heavy-tailed (log-normal magnitudes), and structured dynamic range -- whole images or whole
   channels scaled down by up to 2^-42 (e.g. the loss gradient of confidently classified images).
2. Over a run: VGG-11 trained 100 steps at the reference hyperparameters (lr 0.1, momentum 0.9,
   wd 1e-4, B=256; /root/reference/src/Part 1/main.py:114-115) through the native engine follows
   the torch fp32 (MIOpen) loss curve from the same init as closely as fp32 rounding noise itself
   allows (a torch run from an init perturbed by 2^-23 relative sets the band).
"""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

ENGINES = ["f16x2", "x3", "f32"]

CASES = [
    # N, C, H, W, Co, k, s, p
    (8, 3, 32, 32, 64, 3, 1, 1),      # VGG layer 0 (K = 27)
    (8, 64, 16, 16, 128, 3, 1, 1),    # VGG layer 1
    (8, 128, 8, 8, 256, 3, 1, 1),
    (8, 256, 8, 8, 256, 3, 1, 1),
    (8, 256, 4, 4, 512, 3, 1, 1),
    (8, 512, 2, 2, 512, 3, 1, 1),     # split-K regime
    (3, 64, 14, 14, 64, 1, 1, 0),     # 1x1, M tail
    (2, 64, 15, 15, 128, 3, 2, 1),    # strided 3x3, odd size
    (2, 128, 14, 14, 256, 1, 2, 0),   # 1x1 stride-2 downsample
    (2, 3, 64, 64, 64, 7, 2, 3),      # ResNet stem
]


def C():
    import cs744_distributed_data_parallel_amd as cdp

    return cdp._native.lib()


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def _data(kind, shape, gen):
    t = torch.randn(shape, generator=gen, dtype=torch.float64)
    if kind == "heavy":
        t = t * torch.exp(2.0 * torch.randn(shape, generator=gen, dtype=torch.float64))
    elif kind == "image_spread":  # image n scaled by 2^(-42 n / (N-1)): the last one by 2^-42
        n = shape[0]
        t = t * torch.pow(2.0, -42.0 * torch.arange(n, dtype=torch.float64) / max(1, n - 1)).view(-1, 1, 1, 1)
    elif kind == "channel_spread":  # channel c scaled by 2^(-(3c mod 43))
        t = t * torch.pow(2.0, -((3.0 * torch.arange(shape[1], dtype=torch.float64)) % 43)).view(1, -1, 1, 1)
    return t.float()


def _check(name, got, ref, absref, K):
    c = 4.0
    bound = c * (2.0 ** -22 + K * 2.0 ** -24) * absref + 1e-300
    err = (got.double().cpu() - ref).abs()
    ratio = (err / bound).max().item()
    assert ratio <= 1.0, f"{name}: worst |err|/bound = {ratio:.3g} (K={K})"
    return ratio


F16X2_LIMIT = pytest.mark.xfail(
    strict=True,
    reason="documented f16x2 limitation (docs/PERF.md 'f16x2 accuracy envelope'): operand scales are "
           "per tensor, so a whole image / channel sitting more than ~2^18 below the tensor max loses "
           "its low fp16 term and gets an absolute error floor of 2^-40 max|x| -- outside the fp32 "
           "per-element bound for those outputs. x3 and f32 meet the bound here.")


def _kinds_for(engine):
    out = []
    for kind in ["normal", "heavy", "image_spread", "channel_spread"]:
        marks = [F16X2_LIMIT] if (engine == "f16x2" and kind.endswith("_spread")) else []
        out.append(pytest.param(engine, kind, marks=marks, id=f"{engine}-{kind}"))
    return out


@pytest.mark.parametrize("engine,kind", [p for e in ENGINES for p in _kinds_for(e)])
@pytest.mark.parametrize("N,Ci,H,W,Co,k,s,p", CASES)
def test_conv_gemms_meet_fp32_error_bound_per_element(engine, kind, N, Ci, H, W, Co, k, s, p):
    gen = torch.Generator().manual_seed(7)
    x = _data(kind, (N, Ci, H, W), gen)
    w = (torch.randn(Co, Ci, k, k, generator=gen) * (1.0 / (Ci * k * k) ** 0.5)).float()
    xd, wd = x.double(), w.double()
    y_ref = F.conv2d(xd, wd, None, s, p)
    P, Q = y_ref.shape[2], y_ref.shape[3]
    gy = _data(kind, tuple(y_ref.shape), gen)
    gyd = gy.double()
    # exact fp64 references and the sum_i |a_i||b_i| of every output
    xr = xd.clone().requires_grad_()
    wr = wd.clone().requires_grad_()
    F.conv2d(xr, wr, None, s, p).backward(gyd)
    abs_y = F.conv2d(xd.abs(), wd.abs(), None, s, p)
    xa = torch.zeros_like(xd, requires_grad=True)
    F.conv2d(xa, wd.abs(), None, s, p).backward(gyd.abs())
    wa = torch.zeros_like(wd, requires_grad=True)
    F.conv2d(xd.abs(), wa, None, s, p).backward(gyd.abs())

    xc, wc, gyc = cl(x.cuda()), cl(w.cuda()), cl(gy.cuda())
    orig = C().get_conv_gemm()
    try:
        C().set_conv_gemm(engine)
        y = C().conv2d_fwd(xc, wc, None, s, p, False)[0]
        dx = C().conv2d_dgrad(gyc, wc, list(x.shape), s, p)
        dw = C().conv2d_wgrad(gyc, xc, list(w.shape), s, p)
        torch.cuda.synchronize()
    finally:
        C().set_conv_gemm(orig)
    r = (_check("fwd", y, y_ref, abs_y, Ci * k * k),
         _check("dgrad", dx, xr.grad, xa.grad, Co * k * k),
         _check("wgrad", dw, wr.grad, wa.grad, N * P * Q))
    print(f"{engine} {kind} {(N, Ci, H, W, Co, k, s, p)} worst err/bound fwd {r[0]:.2e} dgrad {r[1]:.2e} "
          f"wgrad {r[2]:.2e}")


# ------------------------------------------------------------------------------------- long run
def _synthetic_task(steps, B, gen, distinct=8):
    """Learnable CIFAR-shaped task: the label is the argmax of a fixed random projection of the
    4x4-average-pooled image; ``distinct`` batches are cycled (epochs over a small training set)."""
    proj = torch.randn(10, 3 * 4 * 4, generator=gen)
    xs, ys = [], []
    for _ in range(distinct):
        x = torch.randn(B, 3, 32, 32, generator=gen)
        feat = F.adaptive_avg_pool2d(x, 4).reshape(B, -1)
        xs.append(x)
        ys.append((feat @ proj.t()).argmax(1))
    return [xs[i % distinct] for i in range(steps)], [ys[i % distinct] for i in range(steps)]


def _train(model, opt, crit, xs, ys, reference):
    prev = os.environ.get("CDP_FORCE_REFERENCE")
    os.environ["CDP_FORCE_REFERENCE"] = "1" if reference else "0"
    losses = []
    try:
        model.train()
        for x, y in zip(xs, ys):
            x, y = x.cuda(non_blocking=True), y.cuda(non_blocking=True)
            if not reference:
                x = cl(x)
            opt.zero_grad()
            loss = crit(model(x), y)
            loss.backward()
            opt.step()
            losses.append(loss.detach())
        torch.cuda.synchronize()
    finally:
        if prev is None:
            os.environ.pop("CDP_FORCE_REFERENCE", None)
        else:
            os.environ["CDP_FORCE_REFERENCE"] = prev
    return torch.stack(losses).double().cpu()


@pytest.mark.parametrize("engine", ["f16x2", "x3"])
def test_vgg11_loss_curve_tracks_torch_fp32(engine):
    import cs744_distributed_data_parallel_amd as cdp

    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    steps, B = 100, 256
    xs, ys = _synthetic_task(steps, B, torch.Generator().manual_seed(3))
    torch.manual_seed(0)
    init = {k: v.clone() for k, v in cdp.VGG11(channels_last=False).state_dict().items()}

    def torch_run(perturb):
        m = cdp.VGG11(channels_last=False)
        m.load_state_dict(init)
        if perturb:
            g = torch.Generator().manual_seed(11)
            with torch.no_grad():
                for prm in m.parameters():
                    prm.mul_(1 + 2.0 ** -23 * torch.randn(prm.shape, generator=g))
        m = m.cuda()
        opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        return _train(m, opt, torch.nn.CrossEntropyLoss(), xs, ys, reference=True)

    ref = torch_run(False)
    pert = torch_run(True)
    orig = C().get_conv_gemm()
    try:
        C().set_conv_gemm(engine)
        m = cdp.VGG11()
        m.load_state_dict(init)
        m = m.cuda()
        opt = cdp.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        nat = _train(m, opt, cdp.CrossEntropyLoss(), xs, ys, reference=False)
    finally:
        C().set_conv_gemm(orig)
    noise = (pert - ref).abs()
    dev = (nat - ref).abs()
    print(f"{engine}: loss ref {ref[0]:.4f} -> {ref[-1]:.4f}, native {nat[0]:.4f} -> {nat[-1]:.4f}; "
          f"mean |native-ref| {dev.mean():.2e} vs fp32-noise {noise.mean():.2e}; "
          f"max {dev.max():.2e} vs {noise.max():.2e}")
    assert torch.isfinite(nat).all()
    assert ref[-10:].mean() < ref[0]  # below the initial loss after the early lr-0.1 transient
    # the first two steps see (nearly) identical weights: rounding-level agreement (from step 3 on
    # the lr-0.1 transient amplifies any rounding difference, which is what the band is for)
    assert (dev[:2] <= 1e-4 * ref[:2].abs() + 1e-5).all(), dev[:5]
    # over the run: within the spread that fp32 rounding noise itself induces (+ a small floor)
    assert dev.mean() <= 3.0 * noise.mean() + 0.02, (dev.mean(), noise.mean())
    assert abs(nat[-10:].mean() - ref[-10:].mean()) <= 3.0 * (pert[-10:].mean() - ref[-10:].mean()).abs() + 0.05


# --------------------------------------------------------------------- headline GEMM plans
# VGG-11 layers 1-7 (layer 0 runs the exact-fp32 stem kernels, test_kernels_gpu.py) at the bench's
# batch (B=256) and at the reference's 8-rank strong-scaling batch (B=32): the conv entry points
# plan tiles and split-K exactly as the training step does (plan_gemm / plan_wgrad in
# csrc/runtime/ops.cpp), so these launches are the headline's GEMM configurations.
VGG_LAYERS = [(64, 128, 16), (128, 256, 8), (256, 256, 8), (256, 512, 4), (512, 512, 4), (512, 512, 2),
              (512, 512, 2)]


def _patches(xp, n, p, q):
    """[S, Ci*9] rows of the zero-padded input around output pixels (n, p, q), (ci, kh, kw) order."""
    idx_h = p[:, None] + torch.arange(3, device=xp.device)[None, :]
    idx_w = q[:, None] + torch.arange(3, device=xp.device)[None, :]
    g = xp[n[:, None, None, None], torch.arange(xp.shape[1], device=xp.device)[None, :, None, None],
           idx_h[:, None, :, None], idx_w[:, None, None, :]]
    return g.reshape(len(n), -1)


@pytest.mark.parametrize("engine", ["f16x2", "x3"])
@pytest.mark.parametrize("B", [256, 32])
@pytest.mark.parametrize("layer", range(1, 8))
def test_headline_plan_gemms_meet_fp32_bound_on_samples(engine, B, layer):
    Ci, Co, HW = VGG_LAYERS[layer - 1]
    gen = torch.Generator(device="cuda").manual_seed(100 + layer)
    x = torch.randn(B, Ci, HW, HW, device="cuda", generator=gen)
    w = torch.randn(Co, Ci, 3, 3, device="cuda", generator=gen) * (1.0 / (Ci * 9) ** 0.5)
    gy = torch.randn(B, Co, HW, HW, device="cuda", generator=gen)
    orig = C().get_conv_gemm()
    try:
        C().set_conv_gemm(engine)
        y = C().conv2d_fwd(cl(x), cl(w), None, 1, 1, False)[0]
        dx = C().conv2d_dgrad(cl(gy), cl(w), list(x.shape), 1, 1)
        dw = C().conv2d_wgrad(cl(gy), cl(x), list(w.shape), 1, 1)
        torch.cuda.synchronize()
    finally:
        C().set_conv_gemm(orig)
    xd, wd, gyd = x.double(), w.double(), gy.double()
    S = 4096 // Co + 1  # output pixels sampled for fwd (x Co columns >= 4096 outputs)
    n = torch.randint(0, B, (S,), device="cuda", generator=gen)
    p = torch.randint(0, HW, (S,), device="cuda", generator=gen)
    q = torch.randint(0, HW, (S,), device="cuda", generator=gen)
    # forward: y[n, :, p, q] = patches(x) @ W^T
    px = _patches(F.pad(xd, (1, 1, 1, 1)), n, p, q)
    wm = wd.reshape(Co, -1)
    ratios = [_check("fwd", y[n, :, p, q], (px @ wm.t()).cpu(), (px.abs() @ wm.abs().t()).cpu(), Ci * 9)]
    # data gradient: a stride-1 pad-1 conv of gy with the flipped, transposed filter
    S2 = 4096 // Ci + 1
    n2 = torch.randint(0, B, (S2,), device="cuda", generator=gen)
    p2 = torch.randint(0, HW, (S2,), device="cuda", generator=gen)
    q2 = torch.randint(0, HW, (S2,), device="cuda", generator=gen)
    pg = _patches(F.pad(gyd, (1, 1, 1, 1)), n2, p2, q2)
    wt = wd.flip(2, 3).transpose(0, 1).reshape(Ci, -1)
    ratios.append(_check("dgrad", dx[n2, :, p2, q2], (pg @ wt.t()).cpu(), (pg.abs() @ wt.abs().t()).cpu(), Co * 9))
    # weight gradient: whole rows of dW for a few output channels, reduction over all B*HW*HW pixels
    rows = torch.randperm(Co, device="cuda", generator=gen)[: 4096 // (Ci * 9) + 1]
    xu = F.unfold(xd, 3, padding=1)  # [B, Ci*9, HW*HW]
    g_sel = gyd[:, rows].reshape(B, len(rows), -1)
    ref = torch.einsum("bkp,bcp->ck", xu, g_sel)
    absref = torch.einsum("bkp,bcp->ck", xu.abs(), g_sel.abs())
    ratios.append(_check("wgrad", dw[rows].reshape(len(rows), -1), ref.cpu(), absref.cpu(), B * HW * HW))
    print(f"{engine} B={B} layer {layer}: worst err/bound fwd {ratios[0]:.2e} dgrad {ratios[1]:.2e} "
          f"wgrad {ratios[2]:.2e}")
