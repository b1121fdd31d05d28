"""ResNet-50 numerics at the bench's shapes (BASELINE.json config #5; the DDP model of
``/root/reference/src/Part 3/main.py:61`` at ImageNet scale).

1. Every distinct ResNet-50 convolution at the bench's 64 x 224^2 -- the 7x7/s2 stem, the 1x1 GEMMs
   (stride 1 and the stride-2 downsamples), the 3x3 convs (stride 1 and 2) -- runs its forward, data
   gradient and weight gradient through the native entry points, i.e. through the planner's own
   tile / split-K choices at this batch (csrc/runtime/ops.cpp plan_gemm / plan_wgrad and the tuned
   tables), and every checked output must satisfy the fp32 dot-product bound of
   tests/test_accuracy_gpu.py against an fp64 reference: forward and data gradient on whole images
   (two of the 64; f16x2 scales rows per image, so the other images' presence still matters),
   weight gradient on whole rows of dW (a handful of output channels, reduced over all 64 images).
2. A 20-step ResNet-50 training run at 224^2 (batch 16) through the native engine follows the torch
   fp32 (MIOpen) loss trajectory from the same init within the band that fp32 rounding noise itself
   opens (a torch run from an init perturbed by 2^-23 relative).
"""
import pytest
import torch
import torch.nn.functional as F

from test_accuracy_gpu import C, _check, _train, cl

pytestmark = pytest.mark.gpu

B = 64


def _resnet50_convs():
    """(Ci, H, W, Co, k, stride, pad) of every distinct conv of ResNet-50 at 224^2, in model order."""
    import cs744_distributed_data_parallel_amd as cdp

    m = cdp.get_model("resnet50", channels_last=False)
    seen, out = set(), []

    def hook(mod, inp, _out):
        x = inp[0]
        key = (x.shape[1], x.shape[2], x.shape[3], mod.out_channels, mod.kernel_size[0], mod.stride[0],
               mod.padding[0])
        if key not in seen:
            seen.add(key)
            out.append(key)

    hs = [mm.register_forward_hook(hook) for mm in m.modules() if isinstance(mm, torch.nn.Conv2d)]
    import os

    prev = os.environ.get("CDP_FORCE_REFERENCE")
    os.environ["CDP_FORCE_REFERENCE"] = "1"
    try:
        with torch.no_grad():
            m.eval()(torch.zeros(1, 3, 224, 224))
    finally:
        if prev is None:
            os.environ.pop("CDP_FORCE_REFERENCE", None)
        else:
            os.environ["CDP_FORCE_REFERENCE"] = prev
    for h in hs:
        h.remove()
    return out


CONVS = _resnet50_convs()


def test_resnet50_conv_inventory():
    """The stem, 1x1 (stride 1 and 2), 3x3 (stride 1 and 2) classes are all in the list."""
    kinds = {(k, s) for _, _, _, _, k, s, _ in CONVS}
    assert {(7, 2), (1, 1), (1, 2), (3, 1), (3, 2)} <= kinds, kinds
    assert len(CONVS) >= 20, len(CONVS)


@pytest.mark.parametrize("engine", ["f16x2", "x3"])
@pytest.mark.parametrize("Ci,H,W,Co,k,s,p", CONVS, ids=[f"{c[0]}x{c[1]}-{c[3]}k{c[4]}s{c[5]}" for c in CONVS])
def test_resnet50_bench_shape_gemms_meet_fp32_bound(engine, Ci, H, W, Co, k, s, p):
    gen = torch.Generator(device="cuda").manual_seed(Ci * 7 + Co + k * 13 + s)
    x = torch.randn(B, Ci, H, W, device="cuda", generator=gen)
    w = torch.randn(Co, Ci, k, k, device="cuda", generator=gen) * (1.0 / (Ci * k * k) ** 0.5)
    P = (H + 2 * p - k) // s + 1
    Q = (W + 2 * p - k) // s + 1
    gy = torch.randn(B, Co, P, Q, device="cuda", generator=gen)
    orig = C().get_conv_gemm()
    try:
        C().set_conv_gemm(engine)
        y = C().conv2d_fwd(cl(x), cl(w), None, s, p, False)[0]
        dx = C().conv2d_dgrad(cl(gy), cl(w), list(x.shape), s, p)
        dw = C().conv2d_wgrad(cl(gy), cl(x), list(w.shape), s, p)
        torch.cuda.synchronize()
    finally:
        C().set_conv_gemm(orig)
    assert y.shape == (B, Co, P, Q) and dx.shape == x.shape and dw.shape == w.shape
    xd, wd, gyd = x.double(), w.double(), gy.double()
    imgs = torch.tensor([5, B - 3], device="cuda")
    # forward and data gradient of two whole images (exact fp64 conv / its transpose, and the
    # sum_i |a_i| |b_i| of every output from the absolute values)
    xs = xd[imgs].clone().requires_grad_()
    F.conv2d(xs, wd, None, s, p).backward(gyd[imgs])
    xa = torch.zeros_like(xd[imgs], requires_grad=True)
    F.conv2d(xa, wd.abs(), None, s, p).backward(gyd[imgs].abs())
    ratios = [
        _check("fwd", y[imgs], F.conv2d(xd[imgs], wd, None, s, p).cpu(),
               F.conv2d(xd[imgs].abs(), wd.abs(), None, s, p).cpu(), Ci * k * k),
        _check("dgrad", dx[imgs], xs.grad.cpu(), xa.grad.cpu(), Co * k * k),
    ]
    # weight gradient: whole rows of dW for a few output channels, reduced over every image / pixel
    nrow = max(1, min(Co, 4096 // (Ci * k * k) + 1))
    rows = torch.randperm(Co, device="cuda", generator=gen)[:nrow]
    xu = F.unfold(xd, k, padding=p, stride=s)  # [B, Ci*k*k, P*Q]
    g_sel = gyd[:, rows].reshape(B, nrow, -1)
    ref = torch.einsum("bkp,bcp->ck", xu, g_sel)
    absref = torch.einsum("bkp,bcp->ck", xu.abs(), g_sel.abs())
    del xu
    ratios.append(_check("wgrad", dw[rows].reshape(nrow, -1), ref.cpu(), absref.cpu(), B * P * Q))
    print(f"{engine} {(Ci, H, W, Co, k, s, p)}: worst err/bound fwd {ratios[0]:.2e} dgrad {ratios[1]:.2e} "
          f"wgrad {ratios[2]:.2e}")


def test_resnet50_loss_trajectory_tracks_torch_fp32():
    import cs744_distributed_data_parallel_amd as cdp

    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    steps, nb = 20, 16
    g = torch.Generator().manual_seed(5)
    proj = torch.randn(10, 3 * 8 * 8, generator=g)
    xs, ys = [], []
    for _ in range(4):  # a learnable task: label = argmax of a projection of the 8x8-pooled image
        x = torch.randn(nb, 3, 224, 224, generator=g)
        xs.append(x)
        ys.append((F.adaptive_avg_pool2d(x, 8).reshape(nb, -1) @ proj.t()).argmax(1))
    xs, ys = [xs[i % 4] for i in range(steps)], [ys[i % 4] for i in range(steps)]
    torch.manual_seed(0)
    init = {k: v.clone() for k, v in cdp.get_model("resnet50", num_classes=10, channels_last=False)
            .state_dict().items()}

    def torch_run(perturb):
        m = cdp.get_model("resnet50", num_classes=10, channels_last=False)
        m.load_state_dict(init)
        if perturb:
            gp = torch.Generator().manual_seed(11)
            with torch.no_grad():
                for prm in m.parameters():
                    prm.mul_(1 + 2.0 ** -23 * torch.randn(prm.shape, generator=gp))
        m = m.cuda()
        opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        return _train(m, opt, torch.nn.CrossEntropyLoss(), xs, ys, reference=True)

    ref = torch_run(False)
    pert = torch_run(True)
    m = cdp.get_model("resnet50", num_classes=10)
    m.load_state_dict(init)
    m = m.cuda()
    opt = cdp.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    nat = _train(m, opt, cdp.CrossEntropyLoss(), xs, ys, reference=False)
    noise = (pert - ref).abs()
    dev = (nat - ref).abs()
    print(f"resnet50: loss ref {ref[0]:.4f} -> {ref[-1]:.4f}, native {nat[0]:.4f} -> {nat[-1]:.4f}; "
          f"mean |native-ref| {dev.mean():.2e} vs fp32-noise {noise.mean():.2e}; max {dev.max():.2e} vs {noise.max():.2e}")
    assert torch.isfinite(nat).all()
    # the first step sees identical weights: rounding-level agreement
    assert dev[0] <= 1e-4 * ref[0].abs() + 1e-5, dev[:3]
    assert dev.mean() <= 3.0 * noise.mean() + 0.02, (dev.mean(), noise.mean())
