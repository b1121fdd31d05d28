"""Fused head / tail launches of the small-batch step (the reference's augment -> conv1 and
fc1 -> CrossEntropyLoss, /root/reference/src/Part 1/main.py:82-93,110 and model.py:40-45), checked
against fp64 torch and against the unfused launches."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B", [32, 256, 7])
def test_fused_classifier_backward_matches_fp64(B, monkeypatch):
    """CrossEntropyLoss(Linear(x)) backward as ONE launch (xent_linear_bwd): dlogits, dx, dW, db match
    an fp64 torch reference to fp32 rounding and equal the two-launch path's values to a few ulps."""
    import cs744_distributed_data_parallel_amd as cdp
    from cs744_distributed_data_parallel_amd.ops import functional as CF

    g = torch.Generator(device="cuda").manual_seed(B)
    x0 = torch.randn(B, 512, device="cuda", generator=g)
    w0 = torch.randn(10, 512, device="cuda", generator=g) * 0.05
    b0 = torch.randn(10, device="cuda", generator=g)
    t = torch.randint(0, 10, (B,), device="cuda", generator=g)

    def run(fused):
        monkeypatch.setenv("CDP_FUSED_CLASSIFIER", "1" if fused else "0")
        x = x0.clone().requires_grad_()
        w = w0.clone().requires_grad_()
        b = b0.clone().requires_grad_()
        logits = CF.linear(x, w, b)
        logits.retain_grad()
        loss = CF.cross_entropy(logits, t)
        (loss * 0.5).backward()  # a non-unit incoming gradient
        torch.cuda.synchronize()
        return [logits.grad, x.grad, w.grad, b.grad]

    fz, un = run(True), run(False)
    xd = x0.double().requires_grad_()
    wd = w0.double().requires_grad_()
    bd = b0.double().requires_grad_()
    ld = F.linear(xd, wd, bd)
    ld.retain_grad()
    (F.cross_entropy(ld, t) * 0.5).backward()
    ref = [ld.grad, xd.grad, wd.grad, bd.grad]
    for name, a, u, r in zip(["dlogits", "dx", "dw", "db"], fz, un, ref):
        torch.testing.assert_close(a.double(), r, rtol=1e-5, atol=1e-7, msg=name)
        torch.testing.assert_close(a, u, rtol=1e-6, atol=1e-8, msg=name)
    assert cdp  # imported for the native library


def test_fused_classifier_falls_back_when_logits_have_a_second_consumer(monkeypatch):
    """The Linear's backward runs its own kernel when its incoming gradient is not the loss's alone."""
    from cs744_distributed_data_parallel_amd.ops import functional as CF

    monkeypatch.setenv("CDP_FUSED_CLASSIFIER", "1")
    g = torch.Generator(device="cuda").manual_seed(3)
    x0 = torch.randn(16, 512, device="cuda", generator=g)
    w0 = torch.randn(10, 512, device="cuda", generator=g) * 0.05
    t = torch.randint(0, 10, (16,), device="cuda", generator=g)
    x = x0.clone().requires_grad_()
    w = w0.clone().requires_grad_()
    logits = CF.linear(x, w, None)
    (CF.cross_entropy(logits, t) + logits.square().mean()).backward()
    xd = x0.double().requires_grad_()
    wd = w0.double().requires_grad_()
    ld = F.linear(xd, wd)
    (F.cross_entropy(ld, t) + ld.square().mean()).backward()
    torch.testing.assert_close(x.grad.double(), xd.grad, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(w.grad.double(), wd.grad, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("B", [32, 256])
def test_vgg11_fused_classifier_takes_the_last_blocks_bn_reduction(B, monkeypatch):
    """In a VGG-11 step the fused classifier backward also reduces the last block's BN backward
    statistics from the dX it forms (one hand-off more than with the unfused classifier), and every
    gradient matches the unfused path's."""
    import cs744_distributed_data_parallel_amd as cdp
    from cs744_distributed_data_parallel_amd.ops import functional as CF

    torch.manual_seed(0)
    model = cdp.VGG11().cuda()
    g = torch.Generator(device="cuda").manual_seed(B)
    x = torch.randn(B, 3, 32, 32, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    t = torch.randint(0, 10, (B,), device="cuda", generator=g)
    crit = cdp.CrossEntropyLoss()

    def grads(fused):
        monkeypatch.setenv("CDP_FUSED_CLASSIFIER", "1" if fused else "0")
        model.zero_grad(set_to_none=True)
        n0 = CF.LINK_HANDOFFS[0]
        crit(model(x), t).backward()
        torch.cuda.synchronize()
        return [p.grad.detach().clone() for p in model.parameters()], CF.LINK_HANDOFFS[0] - n0

    g_f, h_f = grads(True)
    g_u, h_u = grads(False)
    assert h_f == h_u + 1, (h_f, h_u)
    names = [n for n, _ in model.named_parameters()]
    for name, a, b in zip(names, g_f, g_u):
        if name.startswith("layers.") and name.endswith(".bias") and isinstance(
                model.layers[int(name.split(".")[1])], torch.nn.Conv2d):
            continue  # conv bias before training-mode BN: analytically zero, rounding noise
        err = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
        assert err < 1e-5, (name, err)
