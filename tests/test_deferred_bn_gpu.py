"""Deferred downsample BatchNorm (``conv_bn_act(..., defer_apply=True)``).

A ResNet downsample branch (``downsample = Conv2d -> BatchNorm2d``, torchvision's Bottleneck; the
model is BASELINE.json config #5, the reference itself only ships VGG) is only ever read by the
block's residual add. The native
path computes its conv and BN statistics, returns a shape-only placeholder, and the block's last
``conv_bn_act`` applies the downsample's affine BN inside its own residual add (bn.hip
``bn_act_fwd_kernel`` res_y / res_st), so the normalized branch is never written or read back.
These tests pin that the deferred block equals the materialized one (forward, every gradient,
running statistics, train and eval) and that the placeholder refuses misuse.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _block(seed):
    from cs744_distributed_data_parallel_amd.models.resnet import Bottleneck

    torch.manual_seed(seed)
    ds = torch.nn.Sequential(torch.nn.Conv2d(64, 256, 1, 2, bias=False), torch.nn.BatchNorm2d(256))
    blk = Bottleneck(64, 64, stride=2, downsample=ds)
    for m in blk.modules():  # non-trivial affine parameters so a dropped scale/shift shows
        if isinstance(m, torch.nn.BatchNorm2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.5, 0.5)
    return blk.cuda()


def _run(monkeypatch, defer, train, seed=3):
    from cs744_distributed_data_parallel_amd.models import resnet

    monkeypatch.setattr(resnet, "_DEFER_DS", defer)
    blk = _block(seed)
    blk.train(train)
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(4, 64, 28, 28, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    out = blk(x)
    gout = torch.randn(out.shape, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    out.backward(gout)
    torch.cuda.synchronize()
    grads = {n: p.grad.clone() for n, p in blk.named_parameters()}
    bufs = {n: b.clone() for n, b in blk.named_buffers()}
    return out.detach().clone(), x.grad.clone(), grads, bufs


@pytest.mark.parametrize("train", [True, False])
def test_deferred_downsample_matches_materialized(monkeypatch, train):
    o1, dx1, g1, b1 = _run(monkeypatch, True, train)
    o0, dx0, g0, b0 = _run(monkeypatch, False, train)

    def rel(a, b):
        return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()

    assert rel(o1, o0) < 1e-6
    assert rel(dx1, dx0) < 1e-5
    for n in g0:
        assert rel(g1[n], g0[n]) < 1e-5, n
    for n in b0:
        if b0[n].is_floating_point():
            assert rel(b1[n], b0[n]) < 1e-6, n
        else:
            assert torch.equal(b1[n], b0[n]), n


def test_deferred_placeholder_refuses_misuse():
    import cs744_distributed_data_parallel_amd as cdp

    CF = cdp.ops.functional
    torch.manual_seed(0)
    conv, bn = torch.nn.Conv2d(64, 64, 1, bias=False).cuda(), torch.nn.BatchNorm2d(64).cuda()
    conv2, bn2 = torch.nn.Conv2d(64, 64, 3, padding=1, bias=False).cuda(), torch.nn.BatchNorm2d(64).cuda()
    x = torch.randn(2, 64, 8, 8, device="cuda").contiguous(memory_format=torch.channels_last)
    ph = CF.conv_bn_act(x, conv, bn, relu=False, defer_apply=True)
    assert ph.shape == (2, 64, 8, 8)
    # one element expanded: torch itself refuses an in-place write into it
    with pytest.raises(RuntimeError):
        with torch.no_grad():
            ph.add_(1.0)
    # a placeholder whose version moved on (any in-place op that got through) is refused as a residual
    y, st, ver = ph._cdp_deferred_bn
    ph._cdp_deferred_bn = (y, st, ver - 1)
    with pytest.raises(RuntimeError, match="deferred BatchNorm placeholder was modified"):
        CF.conv_bn_act(x, conv2, bn2, relu=True, residual=ph)
    with pytest.raises(RuntimeError, match="defer_apply is for a plain BatchNorm"):
        CF.conv_bn_act(x, conv, bn, relu=True, defer_apply=True)
