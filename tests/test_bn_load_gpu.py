"""BatchNorm (+ReLU) applied on the conv GEMM's operand load (``conv2d_fwd(..., bn_stats=...)``).

The f16x2 conv kernel can read a producer's raw conv output y and form ``relu(y * scale + shift)``
per input channel as it gathers A (csrc/kernels/conv_x3_body.h, BNA), instead of reading an
activation a separate BatchNorm-apply pass wrote. Given the same operand maxima, the GEMM sees
exactly the values the apply pass would have written (the same fma + max), so its output must equal
the materialized path bit for bit -- including the padding taps, which must stay zero rather than
become relu(shift). The reference unit is Conv2d -> BatchNorm2d -> ReLU
(/root/reference/src/Part 1/model.py:18-25).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def native():
    import cs744_distributed_data_parallel_amd as cdp

    return cdp._native.lib()


SHAPES = [
    # (N, C, H, W, Co, k, stride, pad): VGG-11's unpooled consumers at 32 images, ResNet bottlenecks
    (32, 256, 8, 8, 256, 3, 1, 1),
    (32, 512, 4, 4, 512, 3, 1, 1),
    (32, 512, 2, 2, 512, 3, 1, 1),
    (4, 64, 56, 56, 64, 3, 1, 1),
    (4, 64, 56, 56, 256, 1, 1, 0),
    (4, 128, 56, 56, 128, 3, 2, 1),
    (2, 512, 7, 7, 2048, 1, 1, 0),
]


def _stats(C, dev, gen):
    scale = torch.randn(C, device=dev, generator=gen)  # some channels negative
    shift = torch.randn(C, device=dev, generator=gen).abs() + 0.5  # > 0: a wrong padding tap would show
    st = torch.zeros(4, C, device=dev)
    st[2], st[3] = scale, shift
    return st


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("relu", [True, False])
def test_bn_on_load_equals_materialized_apply(native, shape, relu):
    C_ = native
    N, C, H, W, Co, k, stride, pad = shape
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(7)
    prev = C_.get_conv_gemm()
    C_.set_conv_gemm("f16x2")
    try:
        y = torch.randn(N, C, H, W, device=dev, generator=gen).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(Co, C, k, k, device=dev, generator=gen) / (C * k * k) ** 0.5).contiguous(
            memory_format=torch.channels_last)
        st = _stats(C, dev, gen)
        # fma(y, scale, shift) rounded once, as the kernels compute it (y * scale is exact in fp64)
        act = (y.double() * st[2].double().view(1, C, 1, 1) + st[3].double().view(1, C, 1, 1)).float()
        if relu:
            act = act.clamp_min(0)
        act = act.contiguous(memory_format=torch.channels_last)
        am = C_.act_max(act)
        ref = C_.conv2d_fwd(act, w, None, stride, pad, False, am)[0]
        out = C_.conv2d_fwd(y, w, None, stride, pad, False, am, None, st, relu)[0]
        torch.cuda.synchronize()
        assert torch.equal(out, ref), (out - ref).abs().max().item()
        # and both against fp64 (the materialized path is the tested one; this pins the pair)
        r64 = torch.nn.functional.conv2d(act.double(), w.double(), None, stride, pad)
        err = (out.double() - r64).abs().max().item()
        assert err <= 1e-4 * r64.abs().max().item(), err
    finally:
        C_.set_conv_gemm(prev)


def test_bn_on_load_rejects_other_engines(native):
    C_ = native
    dev = torch.device("cuda")
    prev = C_.get_conv_gemm()
    C_.set_conv_gemm("x3")
    try:
        y = torch.randn(2, 64, 8, 8, device=dev).contiguous(memory_format=torch.channels_last)
        w = torch.randn(64, 64, 3, 3, device=dev).contiguous(memory_format=torch.channels_last)
        st = torch.zeros(4, 64, device=dev)
        with pytest.raises(RuntimeError, match="f16x2"):
            C_.conv2d_fwd(y, w, None, 1, 1, False, None, None, st, True)
    finally:
        C_.set_conv_gemm(prev)
