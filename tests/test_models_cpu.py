"""Model zoo parity with the reference (VGG config table, layer stack, state_dict layout, init)."""
import torch
import torch.nn as nn

import cs744_distributed_data_parallel_amd as cdp
from cs744_distributed_data_parallel_amd.models import cfg, get_model, list_models

# /root/reference/src/Part 1/model.py:3-8
REF_CFG = {
    "VGG11": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "VGG13": [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "VGG16": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
    "VGG19": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"],
}

# 34 tensors, 9,231,114 parameters, 58 state_dict keys
VGG11_SHAPES = [
    (64, 3, 3, 3), (64,), (64,), (64,), (128, 64, 3, 3), (128,), (128,), (128,),
    (256, 128, 3, 3), (256,), (256,), (256,), (256, 256, 3, 3), (256,), (256,), (256,),
    (512, 256, 3, 3), (512,), (512,), (512,), (512, 512, 3, 3), (512,), (512,), (512,),
    (512, 512, 3, 3), (512,), (512,), (512,), (512, 512, 3, 3), (512,), (512,), (512,),
    (10, 512), (10,),
]


def _reference_like(name):
    """A plain torch.nn model built the way the reference builds it (model.py:11-46)."""
    layers, c = [], 3
    for v in REF_CFG[name]:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers += [nn.Conv2d(c, v, 3, 1, 1, bias=True), nn.BatchNorm2d(v), nn.ReLU(inplace=True)]
            c = v

    class _VGG(nn.Module):
        def __init__(self):
            super().__init__()
            self.layers = nn.Sequential(*layers)
            self.fc1 = nn.Linear(512, 10)

        def forward(self, x):
            y = self.layers(x)
            return self.fc1(y.view(y.size(0), -1))

    return _VGG()


def test_cfg_table_matches_reference():
    assert cfg == REF_CFG


def test_vgg11_parameter_inventory():
    m = cdp.VGG11()
    shapes = [tuple(p.shape) for p in m.parameters()]
    assert shapes == VGG11_SHAPES
    assert sum(p.numel() for p in m.parameters()) == 9231114
    sd = m.state_dict()
    assert len(sd) == 58
    assert list(sd)[:5] == ["layers.0.weight", "layers.0.bias", "layers.1.weight", "layers.1.bias",
                            "layers.1.running_mean"]
    assert list(sd)[-2:] == ["fc1.weight", "fc1.bias"]


def test_same_init_and_outputs_as_reference_under_seed():
    for name in ["VGG11", "VGG16"]:
        torch.manual_seed(0)
        ref = _reference_like(name)
        torch.manual_seed(0)
        ours = cdp.models.VGG(name)
        for (k1, a), (k2, b) in zip(ref.state_dict().items(), ours.state_dict().items()):
            assert k1 == k2
            assert torch.equal(a, b.contiguous())
        x = torch.randn(4, 3, 32, 32)
        ref.eval()
        ours.eval()
        assert torch.allclose(ref(x), ours(x), atol=1e-5)


def test_state_dict_loads_both_ways():
    ref = _reference_like("VGG11")
    ours = cdp.VGG11()
    ours.load_state_dict(ref.state_dict())
    ref.load_state_dict(ours.state_dict())
    for a, b in zip(ref.parameters(), ours.parameters()):
        assert torch.equal(a, b)


def test_conv_weights_channels_last():
    m = cdp.VGG11()
    for mod in m.layers:
        if isinstance(mod, nn.Conv2d):
            assert mod.weight.is_contiguous(memory_format=torch.channels_last)


def test_factories_and_registry():
    for f in (cdp.models.VGG11, cdp.models.VGG13, cdp.models.VGG16, cdp.models.VGG19):
        out = f()(torch.randn(2, 3, 32, 32))
        assert out.shape == (2, 10)
    assert "resnet50" in list_models() and "vgg11" in list_models()
    assert isinstance(get_model("VGG-11"), cdp.models.VGG)


def test_resnet50_inventory():
    m = cdp.resnet50()
    params = list(m.parameters())
    assert len(params) == 161
    assert sum(p.numel() for p in params) == 25557032
    out = m(torch.randn(1, 3, 64, 64))
    assert out.shape == (1, 1000)
    keys = list(m.state_dict())
    assert "layer1.0.downsample.0.weight" in keys and "fc.weight" in keys


def test_resnet18_forward_backward():
    m = cdp.models.resnet18(num_classes=10)
    out = m(torch.randn(2, 3, 32, 32))
    out.sum().backward()
    assert m.conv1.weight.grad is not None


def test_sgd_post_step_joins_run_once_per_step():
    """SGD.add_post_step_join: the hook DistributedDataParallel.early_buffer_broadcast joins its
    end-of-backward broadcast through runs after every step, once, and registers only once."""
    lin = nn.Linear(4, 3)
    opt = cdp.SGD(lin.parameters(), lr=0.1, momentum=0.9)
    calls = []
    fn = lambda: calls.append(len(calls))  # noqa: E731
    opt.add_post_step_join(fn)
    opt.add_post_step_join(fn)
    for _ in range(3):
        opt.zero_grad()
        lin(torch.randn(2, 4)).sum().backward()
        opt.step()
    assert calls == [0, 1, 2]
