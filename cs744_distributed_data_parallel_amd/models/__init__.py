"""Model zoo: the reference's VGG family (CIFAR-shaped) and the ResNet family (ImageNet-shaped)."""
from .resnet import ResNet, resnet18, resnet34, resnet50, resnet101, resnet152
from .vgg import VGG, VGG11, VGG13, VGG16, VGG19, cfg, make_layers

_REGISTRY = {
    "vgg11": VGG11,
    "vgg13": VGG13,
    "vgg16": VGG16,
    "vgg19": VGG19,
    "resnet18": resnet18,
    "resnet34": resnet34,
    "resnet50": resnet50,
    "resnet101": resnet101,
    "resnet152": resnet152,
}

# input shape (C, H, W) and number of classes per family
INPUT_SHAPES = {k: ((3, 32, 32), 10) if k.startswith("vgg") else ((3, 224, 224), 1000) for k in _REGISTRY}


def get_model(name: str, **kw):
    key = name.lower().replace("-", "").replace("_", "")
    if key not in _REGISTRY:
        raise ValueError(f"unknown model {name!r}; choose from {sorted(_REGISTRY)}")
    return _REGISTRY[key](**kw)


def list_models():
    return sorted(_REGISTRY)


__all__ = [
    "VGG", "VGG11", "VGG13", "VGG16", "VGG19", "cfg", "make_layers",
    "ResNet", "resnet18", "resnet34", "resnet50", "resnet101", "resnet152",
    "get_model", "list_models", "INPUT_SHAPES",
]
