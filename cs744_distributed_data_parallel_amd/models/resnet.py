"""ResNet family (ResNet-18/34/50/101/152) for ImageNet-shaped inputs.

This is the ``BASELINE.json`` config #5 model ("ResNet-50 ImageNet-shaped synthetic, bucketed DDP
on 8xMI355X -- larger-model bucket-sizing stress"): 25.6M parameters in 161 tensors, so the
bucketed reducer sees many more, and much more unevenly sized, gradients than VGG-11's 34.
The module tree (``conv1/bn1/layer1..4/fc``, ``downsample.0/1``) and default initialisation follow
the torchvision layout so checkpoints are interchangeable.

MI355X execution: every ``conv -> BN [-> +residual] [-> ReLU]`` is one fused autograd op
(implicit-GEMM MFMA conv, BN statistics fused into the conv epilogue, BN-apply + residual + ReLU in
one NHWC pass); 1x1 convs are plain GEMMs through the same kernel; strided 3x3 / 1x1 convs use the
strided gather (forward) and the divisibility-masked transposed gather (data gradient).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from ..ops import functional as CF
from ..utils.arena import install_load_hooks

# CDP_DEFER_DS=0: materialize the downsample branch's BatchNorm output (A/B)
_DEFER_DS = os.environ.get("CDP_DEFER_DS", "1") != "0"


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        if CF.use_native(x):
            sink = CF.GradSink.make(x)
            out = CF.conv_bn_act(x, self.conv1, self.bn1, relu=True, dx_sink=sink)
            if self.downsample is None:
                return CF.conv_bn_act(out, self.conv2, self.bn2, relu=True, residual=x, res_sink=sink)
            # the downsample's BatchNorm is applied inside conv2's residual add (defer_apply)
            idt = CF.conv_bn_act(x, self.downsample[0], self.downsample[1], relu=False, dx_sink=sink,
                                 defer_apply=_DEFER_DS)
            return CF.conv_bn_act(out, self.conv2, self.bn2, relu=True, residual=idt)
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        width = planes
        self.conv1 = nn.Conv2d(inplanes, width, 1, 1, 0, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, planes * 4, 1, 1, 0, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        if CF.use_native(x):
            # x's two gradients (conv1 + residual, or conv1 + downsample) are summed inside a
            # data-gradient GEMM epilogue instead of an autograd add (GradSink)
            sink = CF.GradSink.make(x)
            out = CF.conv_bn_act(x, self.conv1, self.bn1, relu=True, dx_sink=sink)
            out = CF.conv_bn_act(out, self.conv2, self.bn2, relu=True)
            if self.downsample is None:
                return CF.conv_bn_act(out, self.conv3, self.bn3, relu=True, residual=x, res_sink=sink)
            # the downsample's BatchNorm is applied inside conv3's residual add (defer_apply)
            idt = CF.conv_bn_act(x, self.downsample[0], self.downsample[1], relu=False, dx_sink=sink,
                                 defer_apply=_DEFER_DS)
            return CF.conv_bn_act(out, self.conv3, self.bn3, relu=True, residual=idt)
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + idt)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000, channels_last=True):
        super().__init__()
        install_load_hooks(self)  # loaded weights refresh the optimizer's prepared products
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if channels_last:
            for m in self.modules():
                if isinstance(m, nn.Conv2d):
                    m.weight.data = m.weight.data.contiguous(memory_format=torch.channels_last)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                nn.Conv2d(self.inplanes, planes * block.expansion, 1, stride, 0, bias=False),
                nn.BatchNorm2d(planes * block.expansion),
            )
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x):
        if CF.use_native(x):
            x = x.contiguous(memory_format=torch.channels_last)
            # one launch: every conv weight's f16x2 operand scale and its W^T for the data gradient
            # (stride-1 convs; the stem's input needs no gradient, stride-2 convs use sub-filters);
            # each conv module holds its entries for the duration of this forward (conv_bn_act
            # reads them)
            convs = [m for m in self.modules() if isinstance(m, nn.Conv2d)]
            need = [m.stride[0] == 1 and (m is not self.conv1 or x.requires_grad) for m in convs]
            wam, wts = CF.weight_prep([m.weight for m in convs], need)
            for i, m in enumerate(convs):
                m._cdp_wamax = wam[i] if wam is not None else None
                m._cdp_wt = wts[i] if wts is not None else None
            try:
                x = CF.conv_bn_act(x, self.conv1, self.bn1, relu=True)
                x = CF.max_pool2d(x, 3, 2, 1)
                x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
            finally:
                for m in convs:
                    m._cdp_wamax = None
                    m._cdp_wt = None
            x = CF.global_avg_pool(x)
            return CF.linear(x, self.fc.weight, self.fc.bias)
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


def resnet18(**kw):
    return ResNet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet34(**kw):
    return ResNet(BasicBlock, [3, 4, 6, 3], **kw)


def resnet50(**kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet101(**kw):
    return ResNet(Bottleneck, [3, 4, 23, 3], **kw)


def resnet152(**kw):
    return ResNet(Bottleneck, [3, 8, 36, 3], **kw)
