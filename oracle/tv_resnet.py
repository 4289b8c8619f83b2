"""Restatement of torchvision's ResNet family (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

torchvision is a third-party dependency of the reference (``models/backbone.py:6,8,65,86-91``)
that is not installed in this image; no version is pinned by the reference (it uses the
``weights=``/``*_Weights`` API, so torchvision >= 0.13).  This module restates the published
layer semantics:

* stem: Conv2d(3,64,7,s2,p3,bias=False) -> norm -> ReLU -> MaxPool2d(3,s2,p1)
* ``_make_layer``: when ``dilate``, ``dilation *= stride; stride = 1``; the first block uses the
  previous dilation, later blocks the new one; ``downsample = Sequential(conv1x1(s), norm)``
  when ``stride != 1 or inplanes != planes*expansion``.
* Bottleneck v1.5 (stride on the 3x3), expansion 4; BasicBlock expansion 1 and
  ``NotImplementedError("Dilation > 1 not supported in BasicBlock")``.
* ``IntermediateLayerGetter`` keeps children up to the last requested one and returns an
  OrderedDict keyed by the requested names.

Attribute names match torchvision so ``state_dict`` keys equal the reference's
(``backbone.body.layerN.i.convK.weight`` ...).  No pretrained weights are ever fetched: the
``weights`` argument is accepted and ignored (parameters are loaded from synthetic state dicts).
"""
from collections import OrderedDict

import torch
from torch import nn


def _conv3x3(cin, cout, stride=1, dilation=1):
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=dilation, dilation=dilation, bias=False)


def _conv1x1(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, dilation=1, norm_layer=None):
        super().__init__()
        if dilation > 1:
            raise NotImplementedError("Dilation > 1 not supported in BasicBlock")
        self.conv1 = _conv3x3(inplanes, planes, stride)
        self.bn1 = norm_layer(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = _conv3x3(planes, planes)
        self.bn2 = norm_layer(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + identity)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, dilation=1, norm_layer=None):
        super().__init__()
        self.conv1 = _conv1x1(inplanes, planes)
        self.bn1 = norm_layer(planes)
        self.conv2 = _conv3x3(planes, planes, stride, dilation)
        self.bn2 = norm_layer(planes)
        self.conv3 = _conv1x1(planes, planes * 4)
        self.bn3 = norm_layer(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + identity)


ARCH = {
    "resnet18": (BasicBlock, [2, 2, 2, 2]),
    "resnet34": (BasicBlock, [3, 4, 6, 3]),
    "resnet50": (Bottleneck, [3, 4, 6, 3]),
    "resnet101": (Bottleneck, [3, 4, 23, 3]),
}


class ResNet(nn.Module):
    def __init__(self, block, layers, replace_stride_with_dilation=None, norm_layer=None):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        self._norm_layer = norm_layer
        self.inplanes = 64
        self.dilation = 1
        rswd = replace_stride_with_dilation or [False, False, False]
        if len(rswd) != 3:
            raise ValueError("replace_stride_with_dilation should be None or a 3-element tuple")
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = norm_layer(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2, dilate=rswd[0])
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2, dilate=rswd[1])
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2, dilate=rswd[2])
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, 1000)

    def _make_layer(self, block, planes, blocks, stride=1, dilate=False):
        norm_layer = self._norm_layer
        downsample = None
        previous_dilation = self.dilation
        if dilate:
            self.dilation *= stride
            stride = 1
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(_conv1x1(self.inplanes, planes * block.expansion, stride),
                                       norm_layer(planes * block.expansion))
        mods = [block(self.inplanes, planes, stride, downsample, previous_dilation, norm_layer)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            mods.append(block(self.inplanes, planes, dilation=self.dilation, norm_layer=norm_layer))
        return nn.Sequential(*mods)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def _builder(name):
    def build(*, weights=None, progress=True, replace_stride_with_dilation=None, norm_layer=None,
              **kwargs):
        block, layers = ARCH[name]
        return ResNet(block, layers, replace_stride_with_dilation=replace_stride_with_dilation,
                      norm_layer=norm_layer)
    build.__name__ = name
    return build


resnet18 = _builder("resnet18")
resnet34 = _builder("resnet34")
resnet50 = _builder("resnet50")
resnet101 = _builder("resnet101")


class _Weights:
    """Stand-in for ``ResNet*_Weights``: ``.DEFAULT`` exists but never triggers a download."""
    DEFAULT = None


ResNet18_Weights = ResNet34_Weights = ResNet50_Weights = ResNet101_Weights = _Weights


class IntermediateLayerGetter(nn.ModuleDict):
    """torchvision.models._utils.IntermediateLayerGetter semantics."""

    def __init__(self, model, return_layers):
        if not set(return_layers).issubset([n for n, _ in model.named_children()]):
            raise ValueError("return_layers are not present in model")
        orig = dict(return_layers)
        return_layers = {str(k): str(v) for k, v in return_layers.items()}
        layers = OrderedDict()
        for name, module in model.named_children():
            layers[name] = module
            if name in return_layers:
                del return_layers[name]
            if not return_layers:
                break
        super().__init__(layers)
        self.return_layers = orig

    def forward(self, x):
        out = OrderedDict()
        for name, module in self.items():
            x = module(x)
            if name in self.return_layers:
                out[self.return_layers[name]] = x
        return out


def install_torchvision_standin():
    """Register this module as ``torchvision`` / ``torchvision.models`` / ``torchvision.models._utils``
    in ``sys.modules`` (used only by the golden generator to import the reference)."""
    import sys
    import types
    tv = types.ModuleType("torchvision")
    models = types.ModuleType("torchvision.models")
    utils = types.ModuleType("torchvision.models._utils")
    for n in ("resnet18", "resnet34", "resnet50", "resnet101", "ResNet18_Weights",
              "ResNet34_Weights", "ResNet50_Weights", "ResNet101_Weights"):
        setattr(models, n, globals()[n])
    utils.IntermediateLayerGetter = IntermediateLayerGetter
    models._utils = utils
    tv.models = models
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.models"] = models
    sys.modules["torchvision.models._utils"] = utils
