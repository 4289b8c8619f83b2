"""ResNet backbone with frozen BatchNorm (models/backbone.py).

Module tree and parameter names follow torchvision's ResNet (``body.conv1``, ``body.bn1``,
``body.layerN.i.{conv1,bn1,conv2,bn2,conv3,bn3,downsample.0,downsample.1}``) so reference
checkpoints load unchanged.  The convolution arithmetic runs in ``retr_amd.resnet`` (NHWC
implicit-GEMM MFMA kernels with FrozenBN folded), not in torch.

Pretrained torchvision weights cannot be fetched offline: the reference downloads them on rank 0
(``models/backbone.py:87-91``); here the body keeps torchvision's random init and a checkpoint
is loaded with ``load_state_dict``.
"""
import math
from collections import OrderedDict

import torch
from torch import nn

from .utils import NestedTensor


class FrozenBatchNorm2d(torch.nn.Module):
    """BatchNorm2d with fixed statistics and affine parameters (buffers only)."""

    def __init__(self, n):
        super().__init__()
        self.register_buffer("weight", torch.ones(n))
        self.register_buffer("bias", torch.zeros(n))
        self.register_buffer("running_mean", torch.zeros(n))
        self.register_buffer("running_var", torch.ones(n))

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        state_dict.pop(prefix + "num_batches_tracked", None)
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys,
                                      unexpected_keys, error_msgs)


def _conv(cin, cout, k, stride=1, padding=0, dilation=1):
    c = nn.Conv2d(cin, cout, k, stride=stride, padding=padding, dilation=dilation, bias=False)
    nn.init.kaiming_normal_(c.weight, mode="fan_out", nonlinearity="relu")
    return c


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, dilation=1):
        super().__init__()
        if dilation > 1:
            raise NotImplementedError("Dilation > 1 not supported in BasicBlock")
        self.conv1 = _conv(inplanes, planes, 3, stride, 1)
        self.bn1 = FrozenBatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = _conv(planes, planes, 3, 1, 1)
        self.bn2 = FrozenBatchNorm2d(planes)
        self.downsample = downsample


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, dilation=1):
        super().__init__()
        self.conv1 = _conv(inplanes, planes, 1)
        self.bn1 = FrozenBatchNorm2d(planes)
        self.conv2 = _conv(planes, planes, 3, stride, dilation, dilation)
        self.bn2 = FrozenBatchNorm2d(planes)
        self.conv3 = _conv(planes, planes * 4, 1)
        self.bn3 = FrozenBatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample


_ARCH = {"resnet18": (BasicBlock, [2, 2, 2, 2]), "resnet34": (BasicBlock, [3, 4, 6, 3]),
         "resnet50": (Bottleneck, [3, 4, 6, 3]), "resnet101": (Bottleneck, [3, 4, 23, 3])}


def resnet_body(name, dilation):
    """torchvision ``resnet*(replace_stride_with_dilation=[False, False, dilation],
    norm_layer=FrozenBatchNorm2d)`` truncated after layer4 (IntermediateLayerGetter)."""
    block, layers = _ARCH[name.lower()]
    body = nn.Module()
    body.conv1 = _conv(3, 64, 7, 2, 3)
    body.bn1 = FrozenBatchNorm2d(64)
    body.relu = nn.ReLU(inplace=True)
    body.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
    inplanes, cur_dil = 64, 1
    for li, (planes, nblk, stride, dil_flag) in enumerate(
            zip([64, 128, 256, 512], layers, [1, 2, 2, 2], [False, False, False, dilation])):
        prev_dil = cur_dil
        if dil_flag:
            cur_dil *= stride
            stride = 1
        ds = None
        if stride != 1 or inplanes != planes * block.expansion:
            ds = nn.Sequential(_conv(inplanes, planes * block.expansion, 1, stride),
                               FrozenBatchNorm2d(planes * block.expansion))
        mods = [block(inplanes, planes, stride, ds, prev_dil)]
        inplanes = planes * block.expansion
        for _ in range(1, nblk):
            mods.append(block(inplanes, planes, 1, None, cur_dil))
        setattr(body, f"layer{li + 1}", nn.Sequential(*mods))
    return body


class BackboneBase(nn.Module):
    def __init__(self, body: nn.Module, train_backbone: bool, num_channels: int,
                 return_interm_layers: bool):
        super().__init__()
        for name, parameter in body.named_parameters():
            if not train_backbone or ("layer2" not in name and "layer3" not in name
                                      and "layer4" not in name):
                parameter.requires_grad_(False)
        if return_interm_layers:
            raise NotImplementedError("return_interm_layers is not on the hot path")
        self.body = body
        self.num_channels = num_channels
        self._runner = None

    def runner(self, cdtype):
        from ..resnet import BackboneRunner
        if self._runner is None or self._runner.cdtype != cdtype:
            self._runner = BackboneRunner(self.body, cdtype)
        return self._runner

    def features(self, tensor_list: NestedTensor, cdtype):
        """-> (NHWC features [B, h, w, Cb] in cdtype, mask [B, h, w] bool)."""
        from .. import _lib
        from .._lib import call, ptr
        x, m = tensor_list.tensors, tensor_list.mask
        assert m is not None
        feats = self.runner(cdtype).run(x)
        b, h, w, _ = feats.shape
        mh = torch.empty(b, h, w, dtype=torch.bool, device=x.device)
        mu = m.contiguous().view(torch.uint8)
        call("retr_mask_nearest", ptr(mu), ptr(mh), b, m.shape[1], m.shape[2], h, w,
             _lib.stream())
        return feats, mh

    def forward(self, tensor_list: NestedTensor):
        """API-compatible: {'0': NestedTensor(features [B, Cb, h, w], mask)}."""
        from ..configuration import compute_dtype
        feats, mh = self.features(tensor_list, getattr(self, "cdtype", torch.bfloat16))
        return {"0": NestedTensor(feats.permute(0, 3, 1, 2), mh)}


class Backbone(BackboneBase):
    """ResNet backbone with frozen BatchNorm."""

    def __init__(self, name: str, train_backbone: bool, return_interm_layers: bool,
                 dilation: bool):
        body = resnet_body(name, dilation)
        num_channels = 512 if name in ("ResNet18", "ResNet34") else 2048
        super().__init__(body, train_backbone, num_channels, return_interm_layers)


def build_backbone(config):
    train_backbone = config.lr_backbone > 0
    return Backbone(config.backbone, train_backbone, False, config.dilation)
