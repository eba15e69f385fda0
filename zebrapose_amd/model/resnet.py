"""Dilated output-stride-8 ResNet encoders -- module tree of reference ``zebrapose/model/resnet.py``.

Same classes, constructor signatures, attribute names and registration order as the
reference (``make_layer`` :8-18, ``BasicBlock`` :20-51, ``ResNet_BasicBlock_OS8``
:170-246, ``ResNet34_OS8`` / ``ResNet50_OS8`` :274-278), so ``state_dict()`` keys and
``parameters()`` order match checkpoints written by the reference.  The stem / layer1 /
layer2 come from torchvision's ResNet34 / ResNet50 (0.10.0 layout, restated in
``_tv_children``); in concat mode ``resnet_layer_{1,2,3}`` share those modules with
``self.resnet`` exactly like resnet.py:191-199 (96 aliased checkpoint keys).

Only the concat (decoder skip) configuration runs: the reference's non-concat forward
passes ``x_128=None`` into ``torch.cat`` (aspp.py:112) and cannot run either.
The computation is done by ``zebrapose_amd.engine``.
"""
from __future__ import annotations

import os
import warnings

import torch
import torch.nn as nn

from .layers import BatchNorm2d, Conv2d, MaxPool2d, ReLU


def make_layer(block, in_channels, channels, num_blocks, stride=1, dilation=1):
    """resnet.py:8-18."""
    strides = [stride] + [1] * (num_blocks - 1)
    blocks = []
    for s in strides:
        blocks.append(block(in_channels=in_channels, channels=channels, stride=s, dilation=dilation))
        in_channels = block.expansion * channels
    return nn.Sequential(*blocks)


class BasicBlock(nn.Module):
    """resnet.py:20-51: relu(bn2(conv2(relu(bn1(conv1 x)))) + downsample(x)), padding = dilation."""
    expansion = 1

    def __init__(self, in_channels, channels, stride=1, dilation=1):
        super().__init__()
        out_channels = self.expansion * channels
        self.stride, self.dilation = stride, dilation
        self.conv1 = Conv2d(in_channels, channels, kernel_size=3, stride=stride, padding=dilation, dilation=dilation,
                            bias=False)
        self.bn1 = BatchNorm2d(channels)
        self.conv2 = Conv2d(channels, channels, kernel_size=3, stride=1, padding=dilation, dilation=dilation, bias=False)
        self.bn2 = BatchNorm2d(channels)
        if stride != 1 or in_channels != out_channels:
            self.downsample = nn.Sequential(Conv2d(in_channels, out_channels, kernel_size=1, stride=stride, bias=False),
                                            BatchNorm2d(out_channels))
        else:
            self.downsample = nn.Sequential()


# ---------------------------------------------------------------- torchvision children
class TVBasicBlock(nn.Module):
    """torchvision.models.resnet.BasicBlock layout (conv3x3 stride on conv1)."""
    expansion = 1

    def __init__(self, inplanes, planes, stride=1):
        super().__init__()
        self.stride, self.dilation = stride, 1
        self.conv1 = Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = BatchNorm2d(planes)
        self.relu = ReLU(inplace=True)
        self.conv2 = Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = BatchNorm2d(planes)
        self.downsample = None
        if stride != 1 or inplanes != planes:
            self.downsample = nn.Sequential(Conv2d(inplanes, planes, 1, stride, bias=False), BatchNorm2d(planes))


class TVBottleneck(nn.Module):
    """torchvision.models.resnet.Bottleneck layout (v1.5: stride on the 3x3 conv2)."""
    expansion = 4

    def __init__(self, inplanes, planes, stride=1):
        super().__init__()
        width = planes
        self.stride = stride
        self.conv1 = Conv2d(inplanes, width, 1, bias=False)
        self.bn1 = BatchNorm2d(width)
        self.conv2 = Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = BatchNorm2d(width)
        self.conv3 = Conv2d(width, planes * 4, 1, bias=False)
        self.bn3 = BatchNorm2d(planes * 4)
        self.relu = ReLU(inplace=True)
        self.downsample = None
        if stride != 1 or inplanes != planes * 4:
            self.downsample = nn.Sequential(Conv2d(inplanes, planes * 4, 1, stride, bias=False),
                                            BatchNorm2d(planes * 4))


def _tv_children(variant):
    """children of torchvision resnet34 / resnet50 up to layer2 (children()[:-4]) plus the
    unused tail (for pretrained-file loading)."""
    conv1 = Conv2d(3, 64, 7, 2, 3, bias=False)
    bn1 = BatchNorm2d(64)
    relu = ReLU(inplace=True)
    maxpool = MaxPool2d(3, 2, 1)
    if variant == 34:
        l1 = nn.Sequential(*[TVBasicBlock(64, 64) for _ in range(3)])
        l2 = nn.Sequential(*[TVBasicBlock(64 if i == 0 else 128, 128, 2 if i == 0 else 1) for i in range(4)])
    else:
        l1 = nn.Sequential(*[TVBottleneck(64 if i == 0 else 256, 64) for i in range(3)])
        l2 = nn.Sequential(*[TVBottleneck(256 if i == 0 else 512, 128, 2 if i == 0 else 1) for i in range(4)])
    return [conv1, bn1, relu, maxpool, l1, l2]


def _load_pretrained(children, variant):
    """resnet.py:185-189 / 207-211 load torchvision weights from pretrained_backbone/resnet/.
    Honour the same file when present (ZP_PRETRAINED_DIR or the reference-relative path)."""
    fname = {34: "resnet34-333f7ec4.pth", 50: "resnet50-19c8e357.pth"}[variant]
    cands = []
    if os.environ.get("ZP_PRETRAINED_DIR"):
        cands.append(os.path.join(os.environ["ZP_PRETRAINED_DIR"], fname))
    cands.append(os.path.join(os.path.dirname(__file__), "..", "..", "pretrained_backbone", "resnet", fname))
    for path in cands:
        if os.path.isfile(path):
            sd = torch.load(path, map_location="cpu", weights_only=True)
            names = ["conv1", "bn1", "relu", "maxpool", "layer1", "layer2"]
            for name, mod in zip(names, children):
                sub = {k[len(name) + 1:]: v for k, v in sd.items() if k.startswith(name + ".")}
                if sub:
                    mod.load_state_dict(sub)
            return path
    return None


class ResNet_BasicBlock_OS8(nn.Module):
    """resnet.py:170-246 (18-layer variant is not part of the north-star path)."""

    def __init__(self, num_layers, concat_decoder):
        super().__init__()
        if num_layers not in (34, 50):
            raise NotImplementedError("num_layers must be 34 or 50")
        self.concat_decoder = concat_decoder
        self.num_layers = num_layers
        children = _tv_children(num_layers)
        self.pretrained_from = _load_pretrained(children, num_layers)
        if self.pretrained_from is None and not os.environ.get("ZP_QUIET"):
            warnings.warn("pretrained backbone file not found; the encoder stem/layer1/layer2 keep their default "
                          "initialisation (load a ZebraPose checkpoint to run inference)", stacklevel=3)
        self.resnet = nn.Sequential(*children)
        if concat_decoder:
            self.resnet_layer_1 = nn.Sequential(*children[:3])
            self.resnet_layer_2 = nn.Sequential(*children[3:5])
            self.resnet_layer_3 = nn.Sequential(*children[5:6])
        c32, c16, chigh = (128, 256, 512) if num_layers == 34 else (512, 1024, 2048)
        self.layer4 = make_layer(BasicBlock, in_channels=c32, channels=c16, num_blocks=6, stride=1, dilation=2)
        self.layer5 = make_layer(BasicBlock, in_channels=c16, channels=chigh, num_blocks=3, stride=1, dilation=4)


def ResNet34_OS8(num_layers=34, concat_decoder=True):
    return ResNet_BasicBlock_OS8(num_layers=num_layers, concat_decoder=concat_decoder)


def ResNet50_OS8(num_layers=50, concat_decoder=True):
    return ResNet_BasicBlock_OS8(num_layers=num_layers, concat_decoder=concat_decoder)
