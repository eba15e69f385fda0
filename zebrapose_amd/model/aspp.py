"""ASPP + upsampling decoder -- module tree of reference ``zebrapose/model/aspp.py``.

``ASPP`` (:5-114, 512-channel input) and ``ASPP_50`` (:117-225, 2048-channel input)
with the reference's attribute names; ``upsample()`` returns the same 9-entry
Sequential (ConvT, BN, ReLU, conv3x3, BN, ReLU, conv3x3, BN, ReLU; :60-80).
The computation is done by ``zebrapose_amd.engine``.
"""
from __future__ import annotations

import torch.nn as nn

from .layers import AdaptiveAvgPool2d, BatchNorm2d, Conv2d, ConvTranspose2d, ReLU


def _upsample(in_channels, num_filters, kernel_size=3, padding=1, output_padding=1):
    return nn.Sequential(
        ConvTranspose2d(in_channels, num_filters, kernel_size=kernel_size, stride=2, padding=padding,
                        output_padding=output_padding, bias=False),
        BatchNorm2d(num_filters), ReLU(inplace=True),
        Conv2d(num_filters, num_filters, kernel_size=3, stride=1, padding=1, bias=False),
        BatchNorm2d(num_filters), ReLU(inplace=True),
        Conv2d(num_filters, num_filters, kernel_size=3, stride=1, padding=1, bias=False),
        BatchNorm2d(num_filters), ReLU(inplace=True))


class _ASPPBase(nn.Module):
    in_high = 512
    x64_channels = 64

    def __init__(self, num_classes, concat=True, output_kernel_size=1):
        super().__init__()
        if output_kernel_size not in (1, 3):
            raise NotImplementedError("output_kernel_size must be 1 or 3")
        self.concat = concat
        self.num_classes = num_classes
        self.output_kernel_size = output_kernel_size
        c = self.in_high
        self.conv_1x1_1 = Conv2d(c, 256, kernel_size=1)
        self.bn_conv_1x1_1 = BatchNorm2d(256)
        self.conv_3x3_1 = Conv2d(c, 256, kernel_size=3, stride=1, padding=6, dilation=6)
        self.bn_conv_3x3_1 = BatchNorm2d(256)
        self.conv_3x3_2 = Conv2d(c, 256, kernel_size=3, stride=1, padding=12, dilation=12)
        self.bn_conv_3x3_2 = BatchNorm2d(256)
        self.conv_3x3_3 = Conv2d(c, 256, kernel_size=3, stride=1, padding=18, dilation=18)
        self.bn_conv_3x3_3 = BatchNorm2d(256)
        self.avg_pool = AdaptiveAvgPool2d(1)
        self.conv_1x1_2 = Conv2d(c, 256, kernel_size=1)
        self.bn_conv_1x1_2 = BatchNorm2d(256)
        self.conv_1x1_3 = Conv2d(1280, 256, kernel_size=1)
        self.bn_conv_1x1_3 = BatchNorm2d(256)
        if concat:
            self.upsample_1 = self.upsample(256, 256, 3, 1, 1)
            self.upsample_2 = self.upsample(256 + self.x64_channels, 256, 3, 1, 1)
        else:
            self.upsample_1 = self.upsample(256, 256, 3, 1, 1)
            self.upsample_2 = self.upsample(256, 256, 3, 1, 1)
        pad = 1 if output_kernel_size == 3 else 0
        self.conv_1x1_4 = Conv2d(256 + 64, num_classes, kernel_size=output_kernel_size, padding=pad)

    def upsample(self, in_channels, num_filters, kernel_size, padding, output_padding):
        return _upsample(in_channels, num_filters, kernel_size, padding, output_padding)


class ASPP(_ASPPBase):
    """aspp.py:5-114 (ResNet34 encoder, 512-channel high feature, 64-channel x_64 skip)."""
    in_high = 512
    x64_channels = 64


class ASPP_50(_ASPPBase):
    """aspp.py:117-225 (ResNet50 encoder, 2048-channel high feature, 256-channel x_64 skip)."""
    in_high = 2048
    x64_channels = 256
