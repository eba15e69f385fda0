"""Entire-mask head of the 3-head network -- module tree of reference ``zebrapose/model/aspp_v3.py``
(:5-102).  Same attribute names / registration order as ``ASPP_v3``: three ASPP branches on the
512-channel high feature (1x1, 3x3 d6, 3x3 d12), image pooling, then a 1x1 over the 1025-channel
concat (4 x 256 + the visible-mask logits resampled to 32x32), the two upsampling stages (the
second one takes [x, x_64, mask_64] = 321 channels) and a 1x1 head over [x, x_128, mask] (321) to
one channel.  The computation is done by ``zebrapose_amd.engine`` (``Engine.forward_v3``).
"""
from __future__ import annotations

import torch.nn as nn

from .aspp import _upsample
from .layers import AdaptiveAvgPool2d, BatchNorm2d, Conv2d


class ASPP_v3(nn.Module):
    def __init__(self, num_classes, concat=True, output_kernel_size=1):
        super().__init__()
        if not concat:
            raise NotImplementedError("ASPP_v3 without concat: the reference forward cannot run it")
        if output_kernel_size not in (1, 3):
            raise NotImplementedError("output_kernel_size must be 1 or 3")
        self.concat = concat
        self.output_kernel_size = output_kernel_size
        self.conv_1x1_1 = Conv2d(512, 256, kernel_size=1)
        self.bn_conv_1x1_1 = BatchNorm2d(256)
        self.conv_3x3_1 = Conv2d(512, 256, kernel_size=3, stride=1, padding=6, dilation=6)
        self.bn_conv_3x3_1 = BatchNorm2d(256)
        self.conv_3x3_2 = Conv2d(512, 256, kernel_size=3, stride=1, padding=12, dilation=12)
        self.bn_conv_3x3_2 = BatchNorm2d(256)
        self.avg_pool = AdaptiveAvgPool2d(1)
        self.conv_1x1_2 = Conv2d(512, 256, kernel_size=1)
        self.bn_conv_1x1_2 = BatchNorm2d(256)
        self.conv_1x1_3 = Conv2d(1025, 256, kernel_size=1)
        self.bn_conv_1x1_3 = BatchNorm2d(256)
        self.upsample_1 = _upsample(256, 256, 3, 1, 1)
        self.upsample_2 = _upsample(256 + 64 + 1, 256, 3, 1, 1)
        pad = 1 if output_kernel_size == 3 else 0
        self.conv_1x1_4 = Conv2d(256 + 64 + 1, num_classes, kernel_size=output_kernel_size, padding=pad)
