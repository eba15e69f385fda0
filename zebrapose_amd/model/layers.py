"""Parameter holders with the exact names / shapes / init of the reference's torch.nn layers.

They subclass the torch.nn classes so ``state_dict()``, ``parameters()``, ``.train()`` /
``.eval()``, ``isinstance`` checks and the default initialisation behave as in the
reference, but they never compute: the forward / backward of the network runs in
libzp (``zebrapose_amd.engine``).  Calling one of them directly raises.
"""
from __future__ import annotations

import torch.nn as nn


def _no_eager(name):
    def forward(self, *a, **k):
        raise RuntimeError(f"{name} is executed by the libzp engine; call the BinaryCodeNet_Deeplab module instead")
    return forward


class Conv2d(nn.Conv2d):
    forward = _no_eager("Conv2d")


class ConvTranspose2d(nn.ConvTranspose2d):
    forward = _no_eager("ConvTranspose2d")


class BatchNorm2d(nn.BatchNorm2d):
    forward = _no_eager("BatchNorm2d")


class ReLU(nn.ReLU):
    forward = _no_eager("ReLU")


class MaxPool2d(nn.MaxPool2d):
    forward = _no_eager("MaxPool2d")


class AdaptiveAvgPool2d(nn.AdaptiveAvgPool2d):
    forward = _no_eager("AdaptiveAvgPool2d")


class Linear(nn.Linear):
    forward = _no_eager("Linear")
