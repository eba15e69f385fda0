"""Drop-in for reference ``zebrapose/model/BinaryCodeNet_v3.py``: the 3-head
network of ``train_v5.py`` -- visible mask, entire mask and binary code.

``BinaryCodeNet_Deeplab_v3(34, L, 2, concat=True)`` has the reference's module tree and
state_dict keys (``net.resnet.*``, ``net.aspp.*`` as BinaryCodeNet_Deeplab, plus
``net.aspp_v3.*``); ``forward(x) -> (mask, entire_mask, code)`` (BinaryCodeNet_v3.py:152-169).
Forward and backward run in libzp through ``Engine.forward_v3`` / ``Engine.backward``: the
gradient of the entire-mask loss flows through the v3 head into the encoder features and, via
the resampled mask inputs, into the visible-mask logits, as autograd does in the reference.
The reference builds its encoder only for ResNet34 (:148-151).  Losses: ``BinaryCodeLoss`` and
``MaskLoss`` of ``zebrapose_amd.model.BinaryCodeNet`` (train_v5.py:236-237, 321-332).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from .BinaryCodeNet import _PREC, BinaryCodeLoss, MaskLoss  # noqa: F401  (train_v5 imports these too)
from .aspp import ASPP
from .aspp_v3 import ASPP_v3
from .resnet import ResNet34_OS8
from .. import staged as _staged
from ..engine import Engine
from ..parallel import finish_grads, grads_sink


class _DeepLabV3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, module, x, *params):
        mask, entire, code, tape = module._engine.forward_v3(x, train=True)
        ctx.module, ctx.tape = module, tape
        ctx.keys = [p.data_ptr() for p in params]
        return mask, entire, code

    @staticmethod
    def backward(ctx, dmask, dentire, dcode):
        sink = grads_sink(ctx.module)
        grads = finish_grads(ctx.module, ctx.module._engine.backward(ctx.tape, dmask, dcode, dentire, grads=sink))
        ctx.tape = None
        by_ptr = {p.data_ptr(): g for p, g in grads.items()}
        return (None, None) + tuple(by_ptr.get(k) for k in ctx.keys)


class DeepLabV3(nn.Module):
    """BinaryCodeNet_v3.py:143-169."""

    def __init__(self, num_resnet_layers, num_classes, concat=False, output_kernel_size=1, precision=None):
        super().__init__()
        self.num_classes = num_classes
        self.concat = concat
        self.num_resnet_layers = num_resnet_layers
        if num_resnet_layers != 34:
            raise NotImplementedError("BinaryCodeNet_Deeplab_v3 builds its encoder for ResNet34 only "
                                      "(BinaryCodeNet_v3.py:148-151)")
        self.resnet = ResNet34_OS8(34, concat)
        self.aspp = ASPP(num_classes=self.num_classes, concat=concat, output_kernel_size=output_kernel_size)
        self.aspp_v3 = ASPP_v3(num_classes=1, concat=concat, output_kernel_size=output_kernel_size)
        prec = precision or os.environ.get("ZP_PRECISION", "fp32")
        object.__setattr__(self, "_engine", Engine(self, _PREC[prec]))

    def set_precision(self, precision):
        object.__setattr__(self, "_engine", Engine(self, _PREC[precision]))

    def forward(self, x):
        params = [p for p in self.parameters()]
        if self.training and torch.is_grad_enabled() and any(p.requires_grad for p in params):
            if self._engine.dtype == torch.float16:
                raise RuntimeError("precision='fp16' is inference-only; train in 'bf16' or 'fp32'")
            if _staged.enabled(self):  # torch DDP over the unchanged DistributedDataParallel(net) line
                mask, entire, code, tape = self._engine.forward_v3(x, train=True)
                return _staged.staged(self, self._engine, (mask, entire, code), tape)
            return _DeepLabV3Fn.apply(self, x, *params)
        mask, entire, code, _ = self._engine.forward_v3(x, train=self.training)
        return mask, entire, code


class BinaryCodeNet_Deeplab_v3(nn.Module):
    """BinaryCodeNet_v3.py:123-140."""

    def __init__(self, num_resnet_layers, binary_code_length, divided_number_each_iteration, concat=False,
                 output_kernel_size=1, precision=None):
        super().__init__()
        self.concat = concat
        if divided_number_each_iteration != 2:
            raise NotImplementedError("only the binary (divided_number_each_iteration == 2) network exists in v3")
        self.net = DeepLabV3(num_resnet_layers, binary_code_length + 1, concat=self.concat,
                             output_kernel_size=output_kernel_size, precision=precision)

    def set_precision(self, precision):
        self.net.set_precision(precision)

    def forward(self, inputs):
        return self.net(inputs)
