"""Drop-in for reference ``zebrapose/model/BinaryCodeNet.py`` on MI355X.

``from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab, BinaryCodeLoss, MaskLoss``
gives the same constructors, module tree / ``state_dict`` keys (392 keys, 96 aliased,
152 parameters for ResNet34), forward signature ``forward(x) -> (mask_logits, code_logits)``
and loss call signatures as the reference (BinaryCodeNet.py:8-174).  The forward and
backward run in libzp (HIP kernels for gfx950) through ``zebrapose_amd.engine``; there is
no PyTorch-op fallback.

Precision: ``precision='fp32'`` (default) is the reference's fp32 arithmetic, within its
tolerance.  Training runs every convolution with exact-f32 MFMA (``v_mfma_f32_16x16x4_f32``) and f32
activations; the eval forward runs a split-fp32 engine, chosen by ``f32_split`` (``ZP_F32_SPLIT``):
  "h2" / True (default): include/zp.h ZP_F32H2 -- activations and weights as two fp16 planes
      (v = hi + lo * 2^-11, 22 bits), every product from hi*hi + (hi*lo + lo*hi) * 2^-11 on fp16
      MFMAs with f32 accumulation (3 MFMAs per f32 MAC); fp16's range is guarded (activations
      |v| >= 65520, weights |w| >= 32 raise a device flag and the forward re-runs on "x3");
  "x3": ZP_F32X3 -- three bf16 planes summing exactly to the f32 value, six bf16 MFMA terms;
  False: exact-f32 MFMA.
Against a float64 forward "x3" is about 2x closer than exact-f32 MFMA and "h2" about as close
(its 256 x 256 tile keeps one f32 accumulator per product block).  ``precision='bf16'``
uses bf16 MFMA with f32 accumulation and bf16 NHWC activations -- the throughput mode
(configs 2-4); ``precision='fp16'`` is the same with IEEE fp16 (``v_mfma_f32_16x16x32_f16``),
inference only (configs[4]: R50 multi-object inference).  Set per instance (``net.set_precision``) or with ``ZP_PRECISION``.
"""
from __future__ import annotations

import os
import warnings

import torch
import torch.nn as nn

from .. import _lib as L
from .. import staged as _staged
from ..engine import Engine
from ..parallel import finish_grads, grads_sink
from .aspp import ASPP, ASPP_50
from .resnet import ResNet34_OS8, ResNet50_OS8

SPLIT_FORMS = ("x3", "h2")  # include/zp.h ZP_F32X3 / ZP_F32H2
DEFAULT_SPLIT = "h2"  # the fp32 eval forward's split form when f32_split is True

model_urls = {
    "resnet18": "https://download.pytorch.org/models/resnet18-5c106cde.pth",
    "resnet34": "https://download.pytorch.org/models/resnet34-333f7ec4.pth",
    "resnet50": "https://download.pytorch.org/models/resnet50-19c8e357.pth",
}

_PREC = {"fp32": torch.float32, "f32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16,
         "f16": torch.float16}


# ============================================================================ losses
class _CodeLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, code, mask01, mask_logits, gt, hist_state, use_hist, mask_code):
        code = code.contiguous()
        B, Lb, H, W = code.shape
        gt_f64 = 1 if gt.dtype == torch.float64 else 0
        if not gt_f64:
            gt = gt.to(torch.uint8)
        gt = gt.contiguous()
        dev = code.device
        ws = torch.empty(int(L.lib.zp_code_loss_ws_bytes(B, Lb, H, W)), dtype=torch.uint8, device=dev)
        out = torch.empty(2, dtype=torch.float64, device=dev)
        coef = torch.empty(Lb, dtype=torch.float64, device=dev)
        L.call("zp_code_loss", code.data_ptr(), L.ptr(mask01), L.ptr(mask_logits), gt.data_ptr(), gt_f64, B, Lb, H, W,
               int(use_hist), int(mask_code), hist_state.data_ptr(), out.data_ptr(), coef.data_ptr(), ws.data_ptr(),
               L.stream_ptr())
        ctx.save_for_backward(code, mask01 if mask01 is not None else mask_logits, gt, coef)
        ctx.meta = (mask01 is not None, gt_f64, mask_code)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        code, m, gt, coef = ctx.saved_tensors
        is01, gt_f64, mask_code = ctx.meta
        B, Lb, H, W = code.shape
        g = g.to(torch.float64).contiguous()
        dcode = torch.empty_like(code)
        L.call("zp_code_loss_bwd", code.data_ptr(), m.data_ptr() if is01 else None, None if is01 else m.data_ptr(),
               gt.data_ptr(), gt_f64, B, Lb, H, W, int(mask_code), coef.data_ptr(), g.data_ptr(), dcode.data_ptr(),
               L.stream_ptr())
        return dcode, None, None, None, None, None, None


class BinaryCodeLoss(nn.Module):
    """BinaryCodeNet.py:8-67.  Device implementation of the configuration the trainers use
    ('BCE', mask_binary_code_loss, histogram-weighted or plain); 'L1' / 'CE' are ablation
    branches outside the hot path."""

    def __init__(self, binary_code_loss_type, mask_binary_code_loss, divided_number_each_iteration,
                 use_histgramm_weighted_binary_loss=False):
        super().__init__()
        if binary_code_loss_type != "BCE":
            raise NotImplementedError(f"binary code loss type {binary_code_loss_type!r}: only 'BCE' runs on device")
        self.binary_code_loss_type = binary_code_loss_type
        self.mask_binary_code_loss = mask_binary_code_loss
        self.divided_number_each_iteration = divided_number_each_iteration
        self.use_histgramm_weighted_binary_loss = use_histgramm_weighted_binary_loss
        self._hist = None  # f64 [L + 1] device state: EMA histogram + "initialised" flag

    @property
    def histogram(self):
        """BinaryCodeNet.py:32,37-41 module state (None before the first call; per rank; not saved)."""
        if self._hist is None or not self.use_histgramm_weighted_binary_loss:
            return None
        return self._hist[:-1]

    def _state(self, L_, dev):
        if self._hist is None or self._hist.numel() != L_ + 1 or self._hist.device != dev:
            self._hist = torch.zeros(L_ + 1, dtype=torch.float64, device=dev)
        return self._hist

    def forward(self, pred_binary_code, pred_mask, groundtruth_code):
        """pred_mask: the 0/1 mask (f64 in the reference, train_v6.py:325-326)."""
        if pred_mask.dtype != torch.float64:
            pred_mask = pred_mask.to(torch.float64)
        st = self._state(pred_binary_code.shape[1], pred_binary_code.device)
        return _CodeLossFn.apply(pred_binary_code, pred_mask.contiguous(), None, groundtruth_code, st,
                                 self.use_histgramm_weighted_binary_loss, self.mask_binary_code_loss)

    def forward_from_logits(self, pred_binary_code, pred_mask_logits, groundtruth_code):
        """Same loss with the mask thresholded on device from the mask logits (no host round trip)."""
        st = self._state(pred_binary_code.shape[1], pred_binary_code.device)
        return _CodeLossFn.apply(pred_binary_code, None, pred_mask_logits.detach().contiguous(), groundtruth_code, st,
                                 self.use_histgramm_weighted_binary_loss, self.mask_binary_code_loss)


class BinaryLossWeighted(nn.Module):
    """BinaryCodeNet.py:70-81 (fused into zp_code_loss; kept for API completeness)."""

    def __init__(self, baseloss=None):
        super().__init__()
        self.base_loss = baseloss


class _MaskLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g):
        x = x.contiguous()
        g = g.contiguous().float()
        n = x.numel()
        assert g.numel() == n
        out = torch.empty((), dtype=torch.float32, device=x.device)
        ws = torch.empty(int(L.lib.zp_mask_loss_ws_bytes(n)), dtype=torch.uint8, device=x.device)
        L.call("zp_mask_loss", x.data_ptr(), g.data_ptr(), n, out.data_ptr(), ws.data_ptr(), L.stream_ptr())
        ctx.save_for_backward(x, g)
        return out

    @staticmethod
    def backward(ctx, gs):
        x, g = ctx.saved_tensors
        gs = gs.to(torch.float32).contiguous()
        dx = torch.empty_like(x)
        L.call("zp_mask_loss_bwd", x.data_ptr(), g.data_ptr(), x.numel(), gs.data_ptr(), dx.data_ptr(),
               L.stream_ptr())
        return dx, None


class MaskLoss(nn.Module):
    """BinaryCodeNet.py:84-93: L1(sigmoid(mask[:, 0]), gt_mask), mean."""

    def forward(self, pred_mask, groundtruth_mask):
        if pred_mask.shape[1] != 1:
            raise ValueError("MaskLoss expects [B, 1, H, W] mask logits")
        return _MaskLossFn.apply(pred_mask, groundtruth_mask)


class HammingLoss(nn.Module):
    """BinaryCodeNet.py:96-109 -- computed inside zp_code_loss (histogram + mean)."""

    def forward(self, predicted_code_prob, GT_code, mask):
        st = torch.zeros(predicted_code_prob.shape[1] + 1, dtype=torch.float64, device=predicted_code_prob.device)
        fn = BinaryCodeLoss("BCE", True, 2, True)
        fn._hist = st
        with torch.no_grad():
            fn.forward(predicted_code_prob, mask, GT_code)
        h = st[:-1].clone()
        return h.mean(), h


# ============================================================================ network
class _DeepLabFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, module, x, *params):
        mask, code, tape = module._engine.forward(x, train=True)
        ctx.module, ctx.tape = module, tape
        ctx.keys = [p.data_ptr() for p in params]
        ctx.param_like = [(p.shape, p.dtype, p.device) for p in params]
        return mask, code

    @staticmethod
    def backward(ctx, dmask, dcode):
        sink = grads_sink(ctx.module)
        grads = finish_grads(ctx.module, ctx.module._engine.backward(ctx.tape, dmask, dcode, grads=sink))
        ctx.tape = None
        by_ptr = {p.data_ptr(): g for p, g in grads.items()}
        out = []
        for k, (shape, dt, dev) in zip(ctx.keys, ctx.param_like):
            g = by_ptr.get(k)
            out.append(g)
        return (None, None) + tuple(out)


class DeepLabV3(nn.Module):
    """BinaryCodeNet.py:146-174 (binary-code variant); forward executed by libzp."""

    def __init__(self, num_resnet_layers, num_classes, concat=False, output_kernel_size=1, precision=None):
        super().__init__()
        self.num_classes = num_classes
        self.concat = concat
        self.num_resnet_layers = num_resnet_layers
        if num_resnet_layers == 34:
            self.resnet = ResNet34_OS8(34, concat)
            self.aspp = ASPP(num_classes=self.num_classes, concat=concat, output_kernel_size=output_kernel_size)
        elif num_resnet_layers == 50:
            self.resnet = ResNet50_OS8(50, concat)
            self.aspp = ASPP_50(num_classes=self.num_classes, concat=concat, output_kernel_size=output_kernel_size)
        else:
            raise NotImplementedError("num_resnet_layers must be 34 or 50")
        prec = precision or os.environ.get("ZP_PRECISION", "fp32")
        object.__setattr__(self, "_engine", Engine(self, _PREC[prec]))
        object.__setattr__(self, "_engines_split", {})
        env = os.environ.get("ZP_F32_SPLIT", "1")
        self.f32_split = False if env == "0" else (env if env in SPLIT_FORMS else True)
        # range guard of the two-plane form (include/zp.h zp_split_range_flag): every "h2" eval
        # forward reads the device flag once when it is done (one 4-byte readback); a forward that
        # met a value beyond fp16's range is re-run on the full-range "x3" form, which this network
        # then keeps (range_fallbacks counts the switches).  ZP_RANGE_CHECK=0 turns the readback off.
        self.range_check = os.environ.get("ZP_RANGE_CHECK", "1") != "0"
        self.range_fallbacks = 0

    def set_precision(self, precision):
        object.__setattr__(self, "_engine", Engine(self, _PREC[precision]))
        object.__setattr__(self, "_engines_split", {})

    def eval_engine(self):
        """The engine that runs this network's eval (inference) forward: for precision 'fp32' the
        split-fp32 engine of form ``f32_split`` ("x3" / "h2"; True = DEFAULT_SPLIT; False / "off":
        the exact-f32 MFMA engine), else the precision's own engine."""
        sp = self.f32_split
        if self._engine.dtype == torch.float32 and sp and sp != "off":
            kind = sp if sp in SPLIT_FORMS else DEFAULT_SPLIT
            eng = self._engines_split.get(kind)
            if eng is None:
                eng = self._engines_split[kind] = Engine(self, torch.float32, split=kind)
            return eng
        return self._engine

    def h2_active(self):
        """True when the eval forward runs the two-plane split form (and so needs the range guard)."""
        if self.training or self._engine.dtype != torch.float32:
            return False
        eng = self.eval_engine()
        return eng.split == "h2"

    def range_fallback(self):
        """Switch the eval forward to the full-range three-plane form after a range-guard hit."""
        warnings.warn("zebrapose_amd: an activation or weight of the fp32 eval forward exceeds fp16's range "
                      "(activations |v| >= 65520, weights |w| >= 32); the two-plane split engine is replaced by the full-range x3 engine for "
                      "this network", RuntimeWarning, stacklevel=3)
        self.f32_split = "x3"
        self.range_fallbacks += 1
        # the two-plane packings may hold infinities: a later switch back to "h2" repacks (and
        # re-checks) them
        self._engines_split.pop("h2", None)

    @property
    def precision(self):
        return {torch.bfloat16: "bf16", torch.float16: "fp16"}.get(self._engine.dtype, "fp32")

    def forward(self, x):
        params = [p for p in self.parameters()]
        if self.training and torch.is_grad_enabled() and any(p.requires_grad for p in params):
            if self._engine.dtype == torch.float16:
                raise RuntimeError("precision='fp16' is inference-only (configs[4]); train in 'bf16' or 'fp32'")
            if _staged.enabled(self):  # torch DDP over the unchanged DistributedDataParallel(net) line
                mask, code, tape = self._engine.forward(x, train=True)
                return _staged.staged(self, self._engine, (mask, code), tape)
            return _DeepLabFn.apply(self, x, *params)
        eng = self._engine if self.training else self.eval_engine()
        mask, code, _ = eng.forward(x, train=self.training)
        if eng.split == "h2" and self.range_check and not torch.cuda.is_current_stream_capturing():
            # (a captured forward is checked by its GraphedInference after each replay).  The read
            # waits for the forward: every guarded eager call synchronises the host with the GPU
            flag = eng.range_word(x.device)
            hit = int(flag.item())
            eng.unread_packs = False
            if hit:
                self.range_fallback()
                mask, code, _ = self.eval_engine().forward(x, train=False)
        return mask, code


class BinaryCodeNet_Deeplab(nn.Module):
    """BinaryCodeNet.py:122-143."""

    def __init__(self, num_resnet_layers, binary_code_length, divided_number_each_iteration, concat=False,
                 output_kernel_size=1, precision=None):
        super().__init__()
        self.concat = concat
        if divided_number_each_iteration != 2:
            raise NotImplementedError("DeepLabV3_non_binary (CE ablation, BinaryCodeNet.py:177-196) is outside "
                                      "the hot path")
        self.net = DeepLabV3(num_resnet_layers, binary_code_length + 1, concat=self.concat,
                             output_kernel_size=output_kernel_size, precision=precision)

    def set_precision(self, precision):
        self.net.set_precision(precision)

    def forward(self, inputs):
        return self.net(inputs)
