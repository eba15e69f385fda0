"""Drop-in for reference ``zebrapose/common_ops.py`` (:5-38).

The logit -> bit threshold runs on the device (``zp_threshold``): sigmoid(x) > 0.5 as the
reference evaluates it on the CPU in fp32 is exactly ``x > 8.940696716308594e-08``
(NaN -> 0); the result is returned as the reference's float64 0/1 numpy array.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L


def _threshold_f64(t: torch.Tensor) -> torch.Tensor:
    t = t.detach()
    if not t.is_cuda:
        raise ValueError("expected a device (HIP) tensor of logits")
    t = t.contiguous().float()
    out = torch.empty(t.shape, dtype=torch.float64, device=t.device)
    L.call("zp_threshold", t.data_ptr(), t.numel(), 1, out.data_ptr(), L.stream_ptr())
    return out


def threshold_device(logits: torch.Tensor) -> torch.Tensor:
    """Device-resident f64 0/1 bits (no host round trip)."""
    return _threshold_f64(logits)


def from_output_to_class_mask(pred_mask_prob, thershold=0.5):
    """common_ops.py:5-11 -> numpy float64 0/1 of the same shape."""
    if thershold != 0.5:
        raise NotImplementedError("only the 0.5 threshold of the reference is implemented on device")
    return _threshold_f64(pred_mask_prob).cpu().numpy()


def from_output_to_class_binary_code(pred_code_prob, BinaryCode_Loss_Type, thershold=0.5,
                                     divided_num_each_interation=2, binary_code_length=16):
    """common_ops.py:13-32 (BCE / L1 branch; the CE branch is an ablation outside the hot path)."""
    if BinaryCode_Loss_Type not in ("BCE", "L1"):
        raise NotImplementedError("CE binary code decoding is not part of the hot path")
    if thershold != 0.5:
        raise NotImplementedError("only the 0.5 threshold of the reference is implemented on device")
    return _threshold_f64(pred_code_prob).cpu().numpy()


def get_batch_size(second_dataset_ratio, batch_size):
    """common_ops.py:35-38."""
    batch_size_2_dataset = int(batch_size * second_dataset_ratio)
    batch_size_1_dataset = batch_size - batch_size_2_dataset
    return batch_size_1_dataset, batch_size_2_dataset


__all__ = ["from_output_to_class_mask", "from_output_to_class_binary_code", "get_batch_size", "threshold_device",
           "np"]
