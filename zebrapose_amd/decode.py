"""Device code -> vertex decode, host wrapper over ``zp_decode``.

``Decoder`` keeps the class-id -> 3D LUT(s) resident on the device (f32 [n_obj][2^L][3],
768 KB per object at L = 16) and turns a batch of network outputs into ordered 2D-3D
correspondences without leaving the GPU:

    counts[b]          number of mask pixels of crop b
    xy[b, :counts[b]]  original-image pixel (x, y), int32, row-major mask order
    xyz[b, :counts[b]] LUT vertex (f32), [0, 0, 0] for empty (NaN) classes

Reference: binary_code_helper/CNN_output_to_pose.py:10-64, 100-130,
class_id_encoder_decoder.py:17-28, generate_new_dict.py:4-33, common_ops.py:5-19.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L


def read_lut_file(path):
    """Parse the generator's LUT text file (Generate_Mesh_with_GT_Color.cpp:616-624; loader
    CNN_output_to_pose.py:10-32): header ``"N divide iterations"`` then ``"id x y z"`` lines.
    Returns (total_class, divide_number, iterations, f64 array [N, 3] indexed by id)."""
    with open(path, "r") as f:
        head = f.readline().split(" ")
        total = float(head[0])
        divide = float(head[1])
        iters = float(head[2])
        n = int(total)
        lut = np.full((n, 3), np.nan)
        for line in f:
            parts = line.rstrip("\n").split(" ")
            if len(parts) < 4:
                continue
            lut[int(float(parts[0]))] = [float(parts[1]), float(parts[2]), float(parts[3])]
    return total, divide, iters, lut


class Decoder:
    """Batched on-device decode for one or several objects (lut_index per crop)."""

    def __init__(self, luts, device="cuda", ignore_bit=0):
        if isinstance(luts, np.ndarray) and luts.ndim == 2:
            luts = [luts]
        full_bits = int(round(np.log2(np.asarray(luts[0]).shape[0])))
        self.full_bits = full_bits
        self.ignore_bit = ignore_bit
        self.bits = full_bits - ignore_bit
        tabs = []
        for lut in luts:
            lut = np.asarray(lut, dtype=np.float64)
            if lut.shape != (2 ** full_bits, 3):
                raise ValueError("every LUT must be [2^L, 3]")
            d64 = torch.from_numpy(np.ascontiguousarray(lut)).to(device)
            # ignore_bit > 0: f64 mean of the 2^k children; ignore_bit == 0: the f64 -> f32 cast
            out = torch.empty((2 ** self.bits, 3), dtype=torch.float32, device=device)
            L.call("zp_lut_coarsen", d64.data_ptr(), full_bits, self.bits, out.data_ptr(), L.stream_ptr())
            tabs.append(out)
        self.lut = torch.stack(tabs).contiguous()
        self.device = torch.device(device)

    def __call__(self, mask_logits, code_logits, bboxes, bbox_size=128, lut_index=None, return_ids=False):
        mask_logits = mask_logits.detach().contiguous().float()
        code_logits = code_logits.detach().contiguous().float()
        B, _, H, W = mask_logits.shape
        Lfull = code_logits.shape[1]
        if Lfull < self.bits:
            raise ValueError("fewer code channels than LUT bits")
        dev = mask_logits.device
        if torch.is_tensor(bboxes) and bboxes.device == dev and bboxes.dtype == torch.int32:
            bb = bboxes.reshape(B, 4).contiguous()  # already on the device (graph capture: no host copy)
        else:
            bb = torch.as_tensor(np.asarray(bboxes), dtype=torch.int32).reshape(B, 4).to(dev).contiguous()
        li = None
        if lut_index is not None:
            li = torch.as_tensor(np.asarray(lut_index), dtype=torch.int32).reshape(B).to(dev).contiguous()
        counts = torch.empty(B, dtype=torch.int32, device=dev)
        xy = torch.empty((B, H * W, 2), dtype=torch.int32, device=dev)
        xyz = torch.empty((B, H * W, 3), dtype=torch.float32, device=dev)
        ids = torch.empty((B, H, W), dtype=torch.int32, device=dev) if return_ids else None
        ws = torch.empty(int(L.lib.zp_decode_ws_bytes(B, H, W)), dtype=torch.uint8, device=dev)
        L.call("zp_decode", mask_logits.data_ptr(), code_logits.data_ptr(), B, H, W, Lfull, self.bits,
               self.lut.data_ptr(), L.ptr(li), bb.data_ptr(), int(bbox_size), L.ptr(ids), counts.data_ptr(),
               xy.data_ptr(), xyz.data_ptr(), ws.data_ptr(), L.stream_ptr())
        if return_ids:
            return counts, xy, xyz, ids
        return counts, xy, xyz

    @staticmethod
    def to_host(counts, xy, xyz):
        """-> list of (P2D int64 [N, 2], P3D float32 [N, 3]) per crop."""
        c = counts.cpu().numpy()
        xy = xy.cpu().numpy()
        xyz = xyz.cpu().numpy()
        return [(xy[b, :c[b]].astype(np.int64), xyz[b, :c[b]].copy()) for b in range(len(c))]
