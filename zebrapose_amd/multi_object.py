"""Batched multi-object inference (BASELINE configs[4], SURVEY §8(e) "C5 multi-object"): many
objects' networks resident on one GPU, one batch of crops tagged by object, decoded and solved
on the device in one launch each.

Reference: ``test_vivo.py:99-114, 138-175`` (and ``test.py``) build ONE ``BinaryCodeNet_Deeplab``
per object, load its checkpoint, and run detections one crop at a time: forward ->
``from_output_to_class_mask/_binary_code`` -> ``CNN_outputs_to_object_pose`` with the object's
LUT (``dict_class_id_3D_points``) and the image's ``cam_K``.  Here all objects' weights stay in
HBM (packed to fp16 / bf16 NHWC tiles on first use; 30 R50 objects = 61 GB with the f32
masters), a batch's crops are grouped by object (one forward per object present, on the same
stream), and the whole batch goes through ``zp_decode`` with a per-crop LUT index and through
``zp_pnp_ransac`` with per-crop intrinsics.  Results come back in the caller's crop order.
"""
from __future__ import annotations

import numpy as np
import torch

from .decode import Decoder
from .pnp import PnP


class MultiObjectPose:
    def __init__(self, nets, luts, precision="fp16", bbox_size=128, ignore_bit=0, device="cuda",
                 pnp=None):
        """nets: one ``BinaryCodeNet_Deeplab`` per object (same code length); luts: the matching
        [2^L, 3] class-id -> vertex tables (``read_lut_file`` / ``load_dict_class_id_3D_points``)."""
        if len(nets) != len(luts) or not nets:
            raise ValueError("one LUT per object network")
        self.nets = list(nets)
        for n in self.nets:
            n.eval()
            if precision is not None:
                n.set_precision(precision)
        self.decoder = Decoder(list(luts), device=device, ignore_bit=ignore_bit)
        self.bbox_size = int(bbox_size)
        self.pnp = pnp or PnP()

    @torch.no_grad()
    def __call__(self, crops, obj_index, bboxes, K=None):
        """crops f32 [B, 3, 256, 256] (device, normalised as bop_dataset_pytorch.py:333-347);
        obj_index int [B] (index into ``nets``); bboxes int [B, 4] (post ``get_final_Bbox``);
        K 3x3 or [B, 3, 3].  Returns a dict of device tensors in crop order: mask / code logits,
        counts / xy / xyz (decode), R / t / success / inliers (PnP)."""
        B = crops.shape[0]
        obj = np.asarray(obj_index, dtype=np.int64).reshape(B)
        if B == 0:
            raise ValueError("empty batch")
        if obj.min() < 0 or obj.max() >= len(self.nets):
            raise ValueError("object index out of range")
        order = np.argsort(obj, kind="stable")
        dev = crops.device
        order_t = torch.from_numpy(order).to(dev)
        xs = crops.index_select(0, order_t) if not np.array_equal(order, np.arange(B)) else crops
        so = obj[order]
        bounds = np.flatnonzero(np.diff(so)) + 1
        starts = np.concatenate([[0], bounds])
        ends = np.concatenate([bounds, [B]])
        masks, codes = [], []
        for s, e in zip(starts, ends):
            m, c = self.nets[int(so[s])](xs[s:e])
            masks.append(m)
            codes.append(c)
        mask = torch.cat(masks) if len(masks) > 1 else masks[0]
        code = torch.cat(codes) if len(codes) > 1 else codes[0]
        bb = np.asarray(bboxes).reshape(B, 4)[order]
        if K is not None:
            K = np.asarray(K, dtype=np.float64)
            if K.ndim == 3:
                K = K[order]
        counts, xy, xyz = self.decoder(mask, code, bb, bbox_size=self.bbox_size, lut_index=so.astype(np.int32))
        R, t, ok, inl = self.pnp(counts, xy, xyz, K)
        inv = torch.from_numpy(np.argsort(order, kind="stable")).to(dev)
        out = dict(mask=mask, code=code, counts=counts, xy=xy, xyz=xyz, R=R, t=t, success=ok, inliers=inl)
        if not np.array_equal(order, np.arange(B)):
            out = {k: v.index_select(0, inv) for k, v in out.items()}
        return out
