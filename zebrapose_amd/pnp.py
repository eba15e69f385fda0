"""Batched on-device RANSAC-EPnP over the decode's correspondences.

Replaces, per crop, the reference's
    cv2.solvePnPRansac(Points_3D, Original_Points_2D, K, None, reprojectionError=2,
                       iterationsCount=150, flags=cv2.SOLVEPNP_EPNP); cv2.Rodrigues(rvec)
(binary_code_helper/CNN_output_to_pose.py:152-156) for a whole batch in five kernel launches
(``zp_pnp_ransac``, csrc/zp_pnp.hip), with the reference's success rule (at least 6
correspondences, :126).  Inputs stay on the device: ``PnP()(counts, xy, xyz, K)`` takes
``Decoder``'s outputs directly.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L

LINEMOD_K = np.array([[572.4114, 0.0, 325.2611], [0.0, 573.57043, 242.04899], [0.0, 0.0, 1.0]])  # :101-108


class PnP:
    def __init__(self, iterations=150, reprojection_error=2.0, confidence=0.99, min_points=6):
        self.iterations = int(iterations)
        self.reprojection_error = float(reprojection_error)
        self.confidence = float(confidence)
        self.min_points = int(min_points)

    def __call__(self, counts, xy, xyz, K=None):
        """counts int32 [B], xy int32 [B, HW, 2], xyz f32 [B, HW, 3] (device); K: 3x3 or [B, 3, 3]
        (default: the reference's LINEMOD intrinsics).  Returns (R f64 [B,3,3], t f64 [B,3],
        success bool [B], inliers int32 [B]) on the device."""
        B, HW = xy.shape[0], xy.shape[1]
        dev = xy.device
        if xy.dtype != torch.int32 or xyz.dtype != torch.float32 or counts.dtype != torch.int32:
            raise ValueError("expected counts / xy int32 and xyz float32 (zp_decode outputs)")
        K = LINEMOD_K if K is None else np.asarray(K, dtype=np.float64)
        K = np.broadcast_to(K, (B, 3, 3))
        kv = torch.from_numpy(np.ascontiguousarray(np.stack([K[:, 0, 0], K[:, 1, 1], K[:, 0, 2], K[:, 1, 2]], 1)))
        kv = kv.to(dev)
        R = torch.empty((B, 3, 3), dtype=torch.float64, device=dev)
        t = torch.empty((B, 3), dtype=torch.float64, device=dev)
        ok = torch.empty(B, dtype=torch.int32, device=dev)
        inl = torch.empty(B, dtype=torch.int32, device=dev)
        ws = torch.empty(int(L.lib.zp_pnp_ws_bytes(B, self.iterations)), dtype=torch.uint8, device=dev)
        xy, xyz, counts = xy.contiguous(), xyz.contiguous(), counts.contiguous()
        L.call("zp_pnp_ransac", B, HW, counts.data_ptr(), xy.data_ptr(), xyz.data_ptr(), kv.data_ptr(),
               self.iterations, self.reprojection_error, self.confidence, R.data_ptr(), t.data_ptr(),
               ok.data_ptr(), inl.data_ptr(), ws.data_ptr(), L.stream_ptr())
        success = (ok != 0) & (counts >= self.min_points)
        return R, t, success, inl
