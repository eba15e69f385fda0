"""Drop-in for reference ``zebrapose/metric.py``: ADD / ADI pose errors
computed on the device (``zp_pose_error``, csrc/zp_metric.hip).

``Calculate_ADD_Error_BOP`` / ``Calculate_ADI_Error_BOP`` keep the reference signatures
(metric.py:8-18: host arrays in, float out); ``pose_errors`` is the batched device form.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L

ADD, ADI = 0, 1


def pose_errors(pts, R_est, t_est, R_gt, t_gt, mode=ADD):
    """pts [n,3] (one model), R [B,3,3], t [B,3] (host or device) -> f64 [B] on the device."""
    dev = torch.device("cuda")
    p = torch.as_tensor(np.asarray(pts) if not torch.is_tensor(pts) else pts, dtype=torch.float32).reshape(-1, 3)
    p = p.to(dev).contiguous()

    def d64(x, shape):
        x = torch.as_tensor(x if torch.is_tensor(x) else np.asarray(x), dtype=torch.float64)
        return x.to(dev).reshape(shape).contiguous()
    Re = d64(R_est, (-1, 9))
    B = Re.shape[0]
    te, Rg, tg = d64(t_est, (B, 3)), d64(R_gt, (B, 9)), d64(t_gt, (B, 3))
    n = p.shape[0]
    out = torch.empty(B, dtype=torch.float64, device=dev)
    ws = torch.empty(int(L.lib.zp_pose_error_ws_bytes(B, n, mode)), dtype=torch.uint8, device=dev)
    L.call("zp_pose_error", B, p.data_ptr(), n, Re.data_ptr(), te.data_ptr(), Rg.data_ptr(), tg.data_ptr(), int(mode),
           out.data_ptr(), ws.data_ptr(), L.stream_ptr())
    return out


def Calculate_ADD_Error_BOP(R_GT, t_GT, R_predict, t_predict, vertices):
    """metric.py:8-12 -> pose_error.add(R_predict, t_predict, R_GT, t_GT, vertices)."""
    return float(pose_errors(vertices, R_predict, t_predict, R_GT, t_GT, ADD)[0].item())


def Calculate_ADI_Error_BOP(R_GT, t_GT, R_predict, t_predict, vertices):
    """metric.py:14-18 -> pose_error.adi(R_predict, t_predict, R_GT, t_GT, vertices)."""
    return float(pose_errors(vertices, R_predict, t_predict, R_GT, t_GT, ADI)[0].item())
