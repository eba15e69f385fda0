"""Drop-in for reference ``binary_code_helper/generate_new_dict.py:4-33`` (ignore_bit LUT).

The coarse table (f64 mean of the 2^(old-new) children, NaN-propagating) is computed on the
device by ``zp_lut_coarsen``; the reference's dict return type is kept."""
from __future__ import annotations

import numpy as np
import torch

from .. import _lib as L


def coarsen_lut(lut_f64, num_bit_old_dict, num_bit_new_dict, device="cuda"):
    """f64 [2^old, 3] -> f32 [2^new, 3] on the device."""
    d64 = torch.from_numpy(np.ascontiguousarray(np.asarray(lut_f64, dtype=np.float64))).to(device)
    out = torch.empty((2 ** num_bit_new_dict, 3), dtype=torch.float32, device=device)
    L.call("zp_lut_coarsen", d64.data_ptr(), num_bit_old_dict, num_bit_new_dict, out.data_ptr(), L.stream_ptr())
    return out


def generate_new_corres_dict(full_binary_corres_dict, num_bit_old_dict, num_bit_new_dict):
    """Returns {new_id: array [1, 3]} like the reference (values as float32-rounded f64)."""
    n = 2 ** num_bit_old_dict
    lut = np.stack([np.asarray(full_binary_corres_dict[float(i)] if float(i) in full_binary_corres_dict
                               else full_binary_corres_dict[i], dtype=np.float64).reshape(3) for i in range(n)])
    out = coarsen_lut(lut, num_bit_old_dict, num_bit_new_dict).cpu().numpy().astype(np.float64)
    return {i: out[i].reshape(1, 3) for i in range(out.shape[0])}
