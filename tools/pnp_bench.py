#!/usr/bin/env python3
"""Times zp_pnp_ransac on a batch of synthetic crops (for rocprofv3): B crops x N random
correspondences (worst case: no early RANSAC termination) or --scene (a real pose, 30% outliers)."""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("ZP_QUIET", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--n", type=int, default=7000)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--scene", action="store_true")
    a = ap.parse_args()
    from zebrapose_amd.pnp import PnP
    rng = np.random.default_rng(0)
    HW = 16384
    xy = torch.from_numpy(rng.integers(0, 640, (a.batch, HW, 2)).astype(np.int32)).cuda()
    xyz = torch.from_numpy(rng.uniform(-50, 50, (a.batch, HW, 3)).astype(np.float32)).cuda()
    if a.scene:  # a real pose per crop, 30% outliers: RANSAC terminates early, the refine runs
        K = np.array([[572.4114, 0.0, 325.2611], [0.0, 573.57043, 242.04899], [0.0, 0.0, 1.0]])
        pw = rng.uniform(-60, 60, (a.batch, HW, 3))
        t = np.stack([rng.uniform(-60, 60, a.batch), rng.uniform(-60, 60, a.batch), rng.uniform(500, 1100, a.batch)], 1)
        Xc = pw + t[:, None]
        uv = np.stack([K[0, 0] * Xc[..., 0] / Xc[..., 2] + K[0, 2], K[1, 1] * Xc[..., 1] / Xc[..., 2] + K[1, 2]], -1)
        uv = np.round(uv + rng.normal(0, 0.5, uv.shape))
        out = rng.random((a.batch, HW)) < 0.3
        uv[out] += rng.uniform(-120, 120, (int(out.sum()), 2))
        xy = torch.from_numpy(uv.astype(np.int32)).cuda()
        xyz = torch.from_numpy(pw.astype(np.float32)).cuda()
    counts = torch.full((a.batch,), a.n, dtype=torch.int32).cuda()
    p = PnP()
    p(counts, xy, xyz)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        p(counts, xy, xyz)
    torch.cuda.synchronize()
    print(f"pnp {(time.perf_counter() - t0) / a.iters * 1e3:.3f} ms / batch of {a.batch}")


if __name__ == "__main__":
    main()
