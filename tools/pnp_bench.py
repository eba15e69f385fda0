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
    a = ap.parse_args()
    from zebrapose_amd.pnp import PnP
    rng = np.random.default_rng(0)
    HW = 16384
    xy = torch.from_numpy(rng.integers(0, 640, (a.batch, HW, 2)).astype(np.int32)).cuda()
    xyz = torch.from_numpy(rng.uniform(-50, 50, (a.batch, HW, 3)).astype(np.float32)).cuda()
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
