#!/usr/bin/env python3
"""A/B of training-step variants in ONE process (interleaved rounds, median + min): bench.py's R34
bs=32 256x256 bf16 training step (forward + loss + backward + Adam), synthetic crops / codes.

    python tools/train_ab.py --variants side,noside [--rounds 5 --steps 10]

variant = '+'-joined knobs: side / noside (weight gradients on the engine's second stream or not),
ymask (BN backward reads the stored activation for the ReLU mask instead of recomputing it from raw),
r<N> (k_wgrad2 workgroup rounds, zp_conv_tuning key 4), l<N> (k_wgrad_lds rounds, key 5), phases (the
ConvT weight gradient as four phases instead of the stride-2 conv over dy), nolean (k_wgrad2 off)."""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("ZP_QUIET", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="side,noside")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    import bench
    import zebrapose_amd._lib as L
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    from zebrapose_amd.train import TrainStep
    dev = torch.device("cuda", 0)
    B, S = a.batch, 256
    x = bench.synthetic_crops(B, S, dev, 0)
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="bf16").to(dev)
    bench.calibrate_bn(net, x)
    net.train()
    ts = TrainStep(net, learning_rate=2e-4)
    eng = next(m._engine for m in net.modules() if hasattr(m, "_engine"))
    g = torch.Generator(device="cpu").manual_seed(7)
    gt_code = (torch.rand((B, 16, S // 2, S // 2), generator=g) < 0.5).to(torch.uint8).to(dev)
    gt_mask = (torch.rand((B, S // 2, S // 2), generator=g) < 0.7).float().to(dev)

    def apply(v):
        parts = v.split("+")
        eng.side_wgrad = "noside" not in parts
        eng.bn_mask_from_raw = "ymask" not in parts
        eng.convT_wgrad_swap = "phases" not in parts  # (round 6) ConvT weight gradient as four phases
        L.lib.zp_conv_tuning(3, 0 if "nolean" in parts else 1)  # k_wgrad2 off: the general kernel
        r = [int(q[1:]) for q in parts if q.startswith("r") and q[1:].isdigit()]
        L.lib.zp_conv_tuning(4, r[0] if r else 1)
        lr = [int(q[1:]) for q in parts if q.startswith("l") and q[1:].isdigit()]
        L.lib.zp_conv_tuning(5, lr[0] if lr else 1)

    variants = a.variants.split(",")
    times = {v: [] for v in variants}
    host = {v: [] for v in variants}
    for v in variants:  # warm every variant (packing caches, allocator pools)
        apply(v)
        for _ in range(2):
            ts(x, gt_code, gt_mask)
    torch.cuda.synchronize()
    for r in range(a.rounds):
        for v in variants:
            apply(v)
            ts(x, gt_code, gt_mask)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                loss = ts(x, gt_code, gt_mask)
            host[v].append((time.perf_counter() - t0) / a.steps * 1e3)  # enqueue time (host side)
            torch.cuda.synchronize()
            times[v].append((time.perf_counter() - t0) / a.steps * 1e3)
    for v in variants:
        print(f"{v:>16s}: {np.median(times[v]):7.3f} ms/step (min {np.min(times[v]):7.3f}; host enqueue {np.median(host[v]):7.3f})  loss {float(loss[0]):.4f}",
              flush=True)


if __name__ == "__main__":
    main()
