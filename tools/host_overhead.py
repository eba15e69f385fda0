#!/usr/bin/env python3
"""Host-side enqueue time vs synchronised step time (is a step launch-bound?): R34 bs=32 256x256
bf16 training step (configs[2]) and eval forward + decode (configs[1]).

    python tools/host_overhead.py [--steps 5]"""
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
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    import bench
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    from zebrapose_amd.train import TrainStep
    dev = torch.device("cuda", 0)
    B = a.batch
    x = bench.synthetic_crops(B, 256, dev, 0)
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="bf16").to(dev)
    bench.calibrate_bn(net, x)
    net.train()
    ts = TrainStep(net, learning_rate=2e-4)
    g = torch.Generator(device="cpu").manual_seed(1)
    gt_code = torch.randint(0, 2, (B, 16, 128, 128), generator=g, dtype=torch.uint8).to(dev)
    gt_mask = torch.randint(0, 2, (B, 128, 128), generator=g).float().to(dev)
    for _ in range(3):
        ts(x, gt_code, gt_mask)
    torch.cuda.synchronize()
    enq, tot = [], []
    for _ in range(a.steps):
        t0 = time.perf_counter()
        ts(x, gt_code, gt_mask)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        enq.append((t1 - t0) * 1e3)
        tot.append((t2 - t0) * 1e3)
    print(f"train: enqueue {np.median(enq):.2f} ms, step {np.median(tot):.2f} ms")
    # host time to each phase mark vs GPU time between the marks' events (synchronised step)
    rows = []
    for _ in range(a.steps):
        torch.cuda.synchronize()
        ts.events = []
        marks = {}
        orig = ts._mark

        def mark(label, orig=orig, marks=marks):
            marks[label] = time.perf_counter()
            orig(label)
        ts._mark = mark
        ts(x, gt_code, gt_mask)
        ts._mark = orig
        torch.cuda.synchronize()
        ev = dict(ts.events)
        rows.append((
            (marks["backward"] - marks["start"]) * 1e3, ev["start"].elapsed_time(ev["backward"]),
            (marks["optimizer"] - marks["backward"]) * 1e3, ev["backward"].elapsed_time(ev["optimizer"]),
            (marks["end"] - marks["optimizer"]) * 1e3, ev["optimizer"].elapsed_time(ev["end"])))
    ts.events = None
    m = np.median(np.array(rows), axis=0)
    print(f"train phases host/gpu ms: fwd+loss {m[0]:.2f}/{m[1]:.2f}  backward {m[2]:.2f}/{m[3]:.2f}  "
          f"optimizer {m[4]:.2f}/{m[5]:.2f}")
    # back-to-back steps without a sync in between (what bench.py times)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ts(x, gt_code, gt_mask)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"train back-to-back: enqueue {(t1 - t0) / a.steps * 1e3:.2f} ms/step, wall {(t2 - t0) / a.steps * 1e3:.2f} ms/step")
    net.eval()
    with torch.no_grad():
        for _ in range(3):
            net(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            net(x)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    print(f"eval forward back-to-back: enqueue {(t1 - t0) / a.steps * 1e3:.2f} ms/step, wall {(t2 - t0) / a.steps * 1e3:.2f} ms/step")


if __name__ == "__main__":
    main()
