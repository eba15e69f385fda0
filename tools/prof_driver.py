#!/usr/bin/env python3
"""Kernel-level profiling driver for rocprofv3 (run on the GPU box by tools/prof_round.sh).

--mode train: K training steps (configs[2]: R34 bs=32 bf16, hist-weighted BCE + mask loss,
backward, Adam).  --mode infer: K eval forwards + decode (configs[1]) with NO train-mode BN
calibration pass, so every dispatch of a kernel in the trace belongs to an identical eval step
(the PMC per-launch averages in profiles/ are taken over exactly those).  Prints ms/step."""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("ZP_QUIET", "1")

from bench import calibrate_bn, synthetic_crops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--layer-report", default=None)
    ap.add_argument("--mode", default="train", choices=["train", "infer"])
    ap.add_argument("--stage-log", default=None, help="infer: write the last step's conv launches (stage, kernel, "
                                                       "flops, algorithmic bytes) in launch order here; train: "
                                                       "per kernel label, one step's launches, FLOPs and bytes")
    a = ap.parse_args()
    from bench import lib_sha16
    print(f"lib_sha16 {lib_sha16()}", flush=True)
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    from zebrapose_amd.train import TrainStep
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision=a.precision).to(dev)
    x = synthetic_crops(a.batch, 256, dev, seed=100)
    if a.mode == "infer":
        from bench import synthetic_lut
        from zebrapose_amd.decode import Decoder
        import numpy as np
        net.eval()
        dec = Decoder(synthetic_lut(), device=dev)
        bb = np.array([[10, 20, 128, 128]] * a.batch)

        def step():
            with torch.no_grad():
                m, c = net(x)
                return dec(m, c, bb, bbox_size=128)
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        eng = net.net.eval_engine()
        t0 = time.perf_counter()
        for i in range(a.steps):
            if a.stage_log and i == a.steps - 1:
                eng.stage_log = []  # host-side bookkeeping only: the dispatch sequence is unchanged
            step()
        torch.cuda.synchronize()
        print(f"infer ms/step {(time.perf_counter() - t0) / a.steps * 1e3:.3f}")
        if a.stage_log:
            with open(a.stage_log, "w") as f:
                json.dump({"precision": a.precision, "batch": a.batch, "lib_sha16": lib_sha16(),
                           "launches": [{"stage": st, "kernel": k, "flops": fl, "bytes": nb, "geo": geo}
                                        for st, k, fl, nb, geo in eng.stage_log]}, f, indent=0)
            eng.stage_log = None
        return
    calibrate_bn(net, x)
    net.train()
    ts = TrainStep(net, learning_rate=2e-4)
    g = torch.Generator(device="cpu").manual_seed(7)
    gt_code = (torch.rand((a.batch, 16, 128, 128), generator=g) < 0.5).to(torch.uint8).to(dev)
    gt_mask = (torch.rand((a.batch, 128, 128), generator=g) < 0.7).float().to(dev)
    for _ in range(a.warmup):
        ts(x, gt_code, gt_mask)
    torch.cuda.synchronize()
    if a.stage_log:  # train: per kernel label, the step's launches, algorithmic FLOPs and bytes (engine timing)
        from bench import lib_sha16
        eng = net.net._engine
        eng.timing = []
        ts(x, gt_code, gt_mask)
        torch.cuda.synchronize()
        agg = {}
        for label, e0, e1, flops, kname, nbytes in eng.timing:
            d = agg.setdefault(kname, {"launches": 0, "flops": 0.0, "bytes": 0.0, "us": 0.0})
            d["launches"] += 1
            d["flops"] += flops
            d["bytes"] += nbytes
            d["us"] += e0.elapsed_time(e1) * 1e3
        eng.timing = None
        with open(a.stage_log, "w") as f:
            json.dump({"precision": a.precision, "batch": a.batch, "lib_sha16": lib_sha16(), "mode": "train",
                       "kernels": agg}, f, indent=1)
    if a.layer_report:
        eng = net.net._engine
        eng.timing = []
        ts(x, gt_code, gt_mask)
        torch.cuda.synchronize()
        lay = {}
        for label, e0, e1, flops, kname, _ in eng.timing:
            d = lay.setdefault(label, [kname, 0.0, 0.0, 0])
            d[1] += e0.elapsed_time(e1) * 1e3
            d[2] += flops
            d[3] += 1
        eng.timing = None
        rows = sorted(({"label": k, "kernel": v[0], "n": v[3], "us_total": round(v[1], 1),
                        "tflops": round(v[2] / v[1] * 1e-6, 1)} for k, v in lay.items()), key=lambda r: -r["us_total"])
        with open(a.layer_report, "w") as f:
            json.dump(rows, f, indent=0)
        print(f"conv+wgrad total {sum(r['us_total'] for r in rows) / 1e3:.2f} ms")
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ts(x, gt_code, gt_mask)
    torch.cuda.synchronize()
    print(f"train ms/step {(time.perf_counter() - t0) / a.steps * 1e3:.3f}")


if __name__ == "__main__":
    main()
