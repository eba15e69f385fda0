#!/usr/bin/env python3
"""Same-box A/B of zp_conv_tuning settings on the whole fp32 (two-plane) forward + decode, hipGraph
replayed, at bs = 1 (the reference's per-crop test.py loop) and bs = 32 (the headline), interleaved
over rounds.  Each setting's outputs are compared with the first setting's (the ring depth and
schedule knobs keep the sums in the same order: bit-identical expected).
  python tools/bs1_ab.py --key 19 --values 2,3,4 [--batches 1,32] [--rounds 3]"""
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
    ap.add_argument("--key", type=int, default=19)
    ap.add_argument("--values", default="2,3,4")
    ap.add_argument("--batches", default="1,32")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters1", type=int, default=200)
    ap.add_argument("--iters32", type=int, default=20)
    a = ap.parse_args()
    import bench
    from zebrapose_amd import _lib as L
    from zebrapose_amd.decode import Decoder
    from zebrapose_amd.graphs import GraphedInference
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    dev = torch.device("cuda", 0)
    S = 256
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="fp32").to(dev).eval()
    bench.calibrate_bn(net, bench.synthetic_crops(4, S, dev, seed=3))
    net.eval()
    dec = Decoder(bench.synthetic_lut(), device=dev)
    vals = [int(v) for v in a.values.split(",")]
    res, first = {}, {}
    for r in range(a.rounds):
        for B in [int(b) for b in a.batches.split(",")]:
            x = bench.synthetic_crops(B, S, dev, seed=7)
            bb = np.tile(np.array([[100, 80, 200, 200]]), (B, 1))
            iters = a.iters1 if B == 1 else a.iters32
            for v in vals:
                old = L.lib.zp_conv_tuning(a.key, v)
                try:
                    g = GraphedInference(net, B, S, decoder=dec, bbox_size=S // 2)
                    for _ in range(3):
                        out = g(x, bb)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(iters):
                        g(x, bb)
                    torch.cuda.synchronize()
                    ms = (time.perf_counter() - t0) / iters * 1e3
                    with torch.no_grad():
                        m, c = net(x)
                    torch.cuda.synchronize()
                    ref = first.setdefault(B, (m.clone(), c.clone()))
                    nd = int((ref[0] != m).sum()) + int((ref[1] != c).sum())
                    if nd:
                        print(f"bs={B} key {a.key}={v}: {nd} logits differ from key {a.key}={vals[0]} "
                              f"(max |d| {float((ref[1] - c).abs().max()):.3e})", flush=True)
                    del g, out
                finally:
                    L.lib.zp_conv_tuning(a.key, old)
                res.setdefault((B, v), []).append(ms)
                print(f"round {r} bs={B} key {a.key}={v}: {ms:.3f} ms per step", flush=True)
    for (B, v), ms in sorted(res.items()):
        print(f"bs={B:3d} key {a.key}={v}: min {min(ms):.3f} ms, all {[round(m, 3) for m in ms]}")


if __name__ == "__main__":
    main()
