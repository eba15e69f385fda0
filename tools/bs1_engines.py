#!/usr/bin/env python3
"""bs=1 (the reference's per-crop test.py loop) forward + decode latency per fp32 eval engine (h2 /
x3 split, exact-f32 MFMA) and bf16, eager and hipGraph; plus the h2 engine's per-conv launch times
at bs=1 (HIP events, eager)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("ZP_QUIET", "1")


def main():
    import bench
    from zebrapose_amd.decode import Decoder
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    dev = torch.device("cuda", 0)
    S = 256
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="fp32").to(dev).eval()
    dec = Decoder(bench.synthetic_lut(), device=dev)
    for prec, split in (("fp32", "h2"), ("fp32", "x3"), ("fp32", False), ("bf16", None)):
        net.set_precision(prec)
        net.net.f32_split = split if split is not None else True
        r = bench.bs1_leg(net, dec, S, dev, iters=30)
        print(f"{prec} split={split}: {r}", flush=True)
    net.set_precision("fp32")
    net.net.f32_split = "h2"
    eng = net.net.eval_engine()
    x1 = bench.synthetic_crops(1, S, dev, seed=7)
    with torch.no_grad():
        net(x1)
    eng.timing = []
    with torch.no_grad():
        net(x1)
    torch.cuda.synchronize()
    rows = [(e0.elapsed_time(e1) * 1e3, label, kname) for label, e0, e1, fl, kname, nb in eng.timing]
    eng.timing = None
    print(f"h2 bs=1 conv launches: {len(rows)}, sum {sum(r[0] for r in rows):.1f} us")
    for us, label, kname in sorted(rows, reverse=True)[:15]:
        print(f"  {us:8.1f} us  {label[:60]:60s} {kname}")


if __name__ == "__main__":
    main()
