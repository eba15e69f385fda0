#!/usr/bin/env python3
"""Diagnostic: the head (1x1, 320 -> 17) of the h2 split engine at the bench geometry against a
float64 recomputation from its own joined input; prints where the bad pixels are."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("ZP_QUIET", "1")


def main():
    from oracle import ref_cpu
    from tests.test_gpu_bench_geometry import bench_crops
    from zebrapose_amd.engine import joined
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "r34_bn_buffers256.npz")))
    sd = ref_cpu.synthetic_state(34, 16, 0, g)
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="fp32")
    net.load_state_dict(sd)
    net = net.cuda().eval()
    x = bench_crops().cuda()
    for form in sys.argv[1:] or ["h2", "x3"]:
        net.net.f32_split = form
        eng = net.net.eval_engine()
        eng.trace = []
        with torch.no_grad():
            net(x)
        torch.cuda.synchronize()
        kind, unit, xa, out, r = eng.trace[-1]
        assert kind == "head"
        xin = joined(xa.buf).double()  # [B, H, W, 320]
        w = unit.conv.weight.detach().double().view(17, 320)
        b = unit.conv.bias.detach().double()
        ref = torch.einsum("bhwc,oc->bohw", xin, w) + b.view(1, 17, 1, 1)
        got = torch.cat([out[0], out[1]], 1).double()
        d = (got - ref).abs()
        B, C, H, W = d.shape
        bad = (d > 1e-3).nonzero()
        print(f"{form}: max {d.max().item():.3g}, bad {len(bad)} of {d.numel()}")
        if len(bad):
            pix = (bad[:, 0] * H + bad[:, 2]) * W + bad[:, 3]
            print("  channels", torch.bincount(bad[:, 1], minlength=17).tolist())
            print("  pixel % 128 hist", torch.bincount(pix % 128, minlength=128).tolist())
            t = pix // 128
            print("  tiles", torch.unique(t).numel(), "first", torch.unique(t)[:20].tolist())
            print("  crops", torch.bincount(bad[:, 0], minlength=B).tolist())
        eng.trace = None


if __name__ == "__main__":
    main()
