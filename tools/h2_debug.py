#!/usr/bin/env python3
"""Diagnostic: run the bench-geometry forward through the x3 and h2 split engines and compare every
traced op's joined output (convs, pools, broadcast) between them, crop 13."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("ZP_QUIET", "1")


def main():
    from oracle import ref_cpu
    from tests.test_gpu_bench_geometry import bench_crops, _label
    from zebrapose_amd.engine import joined
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "r34_bn_buffers256.npz")))
    sd = ref_cpu.synthetic_state(34, 16, 0, g)
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="fp32")
    net.load_state_dict(sd)
    net = net.cuda().eval()
    x = bench_crops().cuda()
    outs = {}
    for form in ("x3", "h2"):
        net.net.f32_split = form
        eng = net.net.eval_engine()
        eng.trace = []
        with torch.no_grad():
            m, c = net(x)
        torch.cuda.synchronize()
        recs = []
        for i, rec in enumerate(eng.trace):
            kind, unit, xa, out, r = rec
            if kind == "head":
                o = torch.cat([out[0], out[1]], 1).cpu()
            elif isinstance(out, torch.Tensor):
                o = out.cpu()
            else:
                o = joined(out.buf)[..., out.c0:out.c0 + out.C].cpu()
            recs.append((kind, i, o))
        eng.trace = None
        outs[form] = recs
    for (k, i, a), (_, _, b) in zip(outs["x3"], outs["h2"]):
        d = (a.double() - b.double()).abs()
        per = d.reshape(d.shape[0], -1).max(1).values
        worst = int(per.argmax())
        loc = (d[worst] == d[worst].max()).nonzero()[0].tolist()
        print(f"{i:3d} {k:10s} max|x3-h2| {d.max().item():.3g} (crop {worst} at {loc}; median crop "
              f"{per.median().item():.3g})  scale {a.abs().max().item():.3g}  h2 finite {bool(torch.isfinite(b).all())}")


if __name__ == "__main__":
    main()
