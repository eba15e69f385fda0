#!/usr/bin/env python3
"""Per-op accuracy of the fp32 eval engines (split-fp32 ZP_F32X3 and ZP_F32H2, exact-f32 MFMA) at the bench
geometry (R34, bs=32, 256x256, BN calibrated at 256): every traced op of crop 13 replayed in float64
from the device's own stored (joined) inputs; per op the rms and max error relative to the op's
rms / max output, side by side; then the end-to-end logits against a float64 forward."""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("ZP_QUIET", "1")


def main():
    from oracle import ref_cpu
    from tests.test_gpu_bench_geometry import bench_crops, _label, _nchw, _bn_of
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "r34_bn_buffers256.npz")))
    sd = ref_cpu.synthetic_state(34, 16, 0, g)
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="fp32")
    net.load_state_dict(sd)
    net = net.cuda().eval()
    x = bench_crops().cuda()
    b = 13
    res = {}
    forms = ("x3", "h2", False)
    for split in forms:
        net.net.f32_split = split
        eng = net.net.eval_engine()
        eng.trace = []
        with torch.no_grad():
            m, c = net(x)
        torch.cuda.synchronize()
        rows = []
        for i, rec in enumerate(eng.trace):
            kind, unit, xa, out, r = rec
            if kind not in ("conv", "head"):
                continue
            conv = unit.conv
            xin = _nchw(xa, b)[:, :unit.cin_w].double()
            w = conv.weight.detach().double().cpu()
            bias = None if conv.bias is None else conv.bias.detach().double().cpu()
            if kind == "head":
                exp = F.conv2d(xin, w, bias)
                mask, code = out
                got = torch.cat([mask[b:b + 1].cpu(), code[b:b + 1].cpu()], 1).double()
            else:
                if unit.kind == "convT":
                    acc = F.conv_transpose2d(xin, w, None, 2, 1, 1)
                else:
                    acc = F.conv2d(xin, w, None, unit.s, unit.p, unit.d)
                bn = _bn_of(unit)
                if bn is None:
                    y = acc + (0 if bias is None else bias.view(1, -1, 1, 1))
                else:
                    s, sh = ref_cpu.fold_f32(*bn, bias=bias)
                    y = acc * s.double().view(1, -1, 1, 1) + sh.double().view(1, -1, 1, 1)
                if r is not None:
                    y = y + _nchw(r, b).double()
                exp = F.relu(y) if unit.relu else y
                got = _nchw(out, b).double()
            d = got - exp
            rows.append((i, _label(rec, i), (d.pow(2).mean().sqrt() / exp.pow(2).mean().sqrt()).item(),
                         (d.abs().max() / exp.abs().max()).item(), d.mean().item() / exp.abs().mean().item()))
        eng.trace = None
        res[split] = (rows, m.cpu(), c.cpu())
    name = {"x3": "x3", "h2": "h2", False: "f32"}
    print(f"{'op':44s}" + "".join(f" {name[k] + ' rms':>10s}" for k in forms) + "".join(f" {name[k] + ' max':>10s}" for k in forms)
          + "".join(f" {name[k] + ' bias':>10s}" for k in forms))
    for rows in zip(*(res[k][0] for k in forms)):
        print(f"{rows[0][1][:44]:44s}" + "".join(f" {r[2]:10.3g}" for r in rows) + "".join(f" {r[3]:10.3g}" for r in rows)
              + "".join(f" {r[4]:10.3g}" for r in rows))
    idx = [0, 13, 31]
    with torch.no_grad():
        sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
        dm, dc = ref_cpu.forward(sd64, x.cpu()[idx].double(), 34)
    for split in forms:
        _, m, c = res[split]
        for nm, got, ref in (("mask", m[idx], dm), ("code", c[idx], dc)):
            d = got.double() - ref
            print(f"{name[split]:4s} {nm}: vs float64 max {d.abs().max().item():.3g} rms "
                  f"{d.pow(2).mean().sqrt().item():.3g} mean {d.mean().item():.3g}")


if __name__ == "__main__":
    main()
