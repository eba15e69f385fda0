#!/usr/bin/env python3
"""Split-fp32 conv (k_conv3) layer timing under several schedule flag sets, one process, interleaved
rounds (same-box A/B):  python tools/conv3_ab.py [--flags 478,470,...] [--layers ...]
Layers: the network's heaviest split-fp32 launches at bs=32.  Algorithmic TFLOP/s are f32 FLOPs
(2 * pixels * taps * Cin * Cout); the ceiling is 2516.6 / 6 = 419 TFLOP/s."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("ZP_QUIET", "1")

LAYERS = {  # name: (kind, cin, cout, k, d, hw)
    "up2conv": ("conv", 256, 256, 3, 1, 128),
    "l5": ("conv", 512, 512, 3, 4, 32),
    "up2T": ("convT", 320, 256, 3, 1, 64),
    "up1T": ("convT", 256, 256, 3, 1, 32),
    "up1conv": ("conv", 256, 256, 3, 1, 64),
    "l1": ("conv", 64, 64, 3, 1, 64),
    "l2": ("conv", 128, 128, 3, 1, 32),
    "l4": ("conv", 256, 256, 3, 2, 32),
    "l4a": ("conv", 128, 256, 3, 2, 32),      # layer4's first conv (128 -> 256)
    "proj": ("conv", 1280, 256, 1, 1, 32),    # ASPP conv_1x1_3
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags", default="478")
    ap.add_argument("--layers", default="up2conv,l5,up2T")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--strip", default="-1", help="zp_conv_tuning key 7 values to A/B (k_conv3s: 0 off, 1, 2)")
    ap.add_argument("--form", default="x3", choices=["x3", "h2"])
    ap.add_argument("--minblocks", default="256", help="zp_conv_tuning key 8 values to A/B (comma list)")
    ap.add_argument("--wide", default="-1", help="zp_conv_tuning key 10 values to A/B (k_conv3w: 0 off, 1 on)")
    ap.add_argument("--splitk", default="1", help="zp_conv_tuning key 12 values to A/B (k_conv3w split-K: 0, 1, 2)")
    ap.add_argument("--acc", default="-1", help="zp_conv_tuning key 13 values to A/B (k_conv3w accumulation: 0 flushed, "
                    "1 one scaled accumulator, 2 per-step partial)")
    ap.add_argument("--tp128", default="-1", help="zp_conv_tuning key 14 values to A/B (k_conv3w 256 x 128 tile: 0, 1)")
    ap.add_argument("--subint", default="-1", help="zp_conv_tuning key 16 values to A/B (k_conv3 multi-sub interleave: 0, 1)")
    ap.add_argument("--mf32", default="-1", help="zp_conv_tuning key 18 values to A/B (k_conv3w on 32x32x16 MFMAs: 0, 1)")
    ap.add_argument("--pfb", default="-1", help="zp_conv_tuning key 21 values to A/B (k_conv3w strip tile: next-step "
                    "pixel fragments read before the barrier: 0, 1)")
    ap.add_argument("--graph", action="store_true", help="time hipGraph replays of the iters launches (no host "
                    "launch overhead: the bs = 1 launches are shorter than their eager enqueue)")
    ap.add_argument("--wsubint", default="-1", help="zp_conv_tuning key 17 values to A/B (k_conv3w ConvT phases "
                    "interleaved per pixel tile: 0, 1)")
    a = ap.parse_args()
    from zebrapose_amd import _lib as L
    from zebrapose_amd.engine import Engine, Unit, Act
    from zebrapose_amd.model import layers as LY
    dev = torch.device("cuda", 0)
    flags = [int(f) for f in a.flags.split(",")]
    res = {}
    setups = []
    for name in a.layers.split(","):
        if name == "aspp":  # the merged ASPP launch: 1x1 + 3x3 d6 / d12 / d18, 512 -> 4 x 256 at 32 x 32
            eng = Engine(torch.nn.Module(), torch.float32, split=a.form)
            units = []
            for kk, dd in ((1, 1), (3, 6), (3, 12), (3, 18)):
                conv = LY.Conv2d(512, 256, kk, 1, 0 if kk == 1 else dd, dd, bias=True).to(dev)
                units.append(Unit(conv, LY.BatchNorm2d(256).to(dev).eval(), relu=True))
            xs = eng._empty((a.batch, 32, 32, 512), dev)
            xs._base.copy_(torch.randn(xs._base.shape, device=dev).clamp(min=0).to(xs.dtype))
            A = eng._empty((a.batch, 32, 32, 1280), dev)
            outs = [Act(A, 256 * i, 256) for i in range(4)]
            fl = 2.0 * a.batch * 32 * 32 * (1 + 9 + 9 + 9) * 512 * 256

            class _Aspp:
                def __init__(s2, units, outs):
                    s2.units, s2.outs = units, outs
            setups.append((name, eng, _Aspp(units, outs), Act(xs), Act(A), fl))
            continue
        kind, cin, cout, k, d, hw = LAYERS[name]
        if kind == "conv":
            conv = LY.Conv2d(cin, cout, k, 1, d * (k // 2), d, bias=False).to(dev)
        else:
            conv = LY.ConvTranspose2d(cin, cout, 3, 2, 1, output_padding=1, bias=False).to(dev)
        bn = LY.BatchNorm2d(cout).to(dev).eval()
        unit = Unit(conv, bn, relu=True)
        eng = Engine(torch.nn.Module(), torch.float32, split=a.form)
        xs = eng._empty((a.batch, hw, hw, cin), dev)
        xs._base.copy_(torch.randn(xs._base.shape, device=dev).clamp(min=0).to(xs.dtype))
        OH, OW = unit.out_hw(hw, hw)
        y = Act(eng._empty((a.batch, OH, OW, cout), dev))
        taps = 9 if kind == "conv" else 9 / 4 * 4  # convT: 4 phases x 9/4 taps over the input grid
        fl = 2.0 * a.batch * hw * hw * (k * k if kind == "conv" else 9) * cin * cout
        setups.append((name, eng, unit, Act(xs), y, fl))
    mbs = [int(m) for m in a.minblocks.split(",")]
    strips = [int(m) for m in a.strip.split(",")]
    wides = [int(m) for m in a.wide.split(",")]
    sks = [int(m) for m in a.splitk.split(",")]
    accs = [int(m) for m in a.acc.split(",")]
    t128 = [int(m) for m in a.tp128.split(",")]
    sis = [int(m) for m in a.subint.split(",")]
    wsis = [int(m) for m in a.wsubint.split(",")]
    mfs = [int(m) for m in a.mf32.split(",")]
    pfbs = [int(m) for m in a.pfb.split(",")]
    first = {}
    import itertools
    for r in range(a.rounds):
        for f0, mb, sm, wd, sk, ac, tq, si, ws, mf, pb in itertools.product(flags, mbs, strips, wides, sks, accs, t128,
                                                                             sis, wsis, mfs, pfbs):
            L.lib.zp_conv_tuning(1, f0)
            L.lib.zp_conv_tuning(8, mb)
            L.lib.zp_conv_tuning(7, sm)
            L.lib.zp_conv_tuning(10, wd)
            L.lib.zp_conv_tuning(12, sk)
            L.lib.zp_conv_tuning(13, ac)
            L.lib.zp_conv_tuning(14, tq)
            L.lib.zp_conv_tuning(16, si)
            L.lib.zp_conv_tuning(17, ws)
            L.lib.zp_conv_tuning(18, mf)
            L.lib.zp_conv_tuning(21, pb)
            f = (f0, mb, sm, wd, sk, ac, tq, si, ws, mf, pb)
            for name, eng, unit, x, y, fl in setups:
                def run1():
                    if hasattr(unit, "outs"):
                        eng.aspp_branches_fwd(unit.units, x, unit.outs, None)
                    else:
                        eng.unit_fwd(unit, x, y, None)
                for _ in range(2):
                    run1()
                torch.cuda.synchronize()
                if r == 0:  # outputs of every setting against the first one (bit-identical expected)
                    ref = first.setdefault(name, y.buf._base.clone())
                    nd = int((ref != y.buf._base).sum())
                    if nd:
                        msg = ""
                        if a.form == "h2" and ref.dim() == 5 and ref.dtype == torch.float16:
                            def join(b):
                                return b[0].float() + b[1].float() / 2048.0
                            jr, jy = join(ref), join(y.buf._base)
                            msg = (f"; joined f32: max |diff| {float((jr - jy).abs().max()):.3e}, "
                                   f"max |ref| {float(jr.abs().max()):.3e}")
                        print(f"{name} {f}: {nd} of {ref.numel()} stored halves differ from the first setting{msg}")
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                if a.graph:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        for _ in range(a.iters):
                            run1()
                    g.replay()
                    torch.cuda.synchronize()
                    e0.record()
                    g.replay()
                    e1.record()
                    torch.cuda.synchronize()
                    del g
                else:
                    e0.record()
                    for _ in range(a.iters):
                        run1()
                    e1.record()
                    torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / a.iters
                res.setdefault((name, f), []).append(us)
    L.lib.zp_conv_tuning(1, -1)
    L.lib.zp_conv_tuning(8, 256)
    L.lib.zp_conv_tuning(7, -1)
    L.lib.zp_conv_tuning(10, -1)
    L.lib.zp_conv_tuning(12, 1)
    L.lib.zp_conv_tuning(13, -1)
    L.lib.zp_conv_tuning(14, -1)
    L.lib.zp_conv_tuning(16, -1)
    L.lib.zp_conv_tuning(17, -1)
    L.lib.zp_conv_tuning(18, -1)
    L.lib.zp_conv_tuning(21, -1)
    for (name, f), v in sorted(res.items()):
        fl = [s[5] for s in setups if s[0] == name][0]
        us = min(v)
        print(f"{name:8s} flags {f[0]:6d} minblocks {f[1]:4d} strip {f[2]:2d} wide {f[3]:2d} splitk {f[4]} acc {f[5]:2d} tp128 {f[6]:2d} subint {f[7]:2d} wsubint {f[8]:2d} mf32 {f[9]:2d} pfb {f[10]:2d}: {us:9.1f} us  {fl / us * 1e-6:7.1f} TFLOP/s  ({fl / us * 1e-6 / (2516.6 / (6 if a.form == 'x3' else 3)):.3f} of the {a.form} ceiling)")


if __name__ == "__main__":
    main()
