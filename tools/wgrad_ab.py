#!/usr/bin/env python3
"""Same-box A/B of the bf16 weight-gradient paths at bs = 32 (training geometry), interleaved rounds:
the ConvT weight gradient as four phases (k_wgrad_lds) or as the stride-2 conv over dy (k_wgrad2,
Engine._convT_wgrad_swap), and the stride-2 convs on k_wgrad2 (zp_conv_tuning key 3 = 1) or the
general kernel (key 3 = 0).  TFLOP/s are the algorithmic 2 * pixels * taps * Cin * Cout.
  python tools/wgrad_ab.py [--rounds 3] [--iters 10]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("ZP_QUIET", "1")

CASES = {  # name: (kind, cin, cout, k, s, p, H (input), B)
    "up2T": ("convT", 320, 256, 3, 2, 1, 64, 32),
    "up1T": ("convT", 256, 256, 3, 2, 1, 32, 32),
    "l2a": ("conv", 64, 128, 3, 2, 1, 64, 32),
    "l2ds": ("conv", 64, 128, 1, 2, 0, 64, 32),
    "l4": ("conv", 256, 256, 3, 1, 2, 32, 32),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default=",".join(CASES))
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from zebrapose_amd import _lib as L
    from zebrapose_amd.engine import Engine, Unit, Act
    from zebrapose_amd.model import layers as LY
    dev = torch.device("cuda", 0)
    setups = []
    for name in a.cases.split(","):
        kind, cin, cout, k, s, p, H, B = CASES[name]
        d = 2 if name == "l4" else 1
        if kind == "conv":
            conv = LY.Conv2d(cin, cout, k, s, p, d, bias=False).to(dev)
        else:
            conv = LY.ConvTranspose2d(cin, cout, k, s, p, output_padding=1, bias=False).to(dev)
        unit = Unit(conv, None, relu=False)
        OH, OW = unit.out_hw(H, H)
        x = Act(torch.randn(B, H, H, cin, device=dev).to(torch.bfloat16))
        dy = Act(torch.randn(B, OH, OW, cout, device=dev).to(torch.bfloat16))
        taps = k * k
        grid = H * H if kind == "convT" else OH * OW
        fl = 2.0 * B * grid * taps * cin * cout
        variants = [("swap", 1), ("phases", 1)] if kind == "convT" else [("lean", 1), ("general", 0)]
        setups.append((name, unit, x, dy, fl, variants, H))
    res, ref = {}, {}
    for r in range(a.rounds):
        for name, unit, x, dy, fl, variants, H in setups:
            for vname, key3 in variants:
                eng = Engine(torch.nn.Module(), torch.bfloat16)
                eng.convT_wgrad_swap = vname == "swap"
                old = L.lib.zp_conv_tuning(3, key3)
                try:
                    dw = torch.empty_like(unit.conv.weight)
                    plan = unit.fwd_plan(H, H)
                    for _ in range(2):
                        eng._wgrad(unit, x, plan, dy, dw)
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        eng._wgrad(unit, x, plan, dy, dw)
                    e1.record()
                    torch.cuda.synchronize()
                finally:
                    L.lib.zp_conv_tuning(3, old)
                us = e0.elapsed_time(e1) * 1e3 / a.iters
                if r == 0:
                    w0 = ref.setdefault(name, dw.clone())
                    rel = float((dw - w0).norm() / w0.norm())
                    print(f"{name} {vname}: rel L2 vs {variants[0][0]} {rel:.3g}", flush=True)
                res.setdefault((name, vname), []).append(us)
                print(f"round {r} {name} {vname}: {us:.1f} us", flush=True)
    for (name, vname), v in sorted(res.items()):
        fl = [s[4] for s in setups if s[0] == name][0]
        us = min(v)
        print(f"{name:6s} {vname:8s}: {us:8.1f} us  {fl / us * 1e-6:7.1f} TFLOP/s  ({fl / us * 1e-6 / 2516.6:.3f} of bf16 peak)")


if __name__ == "__main__":
    main()
