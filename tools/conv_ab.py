#!/usr/bin/env python3
"""A/B of conv schedule variants in ONE process (interleaved rounds, median + min), eval forward
(BN folded, ReLU), bf16, random activations.  Variants are zp_conv_tuning knobs (key 1 = conv flags,
key 0 = 256-channel-tile threshold).  Every variant's output is compared bitwise with the first
variant's (a schedule change must not change a single bit: same K order per output).

    python tools/conv_ab.py --layers 256:256:128:1,512:512:32:4 --flags 28,60 [--rounds 7 --iters 10]

layer = cin:cout:hw:dilation[:k]  (3x3 by default; batch --batch); T<cin>:<cout>:<hw> a ConvTranspose2d
(3, s2) and S<cin>:<cout>:<hw>[:1:k] a stride-2 conv of an hw input.  Variant knobs: r<N> = k_wgrad2
rounds (key 4), l<N> = k_wgrad_lds rounds (key 5; l0 = the 1024-workgroup target).  A variant is a flags value,
optionally with extra knobs: "94+noc64" sets zp_conv_tuning(2, 0) (64-channel layers on k_conv)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("ZP_QUIET", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default="256:256:128:1,512:512:32:4,256:256:32:2,256:256:64:1")
    ap.add_argument("--flags", default="28,60")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--json", default=None)
    ap.add_argument("--wgrad", action="store_true", help="time the weight gradient (dy = the output buffer)")
    a = ap.parse_args()
    import zebrapose_amd._lib as L
    from zebrapose_amd.engine import Engine, Unit, Act
    from zebrapose_amd.model import layers as LY
    dev = torch.device("cuda", 0)
    flags = a.flags.split(",")

    def apply(v):
        parts = v.split("+")
        L.lib.zp_conv_tuning(1, int(parts[0]))
        L.lib.zp_conv_tuning(2, 0 if "noc64" in parts[1:] else 1)
        L.lib.zp_conv_tuning(0, 1 << 30 if "no256" in parts[1:] else (1 if "all256" in parts[1:] else 1024))
        L.lib.zp_conv_tuning(3, 0 if "now2" in parts[1:] else 1)
        tg = [int(q[1:]) for q in parts[1:] if q.startswith("r") and q[1:].isdigit()]
        L.lib.zp_conv_tuning(4, tg[0] if tg else 1)
        lg = [int(q[1:]) for q in parts[1:] if q.startswith("l") and q[1:].isdigit()]
        L.lib.zp_conv_tuning(5, lg[0] if lg else 1)
    rows = []
    for spec in a.layers.split(","):
        tr = spec.startswith("T")  # T<cin>:<cout>:<hw>: ConvTranspose2d(3, s2, p1, op1) (aspp.py:60-80)
        s2 = spec.startswith("S")  # S<cin>:<cout>:<hw>[:1:k]: stride-2 conv, hw = input size
        f = [int(v) for v in spec.lstrip("TS").split(":")]
        cin, cout, hw = f[:3]
        d = f[3] if len(f) > 3 else 1
        k = f[4] if len(f) > 4 else 3
        torch.manual_seed(0)
        if tr:
            conv = LY.ConvTranspose2d(cin, cout, 3, 2, 1, 1, bias=False).to(dev)
        else:
            conv = LY.Conv2d(cin, cout, k, 2 if s2 else 1, d * (k // 2), d, bias=False).to(dev)
        torch.nn.init.normal_(conv.weight, 0, (2.0 / (cin * k * k)) ** 0.5)
        bn = LY.BatchNorm2d(cout).to(dev).eval()
        unit = Unit(conv, bn, relu=True)
        eng = Engine(torch.nn.Module(), torch.bfloat16)
        x = Act(torch.randn(a.batch, hw, hw, cin, device=dev).bfloat16())
        ohw = 2 * hw if tr else (hw // 2 if s2 else hw)
        y = Act(torch.empty(a.batch, ohw, ohw, cout, device=dev, dtype=torch.bfloat16))
        fl = 2.0 * a.batch * hw * hw * k * k * cin * cout  # ConvT: 9 taps per input pixel as well
        if s2:
            fl /= 4
        dw = torch.empty_like(conv.weight)
        if a.wgrad:
            y.buf.copy_(torch.randn(y.buf.shape, device=dev).clamp(min=0).bfloat16())
        plan = unit.fwd_plan(hw, hw)

        def run():
            if a.wgrad:
                eng._wgrad(unit, x, plan, y, dw)
            else:
                eng.unit_fwd(unit, x, y, None)
        times = {fv: [] for fv in flags}
        ref = None
        for r in range(a.rounds):
            for fv in flags:
                apply(fv)
                run()
                torch.cuda.synchronize()
                if r == 0 and a.wgrad:
                    if ref is None:
                        ref = dw.clone()
                    else:
                        rel = float((dw - ref).norm() / ref.norm())
                        if not rel < 1e-5:
                            print(f"!! {spec} flags {fv}: dw rel diff {rel:.3g} vs flags {flags[0]}", flush=True)
                elif r == 0:
                    if ref is None:
                        ref = y.buf.clone()
                    else:
                        same = torch.equal(ref.view(torch.int16), y.buf.view(torch.int16))
                        if not same:
                            nd = int((ref.view(torch.int16) != y.buf.view(torch.int16)).sum())
                            print(f"!! {spec} flags {fv}: output differs from flags {flags[0]} in {nd} elements",
                                  flush=True)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                times[fv].append(e0.elapsed_time(e1) * 1e3 / a.iters)
        L.lib.zp_conv_tuning(1, -1)
        L.lib.zp_conv_tuning(2, 1)
        L.lib.zp_conv_tuning(0, 1024)
        L.lib.zp_conv_tuning(3, 1)
        L.lib.zp_conv_tuning(4, 1)
        L.lib.zp_conv_tuning(5, 1)
        for fv in flags:
            med, mn = float(np.median(times[fv])), float(np.min(times[fv]))
            row = {"layer": spec, "flags": fv, "us_median": round(med, 2), "us_min": round(mn, 2),
                   "tflops_median": round(fl / med * 1e-6, 1)}
            rows.append(row)
            print(f"{spec:>16s} flags {fv:>8s}: {med:8.1f} us (min {mn:8.1f})  {fl / med * 1e-6:7.1f} TFLOP/s", flush=True)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(rows, fh, indent=0)


if __name__ == "__main__":
    main()
