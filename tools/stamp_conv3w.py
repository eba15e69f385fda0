#!/usr/bin/env python3
"""Where the wide two-plane tile's K loop spends its cycles: runs single layers (bs 32, fp32 two-plane)
on the diagnostic library built by tools/stamp_build.sh (ZP_LIB=tools/stamp/libzp_stamp.so: the same
kernels with shader-clock stamps, zp_conv3w.hip ZP_STAMP) and reads every wave's segment sums of the
last launch:
  [0] step start (past the previous barrier) -> the step's first fragments landed (lgkmcnt wait),
  [1] -> the end of the step's 8 cout blocks (MFMAs, flushes, later fragment waits, DMA issue),
  [2] -> the next step's LDS-DMA landed (vm_wait),
  [3] -> past the workgroup barrier.
Cycles are shader clocks (s_memtime); the stamps themselves cost a few percent (MI355X_MICROARCH.md).
  python tools/stamp_conv3w.py [--layers up2conv,l5,up1conv,up2T]"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("ZP_LIB", os.path.join(ROOT, "tools", "stamp", "libzp_stamp.so"))
os.environ.setdefault("ZP_QUIET", "1")

import numpy as np  # noqa: E402
import torch  # noqa: E402

LAYERS = {  # name: (kind, cin, cout, k, d, hw)
    "up2conv": ("conv", 256, 256, 3, 1, 128),
    "l5": ("conv", 512, 512, 3, 4, 32),
    "up1conv": ("conv", 256, 256, 3, 1, 64),
    "up2T": ("convT", 320, 256, 3, 1, 64),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default="up2conv,l5,up1conv,up2T")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--pfb", type=int, default=-1, help="zp_conv_tuning key 21 (next-step pixel fragments before the barrier)")
    a = ap.parse_args()
    from zebrapose_amd import _lib as L
    from zebrapose_amd.engine import Engine, Unit, Act
    from zebrapose_amd.model import layers as LY
    assert L.LIB_PATH.endswith("libzp_stamp.so"), L.LIB_PATH
    L.lib.zp_stamp_read.restype = C.c_int
    L.lib.zp_stamp_read.argtypes = [C.c_void_p, C.c_longlong]
    dev = torch.device("cuda", 0)
    L.lib.zp_conv_tuning(21, a.pfb)
    print(f"key 21 = {a.pfb}")
    print("| layer | kernel waves | K steps | cycles per K step | first fragments | MFMA blocks | DMA wait | barrier |")
    print("|---|---|---|---|---|---|---|---|")
    for name in a.layers.split(","):
        kind, cin, cout, k, d, hw = LAYERS[name]
        if kind == "conv":
            conv = LY.Conv2d(cin, cout, k, 1, d * (k // 2), d, bias=False).to(dev)
        else:
            conv = LY.ConvTranspose2d(cin, cout, 3, 2, 1, output_padding=1, bias=False).to(dev)
        unit = Unit(conv, LY.BatchNorm2d(cout).to(dev).eval(), relu=True)
        eng = Engine(torch.nn.Module(), torch.float32, split="h2")
        xs = eng._empty((a.batch, hw, hw, cin), dev)
        xs._base.copy_(torch.randn(xs._base.shape, device=dev).clamp(min=0).to(xs.dtype))
        OH, OW = unit.out_hw(hw, hw)
        y = Act(eng._empty((a.batch, OH, OW, cout), dev))
        eng.stage_log = []
        for _ in range(3):
            eng.unit_fwd(unit, Act(xs), y, None)
        torch.cuda.synchronize()
        kname = eng.stage_log[-1][1]
        M = a.batch * OH * OW if kind == "conv" else a.batch * hw * hw * 4
        waves = (M // 256) * (cout // 256) * 8
        buf = np.zeros(waves * 8, dtype=np.uint64)
        assert L.lib.zp_stamp_read(buf.ctypes.data, buf.size) == 0
        w = buf.reshape(waves, 8).astype(np.float64)
        live = w[:, 4] > 0
        w = w[live]
        seg, tot, nk = w[:, :4], w[:, 4], w[:, 5]
        frac = seg.sum(0) / tot.sum()
        print(f"| {name} | {int(live.sum())} ({kname}) | {np.mean(nk):.1f} | {tot.sum() / nk.sum():.0f} | "
              + " | ".join(f"{100 * f:.1f}%" for f in frac) + " |", flush=True)


if __name__ == "__main__":
    main()
