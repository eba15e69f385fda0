#!/usr/bin/env python3
"""Times the train-mode BN backward passes (zp_bn_bwd_reduce incl. totals, zp_bn_bwd_apply) with the
ReLU mask read from the stored activation (mode 1) or recomputed from raw (mode 2), and the forward
zp_bn_apply, on activation shapes of the R34 bs=32 256x256 training step.

    python tools/bn_ab.py [--rounds 5 --iters 20]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="32x128x128x64,32x64x64x64,32x32x32x128,32x32x32x256,32x32x32x512")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import zebrapose_amd._lib as L
    dev = torch.device("cuda", 0)
    code = L.dtype_code(torch.bfloat16)
    st = L.stream_ptr()
    for spec in a.shapes.split(","):
        B, H, W, Cc = (int(v) for v in spec.split("x"))
        P = B * H * W
        raw = torch.randn(P, Cc, device=dev).bfloat16()
        gout = torch.randn(P, Cc, device=dev).bfloat16()
        gamma = torch.rand(Cc, device=dev) + 0.5
        beta = torch.randn(Cc, device=dev) * 0.5
        mean, invstd = raw.float().mean(0), torch.rsqrt(raw.float().var(0) + 1e-5)
        scale = gamma * invstd
        shift = beta - mean * scale
        save = torch.cat([mean, invstd, scale, shift]).contiguous()
        y = torch.empty_like(raw)
        parts = L.lib.zp_bn_bwd_parts(P, Cc)
        partials = torch.empty(2 * (parts + 1) * Cc, dtype=torch.float32, device=dev)
        dgamma, dbeta = torch.empty(Cc, device=dev), torch.empty(Cc, device=dev)
        dx = torch.empty_like(raw)

        def fwd():
            L.call("zp_bn_apply", raw.data_ptr(), P, Cc, scale.data_ptr(), shift.data_ptr(), None, 0, 0, 1, code,
                   y.data_ptr(), Cc, 0, st)

        def red(mode):
            L.call("zp_bn_bwd_reduce", gout.data_ptr(), Cc, 0, y.data_ptr(), Cc, 0, raw.data_ptr(), P, Cc,
                   save.data_ptr(), mode, code, partials.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(), 0, st)

        def app(mode):
            L.call("zp_bn_bwd_apply", gout.data_ptr(), Cc, 0, y.data_ptr(), Cc, 0, raw.data_ptr(), P, Cc,
                   save.data_ptr(), partials.data_ptr(), gamma.data_ptr(), mode, code, dx.data_ptr(), None, 0, 0, 0,
                   st)
        def fwd_old():
            os.environ["ZP_BN_APPLY_U"] = "0"
            fwd()
            os.environ["ZP_BN_APPLY_U"] = "1"

        def fwd_res():
            L.call("zp_bn_apply", raw.data_ptr(), P, Cc, scale.data_ptr(), shift.data_ptr(), gout.data_ptr(), Cc, 0,
                   1, code, y.data_ptr(), Cc, 0, st)
        legs = {"apply_fwd": fwd, "apply_old": fwd_old, "apply_res": fwd_res, "reduce_m1": lambda: red(1), "reduce_m2": lambda: red(2),
                "bwd_apply_m1": lambda: app(1), "bwd_apply_m2": lambda: app(2)}
        fwd()
        times = {k: [] for k in legs}
        for _ in range(a.rounds):
            for k, f in legs.items():
                f()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    f()
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) * 1e3 / a.iters)
        T = P * Cc * 2
        nread = {"apply_fwd": 2, "apply_old": 2, "apply_res": 3, "reduce_m1": 3, "reduce_m2": 2, "bwd_apply_m1": 4, "bwd_apply_m2": 3}
        print(spec, " ".join(f"{k} {np.median(v):7.1f}us ({nread[k] * T / np.median(v) / 1e3:5.0f} GB/s)"
                             for k, v in times.items()), flush=True)


if __name__ == "__main__":
    main()
