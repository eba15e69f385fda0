"""Implicit-GEMM geometry: tap lists for convolutions, transposed convolutions and their
data / weight gradients (host-side planning; no arithmetic on tensors).

A *sub-problem* is: for every grid point g = (gy, gx) and tap t, read input pixel
(gy*s + ty[t], gx*s + tx[t]) and accumulate into output pixel (gy*oys + oyo, gx*oxs + oxo)
with weight tap (ky[t], kx[t]).  (include/zp.h, zp_conv_sub)

* ``nn.Conv2d(k, stride s, pad p, dilation d)``: one sub, ty = ky*d - p.
* ``nn.ConvTranspose2d(3, stride 2, pad 1, output_padding 1)`` (model/aspp.py:62-71):
  output o = 2 i - p + k, so each output parity phase (py, px) is a stride-1 conv over
  the input with taps ky == py + p (mod 2) at offset (py + p - ky) / 2.
* data gradient of a stride-1 conv: the same conv with negated offsets and transposed weights.
* data gradient of a stride-2 conv: the ConvTranspose structure (phases) over dy.
* data gradient of ConvTranspose: a stride-2 conv over dy.
"""
from __future__ import annotations

from dataclasses import dataclass, field


@dataclass
class Sub:
    taps: list            # [(ky, kx)] weight taps
    offs: list            # [(ty, tx)] input offsets
    oys: int = 1
    oyo: int = 0
    oxs: int = 1
    oxo: int = 0


@dataclass
class Plan:
    """One zp_conv2d launch: input stride, grid and subs."""
    GH: int
    GW: int
    sy: int
    subs: list = field(default_factory=list)


def out_size(n, k, s, p, d=1):
    return (n + 2 * p - d * (k - 1) - 1) // s + 1


def conv_fwd(IH, IW, k, s, p, d=1) -> Plan:
    OH, OW = out_size(IH, k, s, p, d), out_size(IW, k, s, p, d)
    taps = [(ky, kx) for ky in range(k) for kx in range(k)]
    offs = [(ky * d - p, kx * d - p) for ky, kx in taps]
    return Plan(OH, OW, s, [Sub(taps, offs)])


def _phases(G_out_h, G_out_w, k, p, stride=2):
    """Sub-problems of a stride-2 transposed structure o = 2 i - p + k (output size G_out)."""
    subs = []
    gh = gw = None
    for py in range(stride):
        for px in range(stride):
            taps, offs = [], []
            for ky in range(k):
                if (ky - py - p) % 2:
                    continue
                for kx in range(k):
                    if (kx - px - p) % 2:
                        continue
                    taps.append((ky, kx))
                    offs.append(((py + p - ky) // 2, (px + p - kx) // 2))
            h = (G_out_h - py + 1) // 2
            w = (G_out_w - px + 1) // 2
            if gh is None:
                gh, gw = h, w
            if (h, w) != (gh, gw):
                raise ValueError("odd output sizes are not supported by the phase decomposition")
            if taps:
                subs.append(Sub(taps, offs, 2, py, 2, px))
    return gh, gw, subs


def convT_fwd(IH, IW, k=3, s=2, p=1, op=1) -> Plan:
    assert s == 2
    OH = (IH - 1) * s - 2 * p + k + op
    OW = (IW - 1) * s - 2 * p + k + op
    gh, gw, subs = _phases(OH, OW, k, p)
    return Plan(gh, gw, 1, subs)


def conv_dgrad(IH, IW, k, s, p, d=1) -> Plan:
    """Plan computing dx (IH x IW) from dy of conv_fwd(IH, IW, k, s, p, d); weights packed transposed."""
    if s == 1:
        taps = [(ky, kx) for ky in range(k) for kx in range(k)]
        offs = [(p - ky * d, p - kx * d) for ky, kx in taps]
        return Plan(IH, IW, 1, [Sub(taps, offs)])
    assert s == 2 and d == 1
    gh, gw, subs = _phases(IH, IW, k, p)
    return Plan(gh, gw, 1, subs)


def convT_dgrad(IH, IW, k=3, s=2, p=1) -> Plan:
    """Plan computing dx (IH x IW) from dy of convT_fwd: a stride-2 conv over dy, offsets ky - p."""
    taps = [(ky, kx) for ky in range(k) for kx in range(k)]
    offs = [(ky - p, kx - p) for ky, kx in taps]
    return Plan(IH, IW, s, [Sub(taps, offs)])


def ceil_to(x, m):
    return (x + m - 1) // m * m
