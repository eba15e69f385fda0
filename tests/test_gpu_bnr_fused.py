"""the BN backward reduce taken inside the reader's data-gradient epilogue (zp.h bnr_*,
Engine._bnr_fusable, default on) against the separate zp_bn_bwd_reduce (ZP_BN_BWD_FUSED=0), per conv
kernel variant that carries that epilogue.

Reference: model/resnet.py:41-51 (BasicBlock: conv1 -> BN -> ReLU read only by conv2), train_v6.py:337
(backward).  A two-unit chain A -> B is taped in train mode: unit A = conv + train-mode BN + ReLU
(mode 2: the mask recomputed from A's raw conv output; the ReLU mask is mixed -- shifted BN betas put
~30-70% of the pre-activations below zero), whose output buffer is read only by unit B (conv + BN).
The reverse pass of B, then A runs twice on the same tape and inputs: with the fused reduce and with
it off.  A's dgamma / dbeta (the reduce's sums) must agree to f32 summation order (1e-5 of the
sums' absolute mass), and everything downstream of them -- A's weight gradient and A's input
gradient (zp_bn_bwd_apply from the reduce's totals) -- within storage rounding of the dtype.

Variants: f32 k_conv (LDS merge of the wave halves); bf16 k_conv_strip2 (the paired 8-channel BPAIR
epilogue, zp_conv_tuning key 1 with flag 64); bf16 k_conv_strip (flag 64 off: one part per wave
half); bf16 k_conv for a ConvT reader (its data gradient is a stride-2 conv over the phases'
output).  Channel counts include one that is not a multiple of the 128-channel cout tile (192:
the bf16 kernels take multiples of 64 channels)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [
    # id, dtype, A (cin, cout, H), B (kind, cout, k, s, p), conv flags (None: default)
    ("f32_kconv", torch.float32, (32, 96, 16), ("conv", 64, 3, 1, 1), None),
    ("bf16_strip2", torch.bfloat16, (64, 128, 32), ("conv", 128, 3, 1, 1), None),
    ("bf16_strip2_c192", torch.bfloat16, (64, 192, 32), ("conv", 128, 3, 1, 1), None),
    ("bf16_strip_noflag64", torch.bfloat16, (64, 128, 32), ("conv", 128, 3, 1, 1), 478 - 64),
    ("bf16_convT_reader", torch.bfloat16, (64, 256, 16), ("convT", 256, 3, 2, 1), None),
]


def _mk(kind, cin, cout, k, s, p):
    from zebrapose_amd.model import layers as LY
    if kind == "conv":
        conv = LY.Conv2d(cin, cout, k, s, p, 1, bias=False)
    else:
        conv = LY.ConvTranspose2d(cin, cout, k, s, p, output_padding=1, bias=False)
    bn = LY.BatchNorm2d(cout)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_(0, 0.5)  # shifted betas: a mixed ReLU mask
    return conv, bn


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_bnr_fused_equals_separate_reduce(gpu, case):
    from zebrapose_amd import _lib as L
    from zebrapose_amd.engine import Act, Engine, Tape, Unit
    name, dt, (cin, ca, H), (kb, cb, k, s, p), flags = case
    torch.manual_seed(5)
    convA, bnA = _mk("conv", cin, ca, 3, 1, 1)
    convB, bnB = _mk(kb, ca, cb, k, s, p)
    for m in (convA, bnA, convB, bnB):
        m.to(gpu).train()
    uA, uB = Unit(convA, bnA, relu=True), Unit(convB, bnB, relu=False)
    B = 2
    x = Act(torch.randn(B, H, H, cin, device=gpu).to(dt))
    outA = Act(torch.empty(B, H, H, ca, device=gpu, dtype=dt))
    OH, OW = uB.out_hw(H, H)
    outB = Act(torch.empty(B, OH, OW, cb, device=gpu, dtype=dt))
    gout = torch.randn(B, OH, OW, cb, device=gpu).to(dt)
    old = L.lib.zp_conv_tuning(1, flags) if flags is not None else None
    try:
        eng = Engine(torch.nn.Module(), dt)
        tape = Tape()
        eng.unit_fwd(uA, x, outA, tape)
        eng.unit_fwd(uB, outA, outB, tape)
        torch.cuda.synchronize()
        # the mask really is mixed
        frac_pos = float((outA.buf.float() > 0).float().mean())
        assert 0.2 < frac_pos < 0.8, frac_pos
        res = {}
        for fused in (True, False):
            eng.bn_bwd_fused = fused
            fus = eng._bnr_fusable(tape)
            assert (outA.buf.data_ptr() in fus) == fused, (name, fused, list(fus))
            gmap = {"__bnr_prod__": fus, outB.buf.data_ptr(): gout.clone()}
            grads = {}
            eng.unit_bwd(tape.recs[1], gmap, grads)
            if fused:  # B's data-gradient launch took A's reduce: its partials wait for A's backward
                assert outA.buf.data_ptr() in gmap.get("__bnr__", {}), name
            eng.unit_bwd(tape.recs[0], gmap, grads)
            torch.cuda.synchronize()
            assert not gmap.get("__bnr__"), "a fused reduce was never consumed"
            res[fused] = {"dgamma": grads[bnA.weight].clone(), "dbeta": grads[bnA.bias].clone(),
                          "dWA": grads[convA.weight].clone(), "dx": gmap[x.buf.data_ptr()].float().clone()}
    finally:
        if old is not None:
            L.lib.zp_conv_tuning(1, old)
    a, b = res[True], res[False]
    for key in ("dgamma", "dbeta"):
        mass = float(b[key].abs().sum())
        d = float((a[key] - b[key]).abs().max())
        assert d <= 1e-5 * max(mass, 1.0), (name, key, d, mass)
    tol = 1e-5 if dt == torch.float32 else 2 ** -7
    for key in ("dWA", "dx"):
        rel = float((a[key] - b[key]).norm() / b[key].norm().clamp_min(1e-30))
        assert rel <= tol, (name, key, rel)
    print(f"{name}: mask positive {frac_pos:.2f}; dgamma max |d| {float((a['dgamma'] - b['dgamma']).abs().max()):.3g}, "
          f"dx rel {float((a['dx'] - b['dx']).norm() / b['dx'].norm()):.3g}")
