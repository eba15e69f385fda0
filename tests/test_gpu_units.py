"""Unit-level parity of the libzp conv / BN / pooling kernels against a plain PyTorch fp32 CPU
reference of the same op (conv or transposed conv + train-mode BatchNorm + residual + ReLU,
forward and backward), for every geometry the network uses."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

GEOMS = [
    # kind, cin, cout, k, s, p, d, bias, H
    ("conv", 64, 64, 3, 1, 1, 1, False, 16),
    ("conv", 64, 128, 3, 2, 1, 1, False, 16),
    ("conv", 64, 128, 1, 2, 0, 1, False, 16),
    ("conv", 128, 256, 3, 1, 2, 2, False, 12),
    ("conv", 256, 256, 3, 1, 4, 4, False, 12),
    ("conv", 512, 256, 3, 1, 6, 6, True, 8),
    ("conv", 512, 256, 3, 1, 18, 18, True, 8),
    ("conv", 1280, 256, 1, 1, 0, 1, True, 8),
    # ASPP at its real 32 x 32 size: 8-row tiles inside one image, so k_conv trims the tap rows
    # that only ever read padding (dilation 12: first / last tile; dilation 18: every tile)
    ("conv", 512, 256, 3, 1, 12, 12, True, 32),
    ("conv", 512, 256, 3, 1, 18, 18, True, 32),
    ("convT", 256, 256, 3, 2, 1, 1, False, 8),
    ("convT", 320, 256, 3, 2, 1, 1, False, 8),
    # full-width tiles (W 32 / 64 / 128): the bf16 activation-strip kernel (k_conv_strip)
    ("conv", 128, 128, 3, 1, 1, 1, False, 32),
    ("conv", 64, 64, 3, 1, 1, 1, False, 64),
    ("conv", 256, 256, 3, 1, 2, 2, False, 32),
    ("conv", 512, 512, 3, 1, 4, 4, False, 32),
    ("conv", 256, 256, 3, 1, 1, 1, False, 64),
    ("conv", 256, 256, 3, 1, 1, 1, False, 128),
]


def _mk(kind, cin, cout, k, s, p, d, bias):
    from zebrapose_amd.model import layers as LY
    if kind == "conv":
        conv = LY.Conv2d(cin, cout, k, s, p, d, bias=bias)
    else:
        conv = LY.ConvTranspose2d(cin, cout, k, s, p, output_padding=1, bias=False)
    bn = LY.BatchNorm2d(cout)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_(0, 0.1)
        bn.running_mean.normal_(0, 0.1)
        bn.running_var.uniform_(0.5, 1.5)
    return conv, bn


def _ref_unit(kind, conv, bn, x, res, relu, train, s, p, d):
    w = conv.weight.detach().clone().requires_grad_(True)
    b = conv.bias.detach().clone().requires_grad_(True) if conv.bias is not None else None
    g = bn.weight.detach().clone().requires_grad_(True)
    be = bn.bias.detach().clone().requires_grad_(True)
    rm, rv = bn.running_mean.detach().clone(), bn.running_var.detach().clone()
    xx = x.clone().requires_grad_(True)
    if kind == "conv":
        y = F.conv2d(xx, w, b, s, p, d)
    else:
        y = F.conv_transpose2d(xx, w, None, 2, 1, 1)
    y = F.batch_norm(y, rm, rv, g, be, training=train, momentum=0.1, eps=1e-5)
    if res is not None:
        y = y + res
    if relu:
        y = F.relu(y)
    return y, (xx, w, b, g, be), (rm, rv)


@pytest.fixture(params=["tc-auto", "tc256"])
def tile_mode(request):
    """'tc256' forces the 256-channel conv tile (normally only for launches of >= 512 workgroups)
    onto these small cases so that its code path is checked too."""
    from zebrapose_amd import _lib as L
    old = L.lib.zp_conv_tuning(0, 0 if request.param == "tc256" else 512)
    yield request.param
    L.lib.zp_conv_tuning(0, old)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("geom", GEOMS, ids=[f"{g[0]}{g[1]}-{g[2]}k{g[3]}s{g[4]}d{g[6]}" for g in GEOMS])
@pytest.mark.parametrize("train", [False, True])
def test_unit(gpu, geom, prec, train, tile_mode):
    from zebrapose_amd.engine import Engine, Unit, Act, Tape
    kind, cin, cout, k, s, p, d, bias, H = geom
    torch.manual_seed(0)
    B = 2 if H <= 32 else 1
    conv, bn = _mk(kind, cin, cout, k, s, p, d, bias)
    x = torch.randn(B, cin, H, H)
    unit = Unit(conv, bn, relu=True)
    OH, OW = unit.out_hw(H, H)
    use_res = (kind == "conv" and s == 1 and cin == cout)
    res = torch.randn(B, cout, OH, OW) if use_res else None
    y_ref, leaves, (rm_ref, rv_ref) = _ref_unit(kind, conv, bn, x, res, True, train, s, p, d)
    gout = torch.randn_like(y_ref)
    if train:
        y_ref.backward(gout)

    dt = torch.float32 if prec == "fp32" else torch.bfloat16
    convg, bng = conv.to(gpu), bn.to(gpu)
    eng = Engine(torch.nn.Module(), dt)
    xa = Act(x.permute(0, 2, 3, 1).contiguous().to(gpu, dt))
    ra = Act(res.permute(0, 2, 3, 1).contiguous().to(gpu, dt)) if res is not None else None
    oa = Act(torch.empty(B, OH, OW, cout, device=gpu, dtype=dt))
    tape = Tape() if train else None
    if not train:
        convg.eval(), bng.eval()
    eng.unit_fwd(unit, xa, oa, tape, res=ra)
    y = oa.buf.float().permute(0, 3, 1, 2).cpu()
    tol = 2e-4 if prec == "fp32" else 3e-2
    scale = y_ref.abs().max().item()
    err = (y - y_ref.detach()).abs().max().item()
    assert err <= tol * max(1.0, scale), f"forward max|d| {err} (scale {scale})"
    if not train:
        return
    torch.cuda.synchronize()
    assert torch.allclose(bng.running_mean.cpu(), rm_ref, atol=1e-4 if prec == "fp32" else 1e-2)
    assert torch.allclose(bng.running_var.cpu(), rv_ref, rtol=1e-3 if prec == "fp32" else 3e-2)
    gmap = {oa.buf.data_ptr(): gout.permute(0, 2, 3, 1).contiguous().to(gpu, dt)}
    grads = {}
    eng.unit_bwd(tape.recs[0], gmap, grads)
    xx, w, b, g, be = leaves
    checks = [("dW", grads[convg.weight], w.grad), ("dgamma", grads[bng.weight], g.grad),
              ("dbeta", grads[bng.bias], be.grad)]
    gx = gmap[xa.buf.data_ptr()].float().permute(0, 3, 1, 2).cpu()
    checks.append(("dx", gx, xx.grad))
    if ra is not None:
        gr = gmap[ra.buf.data_ptr()].float().permute(0, 3, 1, 2).cpu()
        checks.append(("dres", gr, gout * (y_ref.detach() > 0)))
    # fp32: elementwise (max |d| / max |ref|); bf16: relative L2 -- a bf16 activation that lands on
    # the other side of 0 flips a ReLU gate, so bf16 gradients are compared in norm, not per element.
    errs = []
    for name, got, want in checks:
        got = got.float().cpu()
        if prec == "fp32":
            # elementwise, except that a ReLU gate whose input sits within the forward's f32
            # reassociation error of 0 may flip (seen on the 4k / 16k-pixel geometries), and
            # dgamma = sum(g * xhat) over 16k pixels cancels heavily in f32 on both sides: then
            # the gradient must still agree in norm to 3e-3
            sc = want.abs().max().item()
            e = (got - want).abs().max().item()
            rel = ((got - want).norm() / max(want.norm().item(), 1e-12)).item()
            if e > 1e-3 * max(sc, 1e-6) and rel > 3e-3:
                errs.append(f"{name}: max|d| {e:.4g} vs scale {sc:.4g}, rel L2 {rel:.3g}")
        else:
            rel = ((got - want).norm() / max(want.norm().item(), 1e-12)).item()
            if rel > 0.05:
                errs.append(f"{name}: rel L2 {rel:.4g}")
    assert not errs, "; ".join(errs)


@pytest.mark.parametrize("geom", GEOMS, ids=[f"{g[0]}{g[1]}-{g[2]}k{g[3]}s{g[4]}d{g[6]}" for g in GEOMS])
def test_unit_fp16_eval(gpu, geom, tile_mode):
    """fp16 (inference-only dtype, configs[4]): eval-mode conv + folded BN + residual + ReLU, fp16
    NHWC in / out, v_mfma_f32_16x16x32_f16 -- against the fp32 CPU reference on the same
    fp16-representable inputs; 11-bit mantissa -> 4e-3 of the output scale."""
    from zebrapose_amd.engine import Engine, Unit, Act
    kind, cin, cout, k, s, p, d, bias, H = geom
    torch.manual_seed(0)
    B = 2 if H <= 32 else 1
    conv, bn = _mk(kind, cin, cout, k, s, p, d, bias)
    x = torch.randn(B, cin, H, H).half().float()
    unit = Unit(conv, bn, relu=True)
    OH, OW = unit.out_hw(H, H)
    use_res = (kind == "conv" and s == 1 and cin == cout)
    res = torch.randn(B, cout, OH, OW).half().float() if use_res else None
    y_ref, _, _ = _ref_unit(kind, conv, bn, x, res, True, False, s, p, d)
    convg, bng = conv.to(gpu).eval(), bn.to(gpu).eval()
    eng = Engine(torch.nn.Module(), torch.float16)
    xa = Act(x.permute(0, 2, 3, 1).contiguous().to(gpu, torch.float16))
    ra = Act(res.permute(0, 2, 3, 1).contiguous().to(gpu, torch.float16)) if res is not None else None
    oa = Act(torch.empty(B, OH, OW, cout, device=gpu, dtype=torch.float16))
    eng.unit_fwd(unit, xa, oa, None, res=ra)
    y = oa.buf.float().permute(0, 3, 1, 2).cpu()
    scale = y_ref.abs().max().item()
    err = (y - y_ref.detach()).abs().max().item()
    assert err <= 4e-3 * max(1.0, scale), f"forward max|d| {err} (scale {scale})"


# configs[4]'s ResNet50-OS8 + ASPP_50 widths (reference model/resnet.py:206-227: torchvision's
# Bottleneck layer1 / layer2 at 64 x 64 / 32 x 32, then BasicBlocks 512 -> 1024 at dilation 2 and
# 1024 -> 2048 at dilation 4; model/aspp.py:117-225: 2048 -> 256 branches, up2's ConvT over the
# [up1 | x_64] concat of 256 + 256 channels), each at the 32 x 32 / 64 x 64 grid it runs on
R50_GEOMS = [
    ("conv", 64, 64, 1, 1, 0, 1, False, 64),      # layer1 Bottleneck conv1 (1x1 reduce)
    ("conv", 64, 256, 1, 1, 0, 1, False, 64),     # conv3 (1x1 expand) / downsample
    ("conv", 256, 64, 1, 1, 0, 1, False, 64),     # the next blocks' conv1
    ("conv", 256, 128, 1, 1, 0, 1, False, 64),    # layer2 block 0 conv1
    ("conv", 128, 128, 3, 2, 1, 1, False, 64),    # its strided 3x3 (torchvision v1.5: stride on the 3x3)
    ("conv", 256, 512, 1, 2, 0, 1, False, 64),    # its strided downsample
    ("conv", 128, 512, 1, 1, 0, 1, False, 32),    # layer2 conv3
    ("conv", 512, 1024, 3, 1, 2, 2, False, 32),   # layer4 block 0 conv1 (BasicBlock, dilation 2)
    ("conv", 512, 1024, 1, 1, 0, 1, False, 32),   # its downsample
    ("conv", 1024, 1024, 3, 1, 2, 2, False, 32),  # layer4 3x3s
    ("conv", 1024, 2048, 3, 1, 4, 4, False, 32),  # layer5 block 0 conv1 (dilation 4)
    ("conv", 1024, 2048, 1, 1, 0, 1, False, 32),  # its downsample
    ("conv", 2048, 2048, 3, 1, 4, 4, False, 32),  # layer5 3x3s
    ("conv", 2048, 256, 1, 1, 0, 1, True, 32),    # ASPP_50 conv_1x1_1
    ("conv", 2048, 256, 3, 1, 6, 6, True, 32),    # conv_3x3_1
    ("conv", 2048, 256, 3, 1, 12, 12, True, 32),  # conv_3x3_2
    ("conv", 2048, 256, 3, 1, 18, 18, True, 32),  # conv_3x3_3
    ("convT", 512, 256, 3, 2, 1, 1, False, 64),   # up2's ConvT over [up1 | x_64]
]


@pytest.mark.parametrize("geom", R50_GEOMS, ids=[f"{g[0]}{g[1]}-{g[2]}k{g[3]}s{g[4]}d{g[6]}h{g[8]}" for g in R50_GEOMS])
def test_unit_fp16_eval_r50(gpu, geom, tile_mode):
    """the fp16 kernels at configs[4]'s R50 widths, per op, against the fp32 CPU
    reference on fp16-representable inputs (4e-3 of the output scale, as test_unit_fp16_eval).  The
    whole R50 fp16 forward is replayed op by op from the device's own inputs in
    test_gpu_multi_object.py::test_configs4_r50_fp16_teacher_forced."""
    test_unit_fp16_eval(gpu, geom, tile_mode)


@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp16"])
def test_maxpool(gpu, prec):
    from zebrapose_amd import _lib as L
    torch.manual_seed(1)
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[prec]
    x = torch.randn(2, 64, 17, 16).to(dt).float()
    xx = x.clone().requires_grad_(True)
    y = F.max_pool2d(xx, 3, 2, 1)
    g = torch.randn_like(y).to(dt).float()
    y.backward(g)
    xd = x.permute(0, 2, 3, 1).contiguous().to(gpu, dt)
    OH, OW = y.shape[2], y.shape[3]
    yd = torch.empty(2, OH, OW, 64, device=gpu, dtype=dt)
    dc = L.dtype_code(dt)
    L.call("zp_maxpool3s2", xd.data_ptr(), 2, 17, 16, 64, 0, 64, dc, yd.data_ptr(), OH, OW, 64, 0, L.stream_ptr())
    assert torch.equal(yd.float().permute(0, 3, 1, 2).cpu(), y.detach())
    if prec == "fp16":  # inference-only dtype: the backward entry point refuses it
        with pytest.raises(RuntimeError, match="inference-only"):
            L.call("zp_maxpool3s2_bwd", xd.data_ptr(), 64, 0, yd.data_ptr(), 64, 0, 2, 17, 16, 64, OH, OW, dc,
                   xd.data_ptr(), 64, 0, 1, L.stream_ptr())
        return
    gd = g.permute(0, 2, 3, 1).contiguous().to(gpu, dt)
    dx = torch.zeros_like(xd)
    L.call("zp_maxpool3s2_bwd", xd.data_ptr(), 64, 0, gd.data_ptr(), 64, 0, 2, 17, 16, 64, OH, OW, dc, dx.data_ptr(), 64,
           0, 1, L.stream_ptr())
    got = dx.float().permute(0, 3, 1, 2).cpu()
    assert (got - xx.grad).abs().max().item() <= (1e-6 if prec == "fp32" else 2e-2)


@pytest.mark.parametrize("ih,iw", [(128, 128), (9, 14), (2, 3), (1, 1)])
def test_maxpool_bwd_channel_slices(gpu, ih, iw):
    """Backward of the stem max pool into a channel slice of a wider buffer (ld/c0 offsets) without
    accumulation, odd and tiny extents included, against torch's max_pool2d backward (bf16 values,
    so ties between equal inputs occur and the first-maximum rule is exercised)."""
    from zebrapose_amd import _lib as L
    torch.manual_seed(3)
    B, C, ld, c0 = 3, 64, 80, 8
    x = (torch.randn(B, C, ih, iw) * 4).round().to(torch.bfloat16).float()  # many exact ties
    xx = x.clone().requires_grad_(True)
    y = F.max_pool2d(xx, 3, 2, 1)
    g = torch.randn_like(y).to(torch.bfloat16).float()
    y.backward(g)
    OH, OW = y.shape[2], y.shape[3]
    xb = torch.zeros(B, ih, iw, ld, dtype=torch.bfloat16)
    xb[..., c0:c0 + C] = x.permute(0, 2, 3, 1).to(torch.bfloat16)
    gb = torch.zeros(B, OH, OW, ld, dtype=torch.bfloat16)
    gb[..., c0:c0 + C] = g.permute(0, 2, 3, 1).to(torch.bfloat16)
    xd, gd = xb.to(gpu), gb.to(gpu)
    dx = torch.full((B, ih, iw, ld), 5.0, dtype=torch.bfloat16, device=gpu)
    L.call("zp_maxpool3s2_bwd", xd.data_ptr(), ld, c0, gd.data_ptr(), ld, c0, B, ih, iw, C, OH, OW,
           L.dtype_code(torch.bfloat16), dx.data_ptr(), ld, c0, 0, L.stream_ptr())
    got = dx.cpu().float()
    assert torch.equal(got[..., :c0], torch.full_like(got[..., :c0], 5.0))  # outside the slice untouched
    assert torch.equal(got[..., c0 + C:], torch.full_like(got[..., c0 + C:], 5.0))
    want = xx.grad.permute(0, 2, 3, 1).to(torch.bfloat16).float()
    assert (got[..., c0:c0 + C] - want).abs().max().item() <= 2e-2


QUAD_GEOMS = [
    # the four ConvTranspose phases in one tile (k_conv_quad): up1 (W 32) and up2 (W 64) shapes, and the
    # data gradient of a 3x3 stride-2 conv (dy 32x32 / 64x64), at batch sizes the CPU reference runs
    ("convT", 256, 256, 3, 2, 1, 1, False, 32),
    ("convT", 320, 256, 3, 2, 1, 1, False, 64),
    ("conv", 64, 128, 3, 2, 1, 1, False, 64),
    ("conv", 128, 64, 3, 2, 1, 1, False, 128),
]


@pytest.fixture
def quad_any():
    """k_conv_quad normally needs >= 256 workgroups; the small cases below force it."""
    from zebrapose_amd import _lib as L
    old = L.lib.zp_conv_tuning(6, 1)
    yield
    L.lib.zp_conv_tuning(6, old)


@pytest.mark.parametrize("prec", ["bf16"])
@pytest.mark.parametrize("geom", QUAD_GEOMS, ids=[f"{g[0]}{g[1]}-{g[2]}s{g[4]}h{g[8]}" for g in QUAD_GEOMS])
@pytest.mark.parametrize("train", [False, True])
def test_unit_quad(gpu, geom, prec, train, quad_any):
    """Same checks as test_unit with the four-phase kernel forced (forward ConvT; in train mode also
    the stride-2 conv's data gradient, which accumulates into its input-gradient slice)."""
    from zebrapose_amd import _lib as L
    from zebrapose_amd.engine import Unit
    import ctypes as C
    kind, cin, cout, k, s, p, d, bias, H = geom
    # the launch under test really is k_conv_quad (variant 3)
    if kind == "convT":
        conv, bn = _mk(kind, cin, cout, k, s, p, d, bias)
        plan = Unit(conv, bn).fwd_plan(H, H)
        assert len(plan.subs) == 4 and plan.GW == H
    test_unit(gpu, geom, prec, train, "tc-auto")


@pytest.mark.parametrize("geom", QUAD_GEOMS[:2], ids=["up1", "up2"])
def test_unit_quad_fp16_eval(gpu, geom, quad_any):
    test_unit_fp16_eval(gpu, geom, "tc-auto")


def test_quad_variant_selected(gpu):
    """zp_conv2d_config reports k_conv_quad (variant 3) for the bench's up2 ConvT launch (bs 32)."""
    from zebrapose_amd import _lib as L
    from zebrapose_amd.engine import Engine, Unit, Act
    from zebrapose_amd.model import layers as LY
    import ctypes as C
    conv = LY.ConvTranspose2d(320, 256, 3, 2, 1, output_padding=1, bias=False).to(gpu)
    bn = LY.BatchNorm2d(256).to(gpu).eval()
    unit = Unit(conv, bn)
    eng = Engine(torch.nn.Module(), torch.bfloat16)
    eng.timing = []
    x = Act(torch.randn(32, 64, 64, 320, device=gpu).bfloat16())
    y = Act(torch.empty(32, 128, 128, 256, device=gpu, dtype=torch.bfloat16))
    eng.unit_fwd(unit, x, y, None)
    torch.cuda.synchronize()
    assert eng.timing[-1][4] == "k_conv_quad<bf16,W=64>", eng.timing[-1][4]
