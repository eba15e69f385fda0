"""The split-fp32 engine (include/zp.h ZP_F32X3; k_conv3): fp32 values as three bf16 planes
(hi + mid + lo, exact) and every conv product formed from its six leading terms on bf16 MFMAs.

  * the split is exact: packed weights joined back equal the f32 checkpoint bit for bit;
  * every conv geometry of the network (3x3 / dilated / strided, 1x1, the four ConvTranspose
    phases, the merged-ASPP shapes, the NCHW head) in eval mode (BN fold, bias, residual, ReLU):
    the split result's error against a float64 CPU reference of the same op is no larger than the
    exact-f32-MFMA kernel's own error (2x + a 2^-24-scale floor) -- i.e. f32-accurate;
  * the pooling / broadcast kernels on split tensors match their f32 definitions exactly.
Network-level parity (the reference fixtures at 64x64 and 256x256, bs=32 teacher-forced) is in
test_gpu_parity.py / test_gpu_bench_geometry.py, parametrised over both fp32 engines."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

GEOMS = [
    # kind, cin, cout, k, s, p, d, bias, H
    ("conv", 64, 64, 3, 1, 1, 1, False, 32),
    ("conv", 64, 128, 3, 2, 1, 1, False, 32),
    ("conv", 64, 128, 1, 2, 0, 1, False, 32),
    ("conv", 128, 256, 3, 1, 2, 2, False, 16),
    ("conv", 256, 256, 3, 1, 4, 4, False, 16),
    ("conv", 512, 256, 3, 1, 12, 12, True, 32),
    ("conv", 512, 256, 3, 1, 18, 18, True, 32),
    ("conv", 1280, 256, 1, 1, 0, 1, True, 8),
    ("conv", 320, 256, 3, 1, 1, 1, False, 24),
    ("convT", 256, 256, 3, 2, 1, 1, False, 16),
    ("convT", 320, 256, 3, 2, 1, 1, False, 8),
    ("conv", 96, 48, 3, 1, 1, 1, False, 20),   # 64-channel tile, ragged Cout / pixel count
]


def _ref64(kind, conv, bn, x, res, relu, s, p, d):
    w = conv.weight.detach().double().cpu()
    b = None if conv.bias is None else conv.bias.detach().double().cpu()
    xx = x.double()
    y = F.conv2d(xx, w, b, s, p, d) if kind == "conv" else F.conv_transpose2d(xx, w, None, 2, 1, 1)
    if bn is not None:
        g, be, rm, rv = (t.detach().double().cpu() for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var))
        y = (y - rm.view(1, -1, 1, 1)) / torch.sqrt(rv.view(1, -1, 1, 1) + 1e-5) * g.view(1, -1, 1, 1) + be.view(1, -1, 1, 1)
    if res is not None:
        y = y + res.double()
    return F.relu(y) if relu else y


def _split_act(t, dev, form="x3"):
    """f32 NHWC host tensor -> plane-0 view of its split on the device: x3 = the exact 3-plane bf16
    split; h2 = fp16 hi + fp16 (residual * 2^11) (22 significant bits)."""
    if form == "h2":
        h = t.half()
        lo = ((t - h.float()) * 2048.0).half()
        planes = torch.stack([h, lo]).to(dev)
        j = planes[0].float() + planes[1].float() / 2048.0
        # 22 significant bits down to fp16's normal range; below it (|t| < 2^-14) an absolute 2^-36
        assert ((j - t.to(dev)).abs() <= 2.0 ** -22 * t.to(dev).abs() + 2.0 ** -36).all()
        return planes[0]
    h = t.to(torch.bfloat16)
    r = t - h.float()
    m = r.to(torch.bfloat16)
    lo = (r - m.float()).to(torch.bfloat16)
    planes = torch.stack([h, m, lo]).to(dev)
    assert torch.equal((planes[0].float() + planes[1].float()) + planes[2].float(), t.to(dev))
    return planes[0]


FORMS = ["x3", "h2"]
# split error vs float64 <= MULT x the exact-f32 kernel's + FLOOR x scale: x3 is f32-accurate (2x);
# h2 stores 22 significant bits (its input / output rounding alone is 2^-23 relative)
BOUND = {"x3": (2.0, 2.0 ** -24), "h2": (4.0, 2.0 ** -21)}


def test_split_weight_pack_is_exact(gpu):
    from zebrapose_amd import _lib as L
    from zebrapose_amd.engine import _i32arr
    g = torch.Generator().manual_seed(3)
    w = torch.randn(96, 40, 3, 3, generator=g) * torch.exp(torch.randn(96, 40, 3, 3, generator=g) * 4)
    w[0, 0] = 0.0
    w[1, 1] = -1e-30
    w = w.to(gpu)
    rows, kp = 128, 9 * 64
    out = torch.empty((3, rows, kp), dtype=torch.bfloat16, device=gpu)
    ky = [t // 3 for t in range(9)]
    kx = [t % 3 for t in range(9)]
    L.call("zp_pack_weight", w.data_ptr(), 96, 40, 3, 3, 0, 9, _i32arr(ky), _i32arr(kx), 64, L.ZP_F32X3,
           out.data_ptr(), rows, kp, L.stream_ptr())
    ref = torch.empty((rows, kp), dtype=torch.float32, device=gpu)
    L.call("zp_pack_weight", w.data_ptr(), 96, 40, 3, 3, 0, 9, _i32arr(ky), _i32arr(kx), 64, L.ZP_F32,
           ref.data_ptr(), rows, kp, L.stream_ptr())
    joined = (out[0].float() + out[1].float()) + out[2].float()
    torch.cuda.synchronize()
    assert torch.equal(joined, ref)
    # each plane is the round-to-nearest bf16 of what the planes above it leave
    assert torch.equal(out[0], ref.to(torch.bfloat16))


# 3x3 stride-1 geometries the strip kernel k_conv3s takes (W 32 / 64 / 128, 256-pixel whole-row
# tiles; dilation up to a 288-row strip), run under strip modes 0 (k_conv3), 1 (64-channel tiles
# on k_conv3s<2>) and 2 (128-channel tiles on k_conv3s<4> too)
STRIP_GEOMS = [
    ("conv", 64, 64, 3, 1, 1, 1, False, 64),
    ("conv", 64, 64, 3, 1, 2, 2, False, 32),
    ("conv", 128, 128, 3, 1, 1, 1, False, 64),
    ("conv", 256, 256, 3, 1, 1, 1, False, 128),
    ("conv", 128, 256, 3, 1, 2, 2, False, 64),
]


def _gid(g):
    return f"{g[0]}{g[1]}-{g[2]}k{g[3]}s{g[4]}d{g[6]}h{g[8]}"


def test_h2_weight_pack(gpu):
    """ZP_F32H2 packing: fp16 hi = RNE(w), lo = RNE((w - hi) * 2^11); joined within 2^-22 relative
    (fp16's normal range), the hi plane equal to the fp16 cast of the f32 pack."""
    from zebrapose_amd import _lib as L
    from zebrapose_amd.engine import _i32arr
    g = torch.Generator().manual_seed(3)
    w = (torch.randn(96, 40, 3, 3, generator=g) * 0.05).to(gpu)
    w[0, 0] = 0.0
    rows, kp = 128, 9 * 64
    out = torch.empty((2, rows, kp), dtype=torch.float16, device=gpu)
    ky = [t // 3 for t in range(9)]
    kx = [t % 3 for t in range(9)]
    L.call("zp_pack_weight", w.data_ptr(), 96, 40, 3, 3, 0, 9, _i32arr(ky), _i32arr(kx), 64, L.ZP_F32H2,
           out.data_ptr(), rows, kp, L.stream_ptr())
    ref = torch.empty((rows, kp), dtype=torch.float32, device=gpu)
    L.call("zp_pack_weight", w.data_ptr(), 96, 40, 3, 3, 0, 9, _i32arr(ky), _i32arr(kx), 64, L.ZP_F32,
           ref.data_ptr(), rows, kp, L.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(out[0], ref.half())
    assert torch.equal(out[1], ((ref - out[0].float()) * 2048.0).half())
    joined = out[0].float() + out[1].float() / 2048.0
    assert ((joined - ref).abs() <= 2.0 ** -22 * ref.abs() + 2.0 ** -36).all()


@pytest.mark.parametrize("splitk", [1, 0], ids=["splitk", "no_splitk"])
@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("min_blocks", [0, 256], ids=["tile_by_cout", "small_grid_64"])
@pytest.mark.parametrize("geom", GEOMS, ids=[_gid(g) for g in GEOMS])
def test_split_conv_is_f32_accurate(gpu, geom, min_blocks, form, splitk):
    """min_blocks = zp_conv_tuning key 8: 0 keeps the 128-channel tiles at these small batches,
    256 (the default) moves launches of < 256 workgroups to 64-channel tiles; splitk = key 9 (these
    B = 2 grids are small: with it on, the one-sub launches run split along K)."""
    from zebrapose_amd import _lib as L
    old = L.lib.zp_conv_tuning(8, min_blocks)
    old_sk = L.lib.zp_conv_tuning(9, splitk)
    try:
        _check_geom(gpu, geom, form)
    finally:
        L.lib.zp_conv_tuning(8, old)
        L.lib.zp_conv_tuning(9, old_sk)


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("geom", STRIP_GEOMS, ids=[_gid(g) for g in STRIP_GEOMS])
def test_split_strip_kernel(gpu, geom, mode, form):
    from zebrapose_amd import _lib as L
    old = L.lib.zp_conv_tuning(7, mode)
    old_mb = L.lib.zp_conv_tuning(8, 0)  # the cout tile by Cout alone
    old_sk = L.lib.zp_conv_tuning(9, 0)  # no split-K (it takes these small grids before the strip kernel)
    old_wsk = L.lib.zp_conv_tuning(12, 0)  # nor the wide tile's (32 + tiles of 256 channels at bs 2)
    try:
        variant = _check_geom(gpu, geom, form)
    finally:
        L.lib.zp_conv_tuning(7, old)
        L.lib.zp_conv_tuning(8, old_mb)
        L.lib.zp_conv_tuning(9, old_sk)
        L.lib.zp_conv_tuning(12, old_wsk)
    cout, H = geom[2], geom[8]
    tc = 128 if cout > 64 else 64
    strip = (mode == 2 or (mode == 1 and tc == 64)) and H * H >= 256
    assert variant == (5 if strip else 4), (variant, mode)


def _check_geom(gpu, geom, form="x3", B=2, names_out=None):
    """Split vs exact-f32-MFMA error against float64; returns the launch variant (zp_conv2d_config)."""
    from zebrapose_amd import _lib as L
    from zebrapose_amd.engine import Engine, Unit, Act, joined
    from zebrapose_amd.model import layers as LY
    kind, cin, cout, k, s, p, d, bias, H = geom
    torch.manual_seed(0)
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
    conv, bn = conv.to(gpu).eval(), bn.to(gpu).eval()
    unit = Unit(conv, bn, relu=True)
    OH, OW = unit.out_hw(H, H)
    x = torch.randn(B, cin, H, H)
    use_res = kind == "conv" and s == 1
    res = torch.randn(B, cout, OH, OW) if use_res else None
    ref = _ref64(kind, conv, bn, x, res, True, s, p, d)
    xh = x.permute(0, 2, 3, 1).contiguous()
    rh = None if res is None else res.permute(0, 2, 3, 1).contiguous()
    out = {}
    for mode in ("x3", "f32"):
        if mode == "x3":
            eng = Engine(torch.nn.Module(), torch.float32, split=form)
            xa = Act(_split_act(xh, gpu, form))
            ra = None if rh is None else Act(_split_act(rh, gpu, form))
            oa = Act(eng._empty((B, OH, OW, cout), gpu))
        else:
            eng = Engine(torch.nn.Module(), torch.float32)
            xa = Act(xh.to(gpu))
            ra = None if rh is None else Act(rh.to(gpu))
            oa = Act(torch.empty(B, OH, OW, cout, device=gpu))
        eng.stage_log = []  # (stage, kernel label, ...) per launch
        eng.unit_fwd(unit, xa, oa, None, res=ra)
        torch.cuda.synchronize()
        out[mode] = joined(oa.buf).permute(0, 3, 1, 2).double().cpu()
        if mode == "x3":
            names = [r[1] for r in eng.stage_log]
            variant = 5 if all(n.startswith("k_conv3s<") for n in names) else 4
            if names_out is not None:
                names_out.extend(names)
    scale = ref.abs().max().item()
    e3 = (out["x3"] - ref).abs().max().item()
    e32 = (out["f32"] - ref).abs().max().item()
    r3 = (out["x3"] - ref).pow(2).mean().sqrt().item()
    r32 = (out["f32"] - ref).pow(2).mean().sqrt().item()
    print(f"{geom} {form}: max|d| split {e3:.3g} f32-MFMA {e32:.3g}; rms split {r3:.3g} f32-MFMA {r32:.3g} "
          f"(scale {scale:.3g})")
    mult, floor = BOUND[form]
    assert e3 <= mult * e32 + floor * scale, (e3, e32, scale)
    return variant


@pytest.mark.parametrize("form", FORMS)
def test_split_head_nchw(gpu, form):
    """The head conv (1x1, 320 -> 17, bias, no BN) on the 32-channel tile writing f32 NCHW mask / code."""
    from zebrapose_amd.engine import Engine, Unit, Act
    from zebrapose_amd.model import layers as LY
    torch.manual_seed(1)
    B, H = 2, 24
    conv = LY.Conv2d(320, 17, 1, 1, 0, 1, bias=True).to(gpu).eval()
    unit = Unit(conv, None, relu=False)
    x = torch.randn(B, 320, H, H)
    ref = _ref64("conv", conv, None, x, None, False, 1, 0, 1)
    err = {}
    for mode in ("x3", "f32"):
        eng = Engine(torch.nn.Module(), torch.float32, split=form if mode == "x3" else None)
        xh = x.permute(0, 2, 3, 1).contiguous()
        xa = Act(_split_act(xh, gpu, form) if mode == "x3" else xh.to(gpu))
        mask = torch.empty(B, 1, H, H, device=gpu)
        code = torch.empty(B, 16, H, H, device=gpu)
        eng.head_fwd(unit, xa, mask, code, None)
        torch.cuda.synchronize()
        err[mode] = (torch.cat([mask, code], 1).double().cpu() - ref).abs().max().item()
    scale = ref.abs().max().item()
    print(f"head {form}: max|d| split {err['x3']:.3g} f32-MFMA {err['f32']:.3g} (scale {scale:.3g})")
    mult, floor = BOUND[form]
    assert err["x3"] <= mult * err["f32"] + floor * scale, err


@pytest.mark.parametrize("form", FORMS)
def test_split_pools_and_broadcast(gpu, form):
    """Max pool, global average pool and broadcast on split tensors: exactly their f32 definitions
    on the joined values (the pooled values re-split: x3 exactly; h2 the split of the f32 result)."""
    from zebrapose_amd import _lib as L
    from zebrapose_amd.engine import joined, SPLIT
    torch.manual_seed(2)
    B, H, C = 2, 17, 64
    dt = L.ZP_F32X3 if form == "x3" else L.ZP_F32H2
    npl, tdt, _ = SPLIT[dt]
    x = torch.randn(B, H, H, 80)
    xa = _split_act(x, gpu, form)
    xj = joined(xa).cpu()  # the values the kernels see (h2: 22-bit)
    st = L.stream_ptr()
    OH = (H - 1) // 2 + 1
    y = torch.empty((npl, B, OH, OH, C), dtype=tdt, device=gpu)[0]
    L.call("zp_maxpool3s2", xa.data_ptr(), B, H, H, 80, 16, C, dt, y.data_ptr(), OH, OH, C, 0, st)
    ref = F.max_pool2d(xj[..., 16:16 + C].permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    torch.cuda.synchronize()
    assert torch.equal(joined(y).cpu(), ref)
    pool = torch.empty((npl, B, 1, 1, 80), dtype=tdt, device=gpu)[0]
    L.call("zp_global_avgpool", xa.data_ptr(), B, H, H, 80, 0, 80, dt, pool.data_ptr(), st)
    pref = xj.double().mean((1, 2)).float().view(B, 1, 1, 80)
    torch.cuda.synchronize()
    if form == "x3":
        assert torch.equal(joined(pool).cpu(), pref)
    else:  # the f32 mean stored in 22 bits
        assert ((joined(pool).cpu() - pref).abs() <= 2.0 ** -22 * pref.abs() + 2.0 ** -36).all()
    out = torch.zeros((npl, B, 5, 5, 96), dtype=tdt, device=gpu)[0]
    L.call("zp_broadcast_hw", pool.data_ptr(), B, 80, dt, out.data_ptr(), 5, 5, 96, 8, st)
    torch.cuda.synchronize()
    assert torch.equal(joined(out)[..., 8:88].cpu(), joined(pool).cpu().expand(B, 5, 5, 80))


@pytest.mark.parametrize("cin", [256, 1280])
def test_split_accumulation_numerics(gpu, cin):
    """Diagnostic: with bf16-representable inputs and weights (mid = lo = 0) the split kernel's
    result is the plain bf16-MFMA accumulation of the exact products, the f32 kernel's the f32-MFMA
    (fmaf chain) accumulation of the same products: their errors against float64 compare the two
    MFMA accumulators directly (printed; the split bound is the f32 one x 2)."""
    from zebrapose_amd.engine import Engine, Unit, Act, joined
    from zebrapose_amd.model import layers as LY
    torch.manual_seed(4)
    B, H, cout = 2, 16, 256
    conv = LY.Conv2d(cin, cout, 1, 1, 0, 1, bias=False)
    with torch.no_grad():
        conv.weight.copy_(conv.weight.to(torch.bfloat16).float())
    conv = conv.to(gpu).eval()
    unit = Unit(conv, None, relu=False)
    x = torch.randn(B, cin, H, H).to(torch.bfloat16).float()
    ref = F.conv2d(x.double(), conv.weight.detach().double().cpu())
    xh = x.permute(0, 2, 3, 1).contiguous()
    res = {}
    for mode in ("x3", "f32"):
        eng = Engine(torch.nn.Module(), torch.float32, x3=mode == "x3")
        xa = Act(_split_act(xh, gpu) if mode == "x3" else xh.to(gpu))
        oa = Act(eng._empty((B, H, H, cout), gpu) if mode == "x3" else torch.empty(B, H, H, cout, device=gpu))
        eng.unit_fwd(unit, xa, oa, None)
        torch.cuda.synchronize()
        d = joined(oa.buf).permute(0, 3, 1, 2).double().cpu() - ref
        res[mode] = (d.abs().max().item(), d.pow(2).mean().sqrt().item(), d.mean().item())
    print(f"K={cin}: bf16-MFMA acc max/rms/mean {res['x3']}, f32-MFMA {res['f32']} (scale {ref.abs().max().item():.3g})")
    assert res["x3"][0] <= 2.0 * res["f32"][0] + 1e-30


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("geom", [("conv", 512, 512, 3, 1, 4, 4, False, 32), ("conv", 256, 256, 3, 1, 2, 2, False, 32),
                                  ("conv", 1280, 256, 1, 1, 0, 1, True, 8), ("convT", 320, 256, 3, 2, 1, 1, False, 16)],
                         ids=["l5_d4", "l4_d2", "aspp_proj", "convT_4phases"])
def test_split_k_small_batch(gpu, geom, form):
    """bs = 1: the small-grid launches are cut along K (zp_conv2d_split_ws > 0, zp_conv_tuning key 9)
    and finished by k_splitk_epi; the result is as accurate as the unsplit kernel's (both against
    float64) and differs from it (the split path ran)."""
    from zebrapose_amd import _lib as L
    from zebrapose_amd.engine import Engine, Unit, Act, joined
    from zebrapose_amd.model import layers as LY
    kind, cin, cout, k, s, p, d, bias, H = geom
    torch.manual_seed(6)
    if kind == "conv":
        conv = LY.Conv2d(cin, cout, k, s, p, d, bias=bias)
    else:  # the four sub-pixel phases: a multi-sub launch split along K per phase
        conv = LY.ConvTranspose2d(cin, cout, k, s, p, output_padding=1, bias=False)
    bn = LY.BatchNorm2d(cout)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_(0, 0.1)
        bn.running_mean.normal_(0, 0.1)
        bn.running_var.uniform_(0.5, 1.5)
    conv, bn = conv.to(gpu).eval(), bn.to(gpu).eval()
    unit = Unit(conv, bn, relu=True)
    OH, OW = unit.out_hw(H, H)
    x = torch.randn(1, cin, H, H)
    res = torch.randn(1, cout, OH, OW) if kind == "conv" else None
    ref = _ref64(kind, conv, bn, x, res, True, s, p, d)
    xh = x.permute(0, 2, 3, 1).contiguous()
    eng = Engine(torch.nn.Module(), torch.float32, split=form)
    xa = Act(_split_act(xh, gpu, form))
    ra = None if res is None else Act(_split_act(res.permute(0, 2, 3, 1).contiguous(), gpu, form))
    out = {}
    for mode in (1, 0):
        old = L.lib.zp_conv_tuning(9, mode)
        try:
            oa = Act(eng._empty((1, OH, OW, cout), gpu))
            eng.unit_fwd(unit, xa, oa, None, res=ra)
            torch.cuda.synchronize()
        finally:
            L.lib.zp_conv_tuning(9, old)
        out[mode] = joined(oa.buf).permute(0, 3, 1, 2).double().cpu()
    e1, e0 = (out[1] - ref).abs().max().item(), (out[0] - ref).abs().max().item()
    print(f"{geom} {form} bs=1: split-K max|d| {e1:.3g}, unsplit {e0:.3g}")
    assert not torch.equal(out[1], out[0])
    assert e1 <= 2.0 * e0 + 2.0 ** -22 * ref.abs().max().item(), (e1, e0)


def test_wide_split_k_strip_small_batch(gpu):
    """bs = 1, up2's 3x3 256 -> 256 at 128 x 128 (64 tiles of 256 x 256): the wide tile runs split
    along K (zp_conv_tuning key 12, 4 slices of whole (chunk, tap row) groups: its strip staging
    needs group-aligned slices) and k_splitk_epi finishes it.  Against float64, as accurate as the
    launch without the wide split-K (k_conv3's tiles), and not bit-identical to it (the wide path
    ran); the stage log names k_conv3w."""
    from zebrapose_amd import _lib as L
    from zebrapose_amd.engine import Engine, Unit, Act, joined
    from zebrapose_amd.model import layers as LY
    torch.manual_seed(7)
    conv = LY.Conv2d(256, 256, 3, 1, 1, 1, bias=False)
    bn = LY.BatchNorm2d(256)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_(0, 0.1)
        bn.running_mean.normal_(0, 0.1)
        bn.running_var.uniform_(0.5, 1.5)
    conv, bn = conv.to(gpu).eval(), bn.to(gpu).eval()
    unit = Unit(conv, bn, relu=True)
    H = 128
    x = torch.randn(1, 256, H, H)
    res = torch.randn(1, 256, H, H)
    ref = _ref64("conv", conv, bn, x, res, True, 1, 1, 1)
    eng = Engine(torch.nn.Module(), torch.float32, split="h2")
    xa = Act(_split_act(x.permute(0, 2, 3, 1).contiguous(), gpu, "h2"))
    ra = Act(_split_act(res.permute(0, 2, 3, 1).contiguous(), gpu, "h2"))
    out, names = {}, {}
    for mode in (1, 0):
        old = L.lib.zp_conv_tuning(12, mode)
        try:
            oa = Act(eng._empty((1, H, H, 256), gpu))
            eng.stage_log = []
            eng.unit_fwd(unit, xa, oa, None, res=ra)
            torch.cuda.synchronize()
            names[mode] = [r[1] for r in eng.stage_log]
        finally:
            L.lib.zp_conv_tuning(12, old)
        out[mode] = joined(oa.buf).permute(0, 3, 1, 2).double().cpu()
    e1, e0 = (out[1] - ref).abs().max().item(), (out[0] - ref).abs().max().item()
    print(f"wide split-K bs=1: max|d| {e1:.3g} ({names[1]}), without {e0:.3g} ({names[0]})")
    assert names[1] == ["k_conv3w<h2>"] and names[0] != names[1]
    assert not torch.equal(out[1], out[0])
    assert e1 <= 2.0 * e0 + 2.0 ** -22 * ref.abs().max().item(), (e1, e0)


# the geometries the 256 x 128 wide tile takes at the bench's bs = 32 (layer4's 3x3s and its first
# conv / downsample at 32 x 32, conv_1x1_3): 128 tiles of 256 x 256, 256 of 256 x 128
TP128_GEOMS = [
    ("conv", 256, 256, 3, 1, 2, 2, False, 32),
    ("conv", 128, 256, 3, 1, 2, 2, False, 32),
    ("conv", 128, 256, 1, 1, 0, 1, False, 32),
    ("conv", 1280, 256, 1, 1, 0, 1, True, 32),
]


@pytest.mark.parametrize("geom", TP128_GEOMS, ids=[_gid(g) for g in TP128_GEOMS])
def test_wide_tp128_is_f32_accurate(gpu, geom):
    """The 256 x 128 two-plane tile (k_conv3w<TP = 128>, zp_conv_tuning key 14; off by default: on
    layer4 it measured 118.7 us against k_conv3's 114.1) at bs = 32: the dispatch picks it, and its error against float64 is within the two-plane bound of the
    exact-f32-MFMA kernel's (as every geometry in test_split_conv_is_f32_accurate)."""
    from zebrapose_amd import _lib as L
    names = []
    old = L.lib.zp_conv_tuning(14, 1)
    try:
        _check_geom(gpu, geom, "h2", B=32, names_out=names)
    finally:
        L.lib.zp_conv_tuning(14, old)
    assert names == ["k_conv3w<h2,TP=128>"], names


MF32_GEOMS = [
    ("conv", 256, 256, 3, 1, 1, 1, False, 64),    # up1's 3x3 (strips), residual
    ("conv", 512, 512, 3, 1, 4, 4, False, 32),    # layer5 d4 (strips)
    ("conv", 256, 512, 1, 1, 0, 1, False, 32),    # layer5's downsample (1x1: per-step tiles)
    ("convT", 256, 256, 3, 2, 1, 1, False, 32),   # up1's ConvT (four phases)
    ("convT", 320, 256, 3, 2, 1, 1, False, 32),   # up2's ConvT over [up1 | x_64] (Cin 320)
]


@pytest.mark.parametrize("geom", MF32_GEOMS, ids=[_gid(g) for g in MF32_GEOMS])
def test_wide_mf32_is_f32_accurate(gpu, geom):
    """k_conv3w32 (round 6, zp_conv_tuning key 18): the 256 x 256 two-plane tile on
    v_mfma_f32_32x32x16_f16 -- the same staging and flushed numerics as k_conv3w, a different MFMA
    shape, lane layout and epilogue pairing (v_permlane32_swap).  At bs 16 / 32 its error against float64
    is within the two-plane bound of the exact-f32-MFMA kernel's (as every geometry in
    test_split_conv_is_f32_accurate), residual on for the stride-1 convs."""
    from zebrapose_amd import _lib as L
    names = []
    old = L.lib.zp_conv_tuning(18, 1)
    try:
        _check_geom(gpu, geom, "h2", B=16 if geom[-1] == 64 else 32, names_out=names)  # (>= 256 tiles)
    finally:
        L.lib.zp_conv_tuning(18, old)
    assert names == ["k_conv3w<h2>"], names


@pytest.mark.parametrize("geom", [("conv", 512, 512, 3, 1, 4, 4, False, 32), ("conv", 256, 256, 3, 1, 1, 1, False, 64)],
                         ids=["l5_d4_K144", "up1_K72"])
def test_wide_accumulation_forms(gpu, geom):
    """k_conv3w's accumulation forms (zp_conv_tuning key 13) on long-K launches, ReLU'd positive
    inputs as in the network, against float64:
      0 = k_conv3's correction accumulator, flushed per K step by a rounding FMA (the default);
      1 = round 4's one scaled accumulator: every correction product is added by the MFMA into the
          large running sum, whose alignment truncates its low bits -- a systematic negative bias;
      2 = per-step partial sums from zero added by v_add_f32: smaller rms, but the corrections are
          still truncated against the step's main partial;
      4 = (round 6) a persistent correction accumulator per block for the whole K loop, joined to the
          main sum by one rounding FMA after it (the 256 x 128 tile);
      mf32 = the flushed form on 32 x 32 x 16 MFMAs (k_conv3w32, key 18).
    The default's mean signed error (relative to the mean |output|) must be within 3x the exact-f32
    MFMA kernel's (+ a 2^-27 floor) and under a tenth of the one-accumulator form's, its rms within
    the two-plane bound of the f32 kernel's."""
    from zebrapose_amd import _lib as L
    from zebrapose_amd.engine import Engine, Unit, Act, joined
    from zebrapose_amd.model import layers as LY
    kind, cin, cout, k, s, p, d, bias, H = geom
    torch.manual_seed(12)
    B = 8
    conv = LY.Conv2d(cin, cout, k, s, p, d, bias=False)
    bn = LY.BatchNorm2d(cout)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_(0, 0.1)
        bn.running_mean.normal_(0, 0.1)
        bn.running_var.uniform_(0.5, 1.5)
    conv, bn = conv.to(gpu).eval(), bn.to(gpu).eval()
    unit = Unit(conv, bn, relu=False)
    x = torch.randn(B, cin, H, H).clamp(min=0)
    ref = _ref64(kind, conv, bn, x, None, False, s, p, d)
    xh = x.permute(0, 2, 3, 1).contiguous()

    def stats(out):
        dd = joined(out.buf).permute(0, 3, 1, 2).double().cpu() - ref
        return dd.mean().item() / ref.abs().mean().item(), dd.pow(2).mean().sqrt().item() / ref.pow(2).mean().sqrt().item()
    stat = {}
    f32 = Engine(torch.nn.Module(), torch.float32)
    oa = Act(torch.empty(B, H, H, cout, device=gpu))
    f32.unit_fwd(unit, Act(xh.to(gpu)), oa, None)
    torch.cuda.synchronize()
    stat["f32"] = stats(oa)
    xa = Act(_split_act(xh, gpu, "h2"))
    eng = Engine(torch.nn.Module(), torch.float32, split="h2")
    old_min, old_acc, old_sk = L.lib.zp_conv_tuning(11, 1), L.lib.zp_conv_tuning(13, -1), L.lib.zp_conv_tuning(12, 0)
    try:
        for acc in (-1, 0, 1, 2, 4, "mf32"):
            old18 = L.lib.zp_conv_tuning(18, 1 if acc == "mf32" else 0)
            L.lib.zp_conv_tuning(13, 0 if acc == "mf32" else acc)
            oa = Act(eng._empty((B, H, H, cout), gpu))
            eng.stage_log = []
            eng.unit_fwd(unit, xa, oa, None)
            torch.cuda.synchronize()
            L.lib.zp_conv_tuning(18, old18)
            want = "k_conv3w<h2,TP=128>" if acc == 4 else "k_conv3w<h2>"
            assert [r[1] for r in eng.stage_log] == [want], eng.stage_log
            stat[acc] = stats(oa)
    finally:
        L.lib.zp_conv_tuning(11, old_min)
        L.lib.zp_conv_tuning(13, old_acc)
        L.lib.zp_conv_tuning(12, old_sk)
    print(f"{geom}: (bias, rms) relative -- f32 MFMA {stat['f32']}, flushed {stat[0]}, one accumulator {stat[1]}, "
          f"per-step partial {stat[2]}, persistent correction accumulator {stat[4]}")
    dflt = L.lib.zp_conv_tuning(13, -1)
    L.lib.zp_conv_tuning(13, dflt)
    # the default (-1) is one of the unbiased forms: the flushed one (0) or, since round 6, the
    # persistent correction accumulator on the 256 x 128 tile (4)
    assert stat[-1] in (stat[0], stat[4])
    for form in (0, 4, "mf32"):  # unbiased: the corrections are never added into the 2^11-larger main sum
        assert abs(stat[form][0]) <= 3.0 * abs(stat["f32"][0]) + 2.0 ** -27, (form, stat)
        assert abs(stat[form][0]) <= abs(stat[1][0]) / 10.0, (form, stat)
        assert stat[form][1] <= BOUND["h2"][0] * stat["f32"][1], (form, stat)


# schedule flags of the two-plane kernels that must not change a single stored bit (zp_conv_tuning
# key 1 = ZP_CONV_FLAGS; 478 = the default set): 268435456 no strip staging (k_conv3w), 134217728
# caller's sub-problem order instead of longest first, 1 plain instead of non-temporal stores, 512
# the 8-byte epilogue (k_conv3 / k_conv3s), 32 the 256-pixel k_conv3s tile
_BITWISE_FLAGS = [268435456, 134217728, 1, 512, 32]


@pytest.mark.parametrize("geom,B,kernel,tp128",
                         [(("conv", 256, 256, 3, 1, 1, 1, False, 64), 16, "k_conv3w<h2>", 1),    # strips
                          (("convT", 256, 256, 3, 2, 1, 1, False, 32), 16, "k_conv3w<h2>", 1),   # 4 phases
                          (("conv", 64, 64, 3, 1, 1, 1, False, 64), 8, "k_conv3s<h2,WC=2>", 1),  # WP = 2
                          (("conv", 256, 256, 3, 1, 2, 2, False, 32), 32, "k_conv3<h2,WC=4,NWP=4>", 0),
                          (("conv", 256, 256, 3, 1, 2, 2, False, 32), 32, "k_conv3w<h2,TP=128>", 1)],
                         ids=["wide3x3", "wideConvT", "strip64", "conv3_layer4", "wide128_layer4"])
def test_schedule_flags_are_bit_identical(gpu, geom, B, kernel, tp128):
    """Round-4 schedule choices (strip staging of the wide tile, longest-first phase order, nt
    stores, the paired 16-byte epilogue, the 128-pixel strip tile) change the data movement only:
    with each switched back, the stored two-plane outputs are bit-identical (residual on for the
    convs)."""
    from zebrapose_amd import _lib as L
    from zebrapose_amd.engine import Engine, Unit, Act
    from zebrapose_amd.model import layers as LY
    kind, cin, cout, k, s, p, d, bias, H = geom
    torch.manual_seed(11)
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
    conv, bn = conv.to(gpu).eval(), bn.to(gpu).eval()
    unit = Unit(conv, bn, relu=True)
    OH, OW = unit.out_hw(H, H)
    x = torch.randn(B, cin, H, H)
    eng = Engine(torch.nn.Module(), torch.float32, split="h2")
    xa = Act(_split_act(x.permute(0, 2, 3, 1).contiguous(), gpu, "h2"))
    ra = None
    if kind == "conv":
        res = torch.randn(B, cout, OH, OW)
        ra = Act(_split_act(res.permute(0, 2, 3, 1).contiguous(), gpu, "h2"))
    outs = {}
    old14 = L.lib.zp_conv_tuning(14, tp128)
    try:
        # (round 6) "subint1": zp_conv_tuning key 17 = 1, the ConvT phases interleaved per pixel tile on
        # one XCD instead of dispatched phase by phase (the default); "pfb0": key 21 = 0, the strip
        # tile's next-step pixel fragments read after the step's barrier instead of before it
        for extra in [0] + _BITWISE_FLAGS + ["subint1", "pfb0"]:
            named = extra in ("subint1", "pfb0")
            old = L.lib.zp_conv_tuning(1, 478 + (0 if named else extra))
            old17 = L.lib.zp_conv_tuning(17, 1 if extra == "subint1" else -1)
            old21 = L.lib.zp_conv_tuning(21, 0 if extra == "pfb0" else -1)
            try:
                oa = Act(eng._empty((B, OH, OW, cout), gpu))
                eng.stage_log = []
                eng.unit_fwd(unit, xa, oa, None, res=ra)
                torch.cuda.synchronize()
            finally:
                L.lib.zp_conv_tuning(1, old)
                L.lib.zp_conv_tuning(17, old17)
                L.lib.zp_conv_tuning(21, old21)
            outs[extra] = oa.buf._base.clone()
    finally:
        L.lib.zp_conv_tuning(14, old14)
    names = [r[1] for r in eng.stage_log]
    print(geom, names)
    assert names == [kernel], names
    for extra in _BITWISE_FLAGS + ["subint1", "pfb0"]:
        assert torch.equal(outs[extra], outs[0]), (geom, extra)


@pytest.mark.parametrize("geom,B", [(("conv", 256, 256, 3, 1, 2, 2, False, 32), 1),   # bs 1 layer4: split-K
                                    (("conv", 64, 128, 3, 2, 1, 1, False, 64), 2),    # layer2's first conv
                                    (("conv", 64, 128, 3, 2, 1, 1, False, 64), 32)],  # the same, unsplit
                         ids=["l4_bs1_splitk", "l2a_bs2_splitk", "l2a_bs32"])
def test_pipe_ring_depth_is_bit_identical(gpu, geom, B):
    """zp_conv_tuning key 19 (round 6): the register-pipelined two-plane 64-channel k_conv3 tile with
    a 3- or 4-stage ring instead of 2 moves the DMA further ahead only -- the stored outputs (split-K
    slices summed by k_splitk_epi, or the direct epilogue) are bit-identical to the default's."""
    from zebrapose_amd import _lib as L
    from zebrapose_amd.engine import Engine, Unit, Act
    from zebrapose_amd.model import layers as LY
    kind, cin, cout, k, s, p, d, bias, H = geom
    torch.manual_seed(12)
    conv = LY.Conv2d(cin, cout, k, s, p, d, bias=bias)
    bn = LY.BatchNorm2d(cout)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_(0, 0.1)
        bn.running_mean.normal_(0, 0.1)
        bn.running_var.uniform_(0.5, 1.5)
    conv, bn = conv.to(gpu).eval(), bn.to(gpu).eval()
    unit = Unit(conv, bn, relu=True)
    OH, OW = unit.out_hw(H, H)
    x = torch.randn(B, cin, H, H)
    eng = Engine(torch.nn.Module(), torch.float32, split="h2")
    xa = Act(_split_act(x.permute(0, 2, 3, 1).contiguous(), gpu, "h2"))
    outs = {}
    for st in (2, 3, 4):
        old = L.lib.zp_conv_tuning(19, st)
        try:
            oa = Act(eng._empty((B, OH, OW, cout), gpu))
            eng.stage_log = []
            eng.unit_fwd(unit, xa, oa, None)
            torch.cuda.synchronize()
        finally:
            L.lib.zp_conv_tuning(19, old)
        assert [r[1] for r in eng.stage_log] == ["k_conv3<h2,WC=2,NWP=2>"], eng.stage_log
        outs[st] = oa.buf._base.clone()
    assert float(outs[2].float().abs().sum()) > 0
    for st in (3, 4):
        assert torch.equal(outs[st], outs[2]), (geom, B, st)
