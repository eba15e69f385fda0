"""Memory-bound helper kernels against torch on the same values: global average pool (ASPP image
branch, aspp.py:94), its backward pieces (per-channel H*W sums, broadcast back over H*W) and the
NCHW f32 -> NHWC input conversion, in the vectorised (16 B) and scalar (odd channel slice) forms."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("C,ld,c0", [(512, 512, 0), (256, 1280, 1024), (20, 24, 2)])
def test_avgpool_sum_broadcast(gpu, prec, C, ld, c0):
    from zebrapose_amd import _lib as L
    dt = torch.float32 if prec == "fp32" else torch.bfloat16
    dc = L.dtype_code(dt)
    torch.manual_seed(0)
    B, H, W = 3, 17, 32
    buf = torch.randn(B, H, W, ld).to(dt)
    x = buf[..., c0:c0 + C].float()
    d = buf.to(gpu)
    out = torch.empty(B, C, dtype=dt, device=gpu)
    L.call("zp_global_avgpool", d.data_ptr(), B, H, W, ld, c0, C, dc, out.data_ptr(), L.stream_ptr())
    want = x.double().mean(dim=(1, 2)).float().to(dt).float()
    assert torch.equal(out.float().cpu(), want)
    L.call("zp_sum_hw", d.data_ptr(), B, H, W, ld, c0, C, dc, out.data_ptr(), L.stream_ptr())
    want = x.sum(dim=(1, 2))
    got = out.float().cpu()
    tol = 1e-5 if prec == "fp32" else 1e-2
    assert ((got - want).abs() <= tol * (want.abs() + 1)).all()
    src = torch.randn(B, C).to(dt).to(gpu)
    y = torch.zeros(B, H, W, ld, dtype=dt, device=gpu)
    L.call("zp_broadcast_hw", src.data_ptr(), B, C, dc, y.data_ptr(), H, W, ld, c0, L.stream_ptr())
    yc = y.cpu()
    assert torch.equal(yc[..., c0:c0 + C], src.cpu()[:, None, None, :].expand(B, H, W, C))
    assert not yc[..., :c0].any() and not yc[..., c0 + C:].any()


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("cpad", [8, 5])
def test_nchw_to_nhwc(gpu, prec, cpad):
    from zebrapose_amd import _lib as L
    dt = torch.float32 if prec == "fp32" else torch.bfloat16
    if prec == "bf16" and cpad == 5:
        pytest.skip("the network pads to a full 16 B vector")
    torch.manual_seed(1)
    x = torch.randn(2, 3, 9, 14)
    y = torch.full((2, 9, 14, cpad), 7.0, dtype=dt, device=gpu)
    L.call("zp_nchw_to_nhwc", x.to(gpu).data_ptr(), 2, 3, 9, 14, cpad, L.dtype_code(dt), y.data_ptr(), L.stream_ptr())
    want = torch.zeros(2, 9, 14, cpad)
    want[..., :3] = x.permute(0, 2, 3, 1)
    assert torch.equal(y.cpu().float(), want.to(dt).float())


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32, torch.float16])
def test_pack_weight_multi_matches_single_packs(gpu, dt):
    """The batched repack of training (one grid row per job) against zp_pack_weight job by job:
    plain 3x3, a tap subset (ConvT phase), transposed (dgrad / ConvT layout), the reversed tap order
    of a data-gradient packing (the compile-time 3x3 forms of k_pack_multi), a padded-channel stem
    (cstride 8 > 3 channels, k_pad tail) and a 1x1 with padded rows."""
    import ctypes as C
    from zebrapose_amd import _lib as L
    torch.manual_seed(0)
    code = L.dtype_code(dt)
    specs = [  # d0, d1, k, transposed, taps, cstride, rows_pad, k_pad
        (128, 64, 3, 0, [(i // 3, i % 3) for i in range(9)], 64, 128, 576),
        (64, 96, 3, 0, [(0, 0), (0, 2), (2, 0), (2, 2)], 96, 64, 384),
        (96, 64, 3, 1, [(i // 3, i % 3) for i in range(9)], 96, 64, 896),
        (96, 64, 3, 1, [(2 - i // 3, 2 - i % 3) for i in range(9)], 96, 64, 896),  # dgrad: taps reversed
        (64, 128, 3, 0, [(2 - i // 3, 2 - i % 3) for i in range(9)], 128, 64, 1152),
        (64, 3, 7, 0, [(i // 7, i % 7) for i in range(49)], 8, 64, 448),
        (17, 320, 1, 0, [(0, 0)], 320, 32, 320),
    ]
    jobs, singles, outs = [], [], []
    srcs = []
    for d0, d1, k, tr, taps, cs, rp, kp in specs:
        src = torch.randn(d0, d1, k, k, device="cuda")
        srcs.append(src)
        ky = [t[0] for t in taps]
        kx = [t[1] for t in taps]
        ref = torch.empty((rp, kp), dtype=dt, device="cuda")
        L.call("zp_pack_weight", src.data_ptr(), d0, d1, k, k, tr, len(taps), (C.c_int * len(ky))(*ky),
               (C.c_int * len(kx))(*kx), cs, code, ref.data_ptr(), rp, kp, L.stream_ptr())
        got = torch.full((rp, kp), 7.0, dtype=dt, device="cuda")  # garbage: every element must be written
        j = L.PackJob()
        j.src, j.dst, j.d0, j.d1, j.kh, j.kw, j.transposed = src.data_ptr(), got.data_ptr(), d0, d1, k, k, tr
        j.ntaps, j.cstride, j.rows_pad, j.k_pad, j.dtype = len(taps), cs, rp, kp, code
        for t, (a, b) in enumerate(taps):
            j.ky[t], j.kx[t] = a, b
        jobs.append(j)
        singles.append(ref)
        outs.append(got)
    arr = (L.PackJob * len(jobs))(*jobs)
    table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).cuda()
    pre = [0]
    for j in jobs:
        pre.append(pre[-1] + j.rows_pad * j.k_pad)
    prefix = torch.tensor(pre, dtype=torch.int64, device="cuda")
    L.call("zp_pack_weight_multi", len(jobs), table.data_ptr(), prefix.data_ptr(), pre[-1], L.stream_ptr())
    for ref, got in zip(singles, outs):
        assert torch.equal(ref, got)


@pytest.mark.parametrize("cin,cout,ldy,cy0", [(32, 320, 320, 0), (64, 64, 128, 64)])
def test_conv1x1_narrow_k(gpu, cin, cout, ldy, cy0):
    """k_conv1x1n (zp_conv2d_config variant 7): a 1x1 conv with 32 / 64 input channels and a wide
    bf16 output -- the head's data gradient in training, 32 -> 320 at 128 x 128 -- against a float64
    matmul of the same bf16 operands, to 1 bf16 ulp of the output (+2^-16 of the scale for cancelling
    sums), written into a channel slice (ldy / cy0) without touching its neighbours."""
    import ctypes as C
    from zebrapose_amd import _lib as L
    torch.manual_seed(cin + cout)
    N, H, W = 4, 128, 128
    x = torch.randn(N, H, W, cin).to(torch.bfloat16).cuda()
    w = (torch.randn(cout, cin, 1, 1) * 0.2)
    rows = L.lib.zp_conv_rows_pad(cout)
    kp = 64
    wp = torch.empty((rows, kp), dtype=torch.bfloat16, device="cuda")
    wd = w.cuda()
    L.call("zp_pack_weight", wd.data_ptr(), cout, cin, 1, 1, 0, 1, (C.c_int * 1)(0), (C.c_int * 1)(0), cin, L.ZP_BF16,
           wp.data_ptr(), rows, kp, L.stream_ptr())
    y = torch.full((N, H, W, ldy), 3.0, dtype=torch.bfloat16, device="cuda")
    a = L.ConvArgs()
    a.dtype, a.x, a.ldx, a.cx0, a.IH, a.IW, a.Cin = L.ZP_BF16, x.data_ptr(), cin, 0, H, W, cin
    a.N, a.GH, a.GW, a.sy, a.sx = N, H, W, 1, 1
    a.Cout, a.k_pad, a.w_rows, a.relu, a.out_mode, a.nsub = cout, kp, rows, 0, L.ZP_OUT_NHWC, 1
    s = a.sub[0]
    s.w, s.y, s.ldy, s.cy0, s.OH, s.OW, s.oys, s.oxs, s.ntaps = wp.data_ptr(), y.data_ptr(), ldy, cy0, H, W, 1, 1, 1
    s.kw, s.dil, s.pad = 1, 1, 0
    tc, tp, st, var = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    L.call("zp_conv2d_config", C.byref(a), C.byref(tc), C.byref(tp), C.byref(st), C.byref(var))
    assert var.value == 7
    L.check(L.lib.zp_conv2d(C.byref(a), L.stream_ptr()), "zp_conv2d")
    torch.cuda.synchronize()
    wb = w.reshape(cout, cin).to(torch.bfloat16).double()
    ref = (x.cpu().double().reshape(-1, cin) @ wb.t()).reshape(N, H, W, cout)
    got = y.cpu()[..., cy0:cy0 + cout].double()
    ulp = ref.abs().clamp_min(1e-30) * 2.0 ** -7
    err = (got - ref).abs()
    assert bool((err <= ulp + 2.0 ** -16 * float(ref.abs().max())).all()), float((err / ulp).max())
    keep = torch.cat([y.cpu()[..., :cy0], y.cpu()[..., cy0 + cout:]], -1)
    assert bool((keep == 3.0).all())
