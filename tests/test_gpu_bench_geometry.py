"""Parity at the configuration the bench reports (BASELINE.json configs[1]: ResNet34 + DeepLabv3,
bs=32, 256x256 crops), in fp32 (the benched headline: the two-plane split engine, with up2's last
conv and the head fused into one launch) and bf16 (the labelled throughput leg), through the
drop-in module and libzp.so.  Reference anchor: model/BinaryCodeNet.py:161-174, aspp.py:83-114, test.py:248.

Weights: the synthetic checkpoint with BN calibrated on 256x256 crops by the real reference
(tests/golden/r34_bn_buffers256.npz, oracle/capture_fixtures.py capture_fwd256): |logit| <= 6 on the
N(0,1) crops it was calibrated on, <= ~240 on the bench's uniform-u8 crops.

Why bf16 is checked layer by layer.  Even with that checkpoint the random-weight network amplifies
tiny perturbations ~50x (oracle: a 1e-6 relative input change moves the code logits by 5e-5
rel-L2).  bf16 storage rounding alone moves the logits by 18.6% rel-L2 against fp32, and -- the
decisive measurement -- the bf16-emulating oracle (oracle/ref_cpu.py forward_lowp) run twice with
only its accumulation order changed (f32 vs f64 convs) differs from itself by 8.7% rel-L2 and 2.9%
of the code bits.  No elementwise network-level bf16 comparison can therefore separate a kernel
bug from 1-ulp rounding flips.  So the bf16 path is checked TEACHER-FORCED: every op of the
B=32 forward is replayed on the host from the device's own stored 16-bit inputs (engine.trace)
with the storage roundings and epilogue arithmetic of the device (oracle/ref_cpu.py lp_conv), and
its stored output must match to within 1 bf16 ulp (plus a tiny absolute term for outputs that
cancel to ~0), with the fraction of not-bit-identical elements bounded (observed 0.02%).  That covers every tile
variant the bs=32 dispatch picks (the 256-channel tile, the strip kernel, the 4-phase ConvT, the
merged ASPP launch) at the bench's own shapes.  The end-to-end bf16 logits are additionally held
against the emulating oracle: the bench's uniform-u8 crops condition far better than the N(0,1)
fixture input, and the bs=32 logits land at 1.1% rel-L2 / 99.8% identical bits from it.

fp32 mode: logits of sampled crops within the north-star's 1e-3 of the fp32 oracle (pinned to
the reference by r34_fwd256.npz), bits identical outside the |logit| <= 1e-3 band, and the same
teacher-forced replay at f32 tolerance.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
THR = np.float32(8.940696716308594e-08)
B, S = 32, 256
SAMPLE = (0, 13, 31)


def bench_crops(seed=100):
    """bench.py synthetic_crops: uint8 crops normalised as bop_dataset_pytorch.py:333-347."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    u8 = torch.randint(0, 256, (B, 3, S, S), generator=g, dtype=torch.uint8)
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    return (u8.float() / 255.0 - mean) / std


@pytest.fixture(scope="module")
def setup(golden):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import ref_cpu
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    sd = ref_cpu.synthetic_state(34, 16, 0, dict(golden("r34_bn_buffers256.npz")))
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="bf16")
    net.load_state_dict(sd)
    return net.cuda().eval(), sd, bench_crops()


def _nchw(act, b):
    """crop b of an NHWC channel slice -> f32 NCHW [1, C, H, W] on the host (the split-fp32 engine's
    three planes joined exactly)."""
    from zebrapose_amd.engine import joined
    return joined(act.buf)[b:b + 1, :, :, act.c0:act.c0 + act.C].permute(0, 3, 1, 2).cpu()


def _ulp_bf16(v):
    """spacing of bf16 at |v| (f32 tensor)."""
    a = v.abs().clamp_min(2.0 ** -126)
    e = torch.floor(torch.log2(a))
    return torch.pow(2.0, e - 7)


def _bn_of(unit):
    bn = unit.bn
    if bn is None:
        return None
    return tuple(t.detach().float().cpu() for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var))


def replay(rec, b, dt):
    """Host replay of one traced eval op for crop b -> (expected, got) f32 NCHW tensors."""
    from oracle import ref_cpu
    kind, unit, x, out, res = rec
    if kind == "input":
        exp = x[b:b + 1].float().cpu()
        exp = exp if dt == torch.float32 else ref_cpu._q(exp, dt)
        got = _nchw(out, b)
        assert not got[:, 3:].any(), "input channel padding must be zero"
        return exp, got[:, :3]
    if kind == "maxpool":
        return F.max_pool2d(_nchw(x, b), 3, 2, 1), _nchw(out, b)
    if kind == "avgpool":
        m = _nchw(x, b).double().mean((2, 3), keepdim=True).float()
        return (m if dt == torch.float32 else ref_cpu._q(m, dt)), _nchw(out, b)
    if kind == "broadcast":
        return _nchw(x, b).expand(-1, -1, out.H, out.W), _nchw(out, b)
    conv = unit.conv
    xin = _nchw(x, b)[:, :unit.cin_w]
    w = conv.weight.detach().float().cpu()
    bias = None if conv.bias is None else conv.bias.detach().float().cpu()
    if kind == "head":
        mask, code = out
        exp = ref_cpu.lp_conv(xin, w, None, bias, None, False, dt=dt, out_f32=True) if dt != torch.float32 else \
            F.conv2d(xin, w, bias)
        got = torch.cat([mask[b:b + 1].cpu(), code[b:b + 1].cpu()], 1)
        return exp, got
    r = None if res is None else _nchw(res, b)
    kw = dict(stride=unit.s, pad=unit.p, dil=unit.d, transposed=unit.kind == "convT")
    if dt == torch.float32:
        if kw["transposed"]:
            acc = F.conv_transpose2d(xin, w, None, 2, 1, 1)
        else:
            acc = F.conv2d(xin, w, None, unit.s, unit.p, unit.d)
        bn = _bn_of(unit)
        if bn is None:
            y = acc + (0 if bias is None else bias.view(1, -1, 1, 1))
        else:
            s, sh = ref_cpu.fold_f32(*bn, bias=bias)
            y = acc * s.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)
        if r is not None:
            y = y + r
        if unit.relu:
            y = F.relu(y)
        return y, _nchw(out, b)
    exp = ref_cpu.lp_conv(xin, w, _bn_of(unit), bias, r, unit.relu, dt=dt, **kw)
    return exp, _nchw(out, b)


def _label(rec, i):
    kind, unit = rec[0], rec[1]
    if unit is None:
        return f"{i}:{kind}"
    return f"{i}:{kind} {unit.kind} k{unit.k} s{unit.s} d{unit.d} {unit.cin_w}->{unit.cout}"


def run_traced(net, x):
    eng = net.net.eval_engine()
    eng.trace = []
    try:
        with torch.no_grad():
            m, c = net(x)
        torch.cuda.synchronize()
        return m, c, eng.trace
    finally:
        eng.trace = None


def test_bf16_bench_geometry_teacher_forced(setup):
    """Every op of the bs=32 256x256 bf16 forward, replayed on the host for crops 0, 13, 31 from
    the device's own stored inputs: stored outputs within 1 bf16 ulp (+ 2^-12 of the layer's RMS
    for cancelling outputs), at most 0.5% of the elements of any layer not bit-identical (observed
    0.02%: the f32 accumulation orders of MFMA and the host conv rarely straddle a bf16 midpoint)."""
    net, sd, x = setup
    net.set_precision("bf16")
    net.cuda().eval()
    m, c, trace = run_traced(net, x.cuda())
    kinds = {r[0] for r in trace}
    assert {"input", "conv", "maxpool", "avgpool", "broadcast", "head"} <= kinds
    assert sum(r[0] == "conv" for r in trace) == 48
    worst_frac, worst_ulp = 0.0, 0.0
    for b in SAMPLE:
        for i, rec in enumerate(trace):
            exp, got = replay(rec, b, torch.bfloat16)
            assert exp.shape == got.shape, (_label(rec, i), exp.shape, got.shape)
            d = (got - exp).abs()
            if rec[0] == "head":  # f32 output: accumulation order only
                scale = float(exp.abs().max())
                assert float(d.max()) <= 2e-5 * max(scale, 1.0), (_label(rec, i), float(d.max()), scale)
                continue
            rms = float(exp.pow(2).mean().sqrt())
            ulp = _ulp_bf16(torch.maximum(exp.abs(), got.abs()))
            tol = ulp + 2.0 ** -12 * rms
            bad = d > tol
            frac = float((d > 0).float().mean())
            worst_frac = max(worst_frac, frac)
            worst_ulp = max(worst_ulp, float((d / ulp).max()))
            assert not bool(bad.any()), (f"crop {b} {_label(rec, i)}: {int(bad.sum())} elements beyond 1 ulp, "
                                         f"max |d| {float(d.max()):.3g} rms {rms:.3g}")
            assert frac <= 0.005, (f"crop {b} {_label(rec, i)}", frac)
    print(f"bf16 teacher-forced: {len(trace)} ops x {len(SAMPLE)} crops; worst not-bit-identical fraction "
          f"{worst_frac:.4f}, worst |d| {worst_ulp:.2f} ulp")


@pytest.mark.parametrize("precision", ["bf16", "fp16"])
def test_16bit_bench_geometry_fused_head(setup, precision):
    """The 16-bit forward as benched: up2's last 3x3 conv and the 1x1 head fused (zp_conv2d_head,
    VERDICT r4 #6; reference aspp.py:105-112 + BinaryCodeNet.py:172).  The strip kernel's epilogue
    feeds its stored-precision outputs (rounded exactly as the unfused path stores them) to the head's
    MFMAs, per 128-channel cout tile; a second launch adds the two tiles' partials and the bias.  Against
    the unfused forward (conv stored into the [up2 | x_128] concat, then the separate head launch) the
    logits differ only by the head sums' f32 summation order: within 1e-6 of the logit scale.  The stage
    log names the fused kernel and holds no separate head launch."""
    net, sd, x = setup
    net.set_precision(precision)
    net.cuda().eval()
    eng = net.net.eval_engine()
    assert eng.head_fusable(x.shape[0], x.shape[2] // 2, x.shape[3] // 2)
    eng.stage_log = []
    with torch.no_grad():
        m, c = net(x.cuda())
    log, eng.stage_log = eng.stage_log, None
    tn = {"bf16": "bf16", "fp16": "f16"}[precision]
    assert any(k == f"k_conv_strip2_head<{tn},WC=4>" for _, k, *_ in log), [k for _, k, *_ in log]
    assert not any(st == "head" for st, *_ in log)
    eng.fuse_head = False
    with torch.no_grad():
        mu, cu = net(x.cuda())
    eng.fuse_head = True
    for a, b in ((m, mu), (c, cu)):
        assert torch.isfinite(a).all()
        d = float((a - b).abs().max())
        scale = float(b.abs().max())
        print(f"{precision} fused vs unfused head: max |d| {d:.3g} = {d / scale:.3g} of the logit scale {scale:.3g}")
        assert d <= 1e-6 * scale
    net.set_precision("bf16")


def test_bf16_bench_geometry_end_to_end(setup):
    """bs=32 bf16 logits of crops 0, 13, 31 against the bf16-emulating oracle and the fp32 oracle, in
    norm and bit agreement, plus the exact on-device decode of those logits."""
    from oracle import ref_cpu
    net, sd, x = setup
    net.set_precision("bf16")
    net.cuda().eval()
    with torch.no_grad():
        m, c = net(x.cuda())
    m, c = m.cpu(), c.cpu()
    xs = x[list(SAMPLE)]
    with torch.no_grad():
        em, ec = ref_cpu.forward_lowp(sd, xs, 34)
        fm, fc = ref_cpu.forward(sd, xs, 34)
    got_m, got_c = m[list(SAMPLE)].numpy(), c[list(SAMPLE)].numpy()
    # observed (MI355X, r02): vs emulated 1.1% / 0.6% (mask / code), 99.8% / 99.9% of the bits; vs fp32
    # 1.4% / 0.8%.  The bench crops (uniform u8) condition much better than the N(0,1) fixture input.
    for name, (om, oc), bound, min_agree in (("emulated bf16", (em, ec), 0.05, 0.99), ("fp32", (fm, fc), 0.08, 0.98)):
        for g, o in ((got_m, om.numpy()), (got_c, oc.numpy())):
            assert np.isfinite(g).all()
            rel = float(np.linalg.norm(g - o) / np.linalg.norm(o))
            agree = float(((g > THR) == (o > THR))[np.abs(o) > 0.25].mean())
            print(f"bs=32 bf16 vs {name}: rel-L2 {rel:.4f}, bits agreeing outside |logit|<=0.25: {agree:.4f}")
            assert rel <= bound, (name, rel)
            assert agree >= min_agree, (name, agree)
    # the decode of the bench step on the GPU's own logits is exact (crop by crop vs the oracle)
    from zebrapose_amd.decode import Decoder
    rng = np.random.default_rng(0)
    lut = rng.standard_normal((65536, 3)) * 50
    lut[::97] = np.nan
    side = rng.integers(64, 401, B)
    bb = np.stack([rng.integers(0, 300, B), rng.integers(0, 200, B), side, side], 1)
    dec = Decoder(lut, device="cuda")
    res = Decoder.to_host(*dec(m.cuda(), c.cuda(), bb, bbox_size=S // 2))
    for b in SAMPLE:
        n, p2d, p3d, _ = ref_cpu.decode_crop(m[b, 0].numpy(), c[b].numpy(), lut, bb[b])
        assert len(res[b][0]) == n
        np.testing.assert_array_equal(res[b][0], p2d)
        np.testing.assert_array_equal(res[b][1], p3d)


@pytest.mark.parametrize("split", ["x3", "h2", False], ids=["split_x3", "split_h2", "f32_mfma"])
def test_fp32_bench_geometry(setup, split):
    """fp32 mode at bs=32: the split-fp32 eval engines (two fp16 planes, ZP_F32H2, the default; three
    bf16 planes, ZP_F32X3) and the exact-f32-MFMA engine: logits of crops 0, 13, 31 within the
    north-star 1e-3 of the fp32 oracle, mask / code bits identical outside the band; every op replayed
    teacher-forced to 1e-5 rel from the device's own stored (joined) inputs (the trace keeps the head
    a separate op: test_fp32_bench_geometry_fused_head covers the fused launch)."""
    from oracle import ref_cpu
    net, sd, x = setup
    net.set_precision("fp32")
    net.net.f32_split = split
    net.cuda().eval()
    m, c, trace = run_traced(net, x.cuda())
    b = SAMPLE[1]
    worst = []
    for i, rec in enumerate(trace):
        exp, got = replay(rec, b, torch.float32)
        scale = max(float(exp.abs().max()), 1e-6)
        worst.append((float((got - exp).abs().max()) / scale, _label(rec, i)))
    worst.sort(reverse=True)
    print("teacher-forced worst ops (max|d| / scale):", [(f"{e:.2e}", l) for e, l in worst[:6]])
    xs = x[list(SAMPLE)]
    with torch.no_grad():
        fm, fc = ref_cpu.forward(sd, xs, 34)
        sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
        dm, dc = ref_cpu.forward(sd64, xs.double(), 34)
    for got, ref, r64 in ((m.cpu()[list(SAMPLE)].numpy(), fm.numpy(), dm.numpy()),
                          (c.cpu()[list(SAMPLE)].numpy(), fc.numpy(), dc.numpy())):
        d = float(np.abs(got - ref).max())
        print(f"bs=32 fp32 max |d| vs CPU f32 oracle {d:.3g}; vs float64 {float(np.abs(got - r64).max()):.3g} "
              f"(CPU f32 oracle vs float64 {float(np.abs(ref - r64).max()):.3g}; |logit| max {np.abs(ref).max():.3g})")
    for e, l in worst:
        assert e <= 1e-5, (l, e)
    for got, ref in ((m.cpu()[list(SAMPLE)].numpy(), fm.numpy()), (c.cpu()[list(SAMPLE)].numpy(), fc.numpy())):
        np.testing.assert_allclose(got, ref, atol=1e-3, rtol=0)
        amb = np.abs(ref) <= 1e-3
        bad = ((got > THR) != (ref > THR)) & ~amb
        assert int(bad.sum()) == 0
        assert amb.mean() <= 1e-3
    net.net.f32_split = True
    net.set_precision("bf16")


@pytest.mark.parametrize("split", ["x3", "h2", False], ids=["split_x3", "split_h2", "f32_mfma"])
def test_fp32_matches_reference_fixture_256(golden, split):
    """The reference's own 256x256 forward (B=2, BN calibrated at 256x256 -- r34_fwd256.npz) through
    the fp32 HIP path (split-fp32 eval engine and exact-f32 MFMA) within the north-star 1e-3."""
    from oracle import ref_cpu
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    f = golden("r34_fwd256.npz")
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="fp32")
    net.net.f32_split = split
    net.load_state_dict(ref_cpu.synthetic_state(34, 16, 0, dict(golden("r34_bn_buffers256.npz"))))
    net = net.cuda().eval()
    with torch.no_grad():
        m, c = net(torch.from_numpy(f["x"]).cuda())
    for got, ref in ((m.cpu().numpy(), f["mask"]), (c.cpu().numpy(), f["code"])):
        print(f"fwd256 fixture fp32 max |d| {np.abs(got - ref).max():.3g}")
        np.testing.assert_allclose(got, ref, atol=1e-3, rtol=0)
        amb = np.abs(ref) <= 1e-3
        assert int((((got > THR) != (ref > THR)) & ~amb).sum()) == 0


def test_fp32_bench_geometry_fused_head(setup):
    """The benched fp32 forward as benched: two planes, up2's last 3x3 conv and the 1x1 head in one
    launch (zp_conv2d_head: the conv's output is never stored; the head reads x_128 itself).  Logits of
    the sampled crops within the north-star 1e-3 of the fp32 oracle, and equal to the unfused two-plane
    forward up to the head sum's f32 rounding: the fused epilogue splits the conv output into the same
    two fp16 planes the unfused path stores (zp_conv3w.hip HEAD epilogue), so the two differ only in the
    order of the head's 320-term sums (a loose bound would hide a channel-mapping error in
    the fused head's weight layout)."""
    from oracle import ref_cpu
    net, sd, x = setup
    net.set_precision("fp32")
    net.net.f32_split = "h2"
    net.cuda().eval()
    eng = net.net.eval_engine()
    assert eng.head_fusable(x.shape[0], x.shape[2] // 2, x.shape[3] // 2)
    eng.stage_log = []
    with torch.no_grad():
        m, c = net(x.cuda())
    log, eng.stage_log = eng.stage_log, None
    assert any(k.startswith("k_conv3w_head") for _, k, *_ in log), [k for _, k, *_ in log]
    assert not any(st == "head" for st, *_ in log)  # no separate head launch
    eng.fuse_head = False
    with torch.no_grad():
        mu, cu = net(x.cuda())
    eng.fuse_head = True
    for a, b in ((m, mu), (c, cu)):
        d = float((a - b).abs().max())
        scale = float(b.abs().max())
        print(f"fused vs unfused head: max |d| {d:.3g} = {d / scale:.3g} of the logit scale {scale:.3g}")
        assert d <= 2e-4 and d <= 1e-6 * scale
    xs = x[list(SAMPLE)]
    with torch.no_grad():
        fm, fc = ref_cpu.forward(sd, xs, 34)
    for got, ref in ((m.cpu()[list(SAMPLE)].numpy(), fm.numpy()), (c.cpu()[list(SAMPLE)].numpy(), fc.numpy())):
        print(f"fused head bs=32 fp32 max |d| vs CPU f32 oracle {float(np.abs(got - ref).max()):.3g}")
        np.testing.assert_allclose(got, ref, atol=1e-3, rtol=0)
        amb = np.abs(ref) <= 1e-3
        assert int((((got > THR) != (ref > THR)) & ~amb).sum()) == 0
    net.net.f32_split = True
    net.set_precision("bf16")


def test_fused_head_matches_reference_fixture_256(golden):
    """The fused up2-conv + head launch at the reference's own 256x256 fixture (B=2: 128 workgroups,
    below the wide tile's default minimum -- zp_conv_tuning key 11 lowered for the test)."""
    from oracle import ref_cpu
    from zebrapose_amd import _lib as L
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    f = golden("r34_fwd256.npz")
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="fp32")
    net.net.f32_split = "h2"
    net.load_state_dict(ref_cpu.synthetic_state(34, 16, 0, dict(golden("r34_bn_buffers256.npz"))))
    net = net.cuda().eval()
    old = L.lib.zp_conv_tuning(11, 1)
    try:
        eng = net.net.eval_engine()
        assert eng.head_fusable(2, 128, 128)
        eng.stage_log = []
        with torch.no_grad():
            m, c = net(torch.from_numpy(f["x"]).cuda())
        assert any(k.startswith("k_conv3w_head") for _, k, *_ in eng.stage_log)
        eng.stage_log = None
    finally:
        L.lib.zp_conv_tuning(11, old)
    for got, ref in ((m.cpu().numpy(), f["mask"]), (c.cpu().numpy(), f["code"])):
        print(f"fwd256 fixture, fused head: max |d| {np.abs(got - ref).max():.3g}")
        np.testing.assert_allclose(got, ref, atol=1e-3, rtol=0)
        amb = np.abs(ref) <= 1e-3
        assert int((((got > THR) != (ref > THR)) & ~amb).sum()) == 0
