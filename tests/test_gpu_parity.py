"""Network-level parity of the HIP path (through the drop-in module and libzp.so) against the
golden vectors captured from the reference (tests/golden) and against the oracle.

Tolerances:
  fp32 mode  logits |d| <= 1e-3 + 1e-4 |ref| elementwise; mask / code bits identical wherever
             |ref logit| > 1e-3 (the ambiguous band is counted, must be tiny).
  bf16 mode  the synthetic random-weight model is ill-conditioned (oracle: rounding only the INPUT
             to bf16 moves the logits by 4% rel-L2), so bf16 is checked in norm against the fp32
             reference: rel-L2 <= 0.20 (observed 0.16) and >= 99% of the bits outside |ref| < 0.25
             identical.  Per-kernel bf16 accuracy is checked tightly in test_gpu_units.py.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
THR = np.float32(8.940696716308594e-08)


@pytest.fixture(scope="module")
def net_and_state(golden):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import ref_cpu
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    bn = dict(golden("r34_bn_buffers.npz"))
    sd = ref_cpu.synthetic_state(34, 16, 0, bn)
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="fp32")
    net.load_state_dict(sd)
    return net.cuda().eval(), sd


def _bits_check(got, ref, band):
    amb = np.abs(ref) <= band
    gb, rb = got > THR, ref > THR
    bad = (gb != rb) & ~amb
    return int(bad.sum()), int(amb.sum())


# (fixture, keys, atol): the 64x64 fixture has logits up to 5.1 -> atol 1e-3 (observed 1.2e-4).
# The 256x256 fixture (BN calibrated at 256x256) is checked in test_gpu_bench_geometry.py.
@pytest.mark.parametrize("split", ["x3", "h2", False], ids=["split_x3", "split_h2", "f32_mfma"])
@pytest.mark.parametrize("fixture,xkey,mkey,ckey,atol",
                         [("r34_fwd64.npz", "fwd64_x", "fwd64_mask", "fwd64_code", 1e-3)])
def test_forward_fp32_matches_reference(net_and_state, golden, fixture, xkey, mkey, ckey, atol, split):
    """fp32 eval forward: the split-fp32 engine (the default) and the exact-f32-MFMA engine."""
    net, _ = net_and_state
    net.set_precision("fp32")
    net.net.f32_split = split
    f = golden(fixture)
    with torch.no_grad():
        m, c = net(torch.from_numpy(f[xkey]).cuda())
    net.net.f32_split = True
    m, c = m.cpu().numpy(), c.cpu().numpy()
    for got, ref in ((m, f[mkey]), (c, f[ckey])):
        np.testing.assert_allclose(got, ref, atol=atol, rtol=1e-4)
        bad, amb = _bits_check(got, ref, atol)
        assert bad == 0, f"{bad} bits differ outside the |logit| <= {atol} band"
        assert amb <= 0.01 * ref.size  # the ambiguous band itself (reported, tiny)


@pytest.mark.parametrize("split", ["x3", "h2", False], ids=["split_x3", "split_h2", "f32_mfma"])
def test_r50_forward_fp32_matches_reference(golden, split):
    """ResNet50_OS8 + ASPP_50 (340M parameters; Bottleneck stem/layer1/layer2, 1024/2048-channel
    BasicBlock layer4/5, 2048-channel ASPP, 512-channel up2 input) through the HIP path, fp32 mode
    (split-fp32 eval engine and exact-f32 MFMA), against the reference's own 64x64 forward
    (oracle/capture_fixtures.py capture_network(50))."""
    from oracle import ref_cpu
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    f = golden("r50_fwd64.npz")
    sd = ref_cpu.synthetic_state(50, 16, 0, dict(golden("r50_bn_buffers.npz")))
    net = BinaryCodeNet_Deeplab(50, 16, 2, concat=True, output_kernel_size=1, precision="fp32")
    net.net.f32_split = split
    net.load_state_dict(sd)
    net = net.cuda().eval()
    with torch.no_grad():
        m, c = net(torch.from_numpy(f["fwd64_x"]).cuda())
    m, c = m.cpu().numpy(), c.cpu().numpy()
    for got, ref in ((m, f["fwd64_mask"]), (c, f["fwd64_code"])):
        np.testing.assert_allclose(got, ref, atol=1e-3, rtol=1e-4)
        bad, amb = _bits_check(got, ref, 1e-3)
        assert bad == 0 and amb <= 0.01 * ref.size
    del net
    torch.cuda.empty_cache()


def test_forward_bf16_within_conditioning_band(net_and_state, golden):
    net, _ = net_and_state
    net.set_precision("bf16")
    f = golden("r34_fwd64.npz")
    with torch.no_grad():
        m, c = net(torch.from_numpy(f["fwd64_x"]).cuda())
    net.set_precision("fp32")
    for got, ref in ((m.cpu().numpy(), f["fwd64_mask"]), (c.cpu().numpy(), f["fwd64_code"])):
        rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
        out = np.abs(ref) > 0.25
        agree = ((got > THR) == (ref > THR))[out].mean()
        print(f"bf16 @64: rel-L2 {rel:.4g}, bits agree {agree:.4f} outside |ref| <= 0.25")
        # observed (r03, every box so far: deterministic kernels): rel-L2 0.160 / 0.118, bits 0.9975 /
        # 0.9981 (mask / code); bound = observed + ~25%
        assert rel <= 0.20, rel
        assert agree >= 0.99, agree


def test_forward_fp16_within_conditioning_band(net_and_state, golden):
    """fp16 (configs[4] dtype): as bf16 but with an 11-bit mantissa, so a tighter band."""
    net, _ = net_and_state
    net.set_precision("fp16")
    f = golden("r34_fwd64.npz")
    with torch.no_grad():
        m, c = net(torch.from_numpy(f["fwd64_x"]).cuda())
    net.set_precision("fp32")
    for got, ref in ((m.cpu().numpy(), f["fwd64_mask"]), (c.cpu().numpy(), f["fwd64_code"])):
        assert np.isfinite(got).all()
        rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
        print(f"fp16 rel-L2 {rel:.4g}")
        assert rel <= 0.06, rel
        out = np.abs(ref) > 0.25
        agree = ((got > THR) == (ref > THR))[out].mean()
        assert agree >= 0.97, agree


def test_r50_forward_fp16_within_band(golden):
    """configs[4] network: ResNet50_OS8 + ASPP_50 in fp16 against the reference's 64x64 forward."""
    from oracle import ref_cpu
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    f = golden("r50_fwd64.npz")
    sd = ref_cpu.synthetic_state(50, 16, 0, dict(golden("r50_bn_buffers.npz")))
    net = BinaryCodeNet_Deeplab(50, 16, 2, concat=True, output_kernel_size=1, precision="fp16")
    net.load_state_dict(sd)
    net = net.cuda().eval()
    with torch.no_grad():
        m, c = net(torch.from_numpy(f["fwd64_x"]).cuda())
    for got, ref in ((m.cpu().numpy(), f["fwd64_mask"]), (c.cpu().numpy(), f["fwd64_code"])):
        assert np.isfinite(got).all()
        rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
        print(f"r50 fp16 rel-L2 {rel:.4g}")
        assert rel <= 0.06, rel
        out = np.abs(ref) > 0.25
        agree = ((got > THR) == (ref > THR))[out].mean()
        assert agree >= 0.97, agree
    net.train()
    with pytest.raises(RuntimeError, match="inference-only"):
        net(torch.from_numpy(f["fwd64_x"]).cuda())
    del net
    torch.cuda.empty_cache()


def test_decode_matches_reference_exactly(golden):
    from zebrapose_amd.decode import Decoder
    d = golden("decode.npz")
    ml = torch.from_numpy(d["mask_logits"]).cuda()
    cl = torch.from_numpy(d["code_logits"]).cuda()
    for ib in (0, 2):
        dec = Decoder(d["lut"], device="cuda", ignore_bit=ib)
        if ib:
            np.testing.assert_array_equal(dec.lut[0].cpu().numpy(), d["lut_ib2"].astype(np.float32))
        counts, xy, xyz, ids = dec(ml, cl, d["bboxes"], bbox_size=128, return_ids=True)
        res = Decoder.to_host(counts, xy, xyz)
        for b, (p2d, p3d) in enumerate(res):
            assert len(p2d) == int(d[f"ib{ib}_b{b}_count"])
            np.testing.assert_array_equal(ids[b].cpu().numpy(), d[f"ib{ib}_b{b}_ids"])
            np.testing.assert_array_equal(p2d, d[f"ib{ib}_b{b}_p2d"])
            np.testing.assert_array_equal(p3d, d[f"ib{ib}_b{b}_p3d"])


def test_decode_edge_cases():
    """empty masks, all-NaN LUT rows, odd sizes (ragged last tile), several objects per batch."""
    from zebrapose_amd.decode import Decoder
    from oracle import ref_cpu
    rng = np.random.default_rng(3)
    lutA = rng.standard_normal((65536, 3)) * 10
    lutB = rng.standard_normal((65536, 3)) * 10
    lutB[::3] = np.nan
    B, H, W = 3, 37, 29
    ml = rng.standard_normal((B, 1, H, W)).astype(np.float32)
    ml[1] = -1.0  # empty crop
    cl = rng.standard_normal((B, 16, H, W)).astype(np.float32)
    bb = np.array([[0, 0, 37, 37], [5, 5, 64, 64], [-100, 50, 300, 250]])
    dec = Decoder([lutA, lutB], device="cuda")
    counts, xy, xyz = dec(torch.from_numpy(ml).cuda(), torch.from_numpy(cl).cuda(), bb, bbox_size=H,
                          lut_index=[0, 1, 1])
    res = Decoder.to_host(counts, xy, xyz)
    for b, lut in enumerate([lutA, lutB, lutB]):
        n, p2d, p3d, _ = ref_cpu.decode_crop(ml[b, 0], cl[b], lut, bb[b], bbox_size=H)
        assert len(res[b][0]) == n
        np.testing.assert_array_equal(res[b][0], p2d)
        np.testing.assert_array_equal(res[b][1], p3d)


def test_threshold_matches_cpu_sigmoid_rule(golden):
    from zebrapose_amd import common_ops
    d = golden("decode.npz")
    got = common_ops.from_output_to_class_mask(torch.from_numpy(d["mask_logits"]).cuda())
    assert got.dtype == np.float64
    np.testing.assert_array_equal(got.astype(np.uint8), d["mask_bits"])
    got = common_ops.from_output_to_class_binary_code(torch.from_numpy(d["code_logits"]).cuda(), "BCE")
    np.testing.assert_array_equal(got.astype(np.uint8), d["code_bits"])


def test_losses_match_oracle_on_identical_logits(golden):
    """BinaryCodeLoss / MaskLoss kernels on the reference's own logits (no network in between)."""
    from oracle import ref_cpu
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeLoss, MaskLoss
    f = golden("r34_train_step.npz")
    code = torch.from_numpy(f["code_logits"]).cuda().requires_grad_(True)
    mask = torch.from_numpy(f["mask_logits"]).cuda().requires_grad_(True)
    gt = torch.from_numpy(f["gt_code"]).cuda()
    gm = torch.from_numpy(f["gt_mask"]).cuda()
    bcl, ml = BinaryCodeLoss("BCE", True, 2, True), MaskLoss()
    mask01 = torch.from_numpy(f["mask01"]).cuda()
    lb = bcl(code, mask01, gt)
    lm = ml(mask, gm)
    assert lb.dtype == torch.float64 and lm.dtype == torch.float32
    np.testing.assert_allclose(lb.item(), float(f["loss_b"]), rtol=1e-12)
    np.testing.assert_allclose(lm.item(), float(f["loss_m"]), rtol=1e-6)
    np.testing.assert_allclose(bcl.histogram.cpu().numpy(), f["hist1"], atol=1e-15)
    (3 * lb + lm).backward()
    # oracle gradients of the same expression
    c2 = torch.from_numpy(f["code_logits"]).requires_grad_(True)
    m2 = torch.from_numpy(f["mask_logits"]).requires_grad_(True)
    st = ref_cpu.HistLossState()
    lb2 = ref_cpu.binary_code_loss(st, c2, torch.from_numpy(f["mask01"]), torch.from_numpy(f["gt_code"]))
    lm2 = ref_cpu.mask_loss(m2, torch.from_numpy(f["gt_mask"]))
    (3 * lb2 + lm2).backward()
    np.testing.assert_allclose(code.grad.cpu().numpy(), c2.grad.numpy(), rtol=1e-5, atol=1e-12)
    np.testing.assert_allclose(mask.grad.cpu().numpy(), m2.grad.numpy(), rtol=1e-4, atol=1e-10)
    # second call: histogram EMA
    lb3 = bcl(code.detach(), mask01, torch.from_numpy(f["gt_code2"]).cuda())
    np.testing.assert_allclose(bcl.histogram.cpu().numpy(), f["hist2"], atol=1e-15)
    np.testing.assert_allclose(lb3.item(), float(f["loss_b2"]), rtol=1e-12)
    # device-threshold path (train step without the host round trip) gives the same loss
    bcl2 = BinaryCodeLoss("BCE", True, 2, True)
    lb4 = bcl2.forward_from_logits(code.detach(), mask.detach(), gt.to(torch.uint8))
    np.testing.assert_allclose(lb4.item(), float(f["loss_b"]), rtol=1e-12)


def test_train_step_fp32_matches_reference(net_and_state, golden):
    """One train_v6.py step in fp32: logits, loss, histogram, BN running stats, gradients.  The
    synthetic model amplifies fp32 reassociation noise (oracle: a 1e-6 relative input perturbation
    moves decoder gradients by ~1% and encoder gradients by ~3% rel-L2), so gradients are checked
    in relative L2 with that budget."""
    from oracle import ref_cpu
    from zebrapose_amd import common_ops
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab, BinaryCodeLoss, MaskLoss
    _, sd = net_and_state
    f = golden("r34_train_step.npz")
    net = BinaryCodeNet_Deeplab(34, 16, 2, True, 1, precision="fp32")
    net.load_state_dict(sd)
    net = net.cuda().train()
    pm, pc = net(torch.from_numpy(f["x"]).cuda())
    np.testing.assert_allclose(pm.detach().cpu().numpy(), f["mask_logits"], atol=3e-3)
    np.testing.assert_allclose(pc.detach().cpu().numpy(), f["code_logits"], atol=3e-3)
    mask01 = torch.tensor(common_ops.from_output_to_class_mask(pm)).cuda()
    bcl, ml = BinaryCodeLoss("BCE", True, 2, True), MaskLoss()
    lb = bcl(pc, mask01, torch.from_numpy(f["gt_code"]).cuda())
    lm = ml(pm, torch.from_numpy(f["gt_mask"]).cuda())
    np.testing.assert_allclose(lb.item(), float(f["loss_b"]), rtol=1e-4)
    np.testing.assert_allclose(lm.item(), float(f["loss_m"]), rtol=1e-4)
    (3 * lb + lm).backward()
    named = dict(net.named_parameters())
    for k in f:
        if k.startswith("grad:"):
            name = k[5:]
            got = named[name].grad.cpu().numpy()[:8]
            ref = f[k]
            rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
            # the random-weight model's own noise floor: a 1e-6 relative input perturbation moves
            # these gradients by 1-3% rel-L2 in the oracle
            budget = 0.01 if "aspp.conv_1x1_4" in name else 0.05
            assert rel <= budget, (name, rel)
    sd2 = net.state_dict()
    for k in f:
        if k.startswith("after:"):
            np.testing.assert_allclose(sd2[k[6:]].cpu().numpy(), f[k], rtol=1e-3, atol=1e-4)


def test_fused_adam_matches_torch():
    from zebrapose_amd.optim import FusedAdam
    torch.manual_seed(0)
    p_ref = torch.randn(1000, dtype=torch.float32, requires_grad=True)
    p = p_ref.detach().clone().cuda().requires_grad_(True)
    o_ref = torch.optim.Adam([p_ref], lr=4e-4)
    o = FusedAdam([p], lr=4e-4)
    for s in range(5):
        g = torch.randn(1000) * (s + 1)
        p_ref.grad = g.clone()
        p.grad = g.cuda()
        o_ref.step()
        o.step()
    torch.cuda.synchronize()
    np.testing.assert_allclose(p.detach().cpu().numpy(), p_ref.detach().numpy(), rtol=1e-5, atol=1e-7)
    st = o.state_dict()["state"][0]
    np.testing.assert_allclose(st["exp_avg"].cpu().numpy(), o_ref.state_dict()["state"][0]["exp_avg"].numpy(),
                               rtol=1e-5, atol=1e-7)


def test_fused_adam_multi_tensor_matches_torch():
    """45 tensors (two zp_adam_multi launches), sizes around the 4096-element block chunk,
    one tensor without a gradient; same op order as torch's single-tensor Adam."""
    from zebrapose_amd.optim import FusedAdam
    torch.manual_seed(1)
    sizes = [1, 7, 4095, 4096, 4097, 12289, 65536 + 3] * 6 + [300, 2, 9]
    ref = [torch.randn(n, dtype=torch.float32, requires_grad=True) for n in sizes]
    dev = [r.detach().clone().cuda().requires_grad_(True) for r in ref]
    o_ref = torch.optim.Adam(ref, lr=3e-4)
    o = FusedAdam(dev, lr=3e-4)
    for s in range(3):
        for i, (r, d) in enumerate(zip(ref, dev)):
            if i == 5:
                r.grad, d.grad = None, None
                continue
            g = torch.randn(r.shape) * (s + 1)
            r.grad = g.clone()
            d.grad = g.cuda()
        o_ref.step()
        o.step()
        if s == 1:  # checkpoint round trip mid-run (utils_v2 saves optimizer_state_dict)
            sd = o.state_dict()
            o = FusedAdam(dev, lr=3e-4)
            o.load_state_dict(sd)
    torch.cuda.synchronize()
    assert float(o.state_dict()["state"][0]["step"]) == 3.0
    for r, d in zip(ref, dev):
        np.testing.assert_allclose(d.detach().cpu().numpy(), r.detach().numpy(), rtol=1e-6, atol=1e-8)


@pytest.mark.parametrize("capturable", [False, True])
def test_fused_adam_intermittent_none_grad(capturable):
    """a parameter whose gradient is None at step 2 only (present at 1, 3, 4, 5).  Step 1
    builds the cached launch plan, step 2 takes the general path (advancing all but one tensor),
    steps 3.. must not reuse a plan that assumes one shared step count: bias correction per tensor
    as torch.optim.Adam, and the saved 'step' state per tensor."""
    from zebrapose_amd.optim import FusedAdam
    torch.manual_seed(4)
    sizes = [17, 4096, 5, 300]
    ref = [torch.randn(n, dtype=torch.float32, requires_grad=True) for n in sizes]
    dev = [r.detach().clone().cuda().requires_grad_(True) for r in ref]
    o_ref = torch.optim.Adam(ref, lr=1e-2)
    o = FusedAdam(dev, lr=1e-2, capturable=capturable)
    for s in range(5):
        for i, (r, d) in enumerate(zip(ref, dev)):
            if i == 1 and s == 1:
                r.grad, d.grad = None, None
                continue
            g = torch.randn(r.shape) * (s + 1)
            r.grad = g.clone()
            d.grad = g.cuda()
        o_ref.step()
        o.step()
    torch.cuda.synchronize()
    sd, sd_ref = o.state_dict()["state"], o_ref.state_dict()["state"]
    for i in range(len(sizes)):
        assert float(sd[i]["step"]) == float(sd_ref[i]["step"]), i
    assert float(sd[1]["step"]) == 4.0 and float(sd[0]["step"]) == 5.0
    for r, d in zip(ref, dev):
        np.testing.assert_allclose(d.detach().cpu().numpy(), r.detach().numpy(), rtol=1e-6, atol=1e-8)


def test_binary_code_helper_dropins(golden):
    """Reference-signature helpers (host arrays in/out, device decode inside)."""
    from zebrapose_amd.binary_code_helper.CNN_output_to_pose import decode_correspondences
    from zebrapose_amd.binary_code_helper.generate_new_dict import generate_new_corres_dict
    d = dict(golden("decode.npz"))  # materialise once: NpzFile re-reads the member on every access
    lut = d["lut"]
    lut_dict = {float(i): lut[i] for i in range(lut.shape[0])}
    for ib in (0, 2):
        dd = lut_dict if ib == 0 else generate_new_corres_dict(lut_dict, 16, 16 - ib)
        if ib:
            got = np.stack([dd[i].reshape(3) for i in range(2 ** 14)])
            np.testing.assert_array_equal(got.astype(np.float32), d["lut_ib2"].astype(np.float32))
            dd = {float(k): v for k, v in dd.items()}
        for b in range(2):
            mask = d["mask_bits"][b, 0]
            code = d["code_bits"][b].transpose(1, 2, 0)
            if ib:
                code = code[:, :, :-ib]
            p2d, p3d = decode_correspondences(mask, code, d["bboxes"][b], 128, dd)
            np.testing.assert_array_equal(p2d, d[f"ib{ib}_b{b}_p2d"])
            np.testing.assert_array_equal(p3d, d[f"ib{ib}_b{b}_p3d"])


def test_decoder_cache_tracks_dict_identity_and_content():
    """CNN_output_to_pose's LUT cache: a new dict (even if it reused a collected dict's id) or an edited
    entry must not decode with a stale LUT; the cache stays bounded."""
    from zebrapose_amd.binary_code_helper import CNN_output_to_pose as C
    mask = np.ones((4, 4), np.uint8)
    code = np.zeros((4, 4, 16))  # every pixel -> class id 0
    bb = np.array([0, 0, 128, 128])

    def mk(v):
        return {float(i): np.array([v, v, v], np.float64) for i in range(65536)}
    d1 = mk(1.0)
    _, p3 = C.decode_correspondences(mask, code, bb, 128, d1)
    assert np.all(p3 == 1.0)
    d1[0.0] = np.array([5.0, 5.0, 5.0])  # edit in place: the sampled fingerprint sees id 0
    _, p3 = C.decode_correspondences(mask, code, bb, 128, d1)
    assert np.all(p3 == 5.0)
    for k in range(40):  # many dicts: new ids, some recycled; never stale, cache bounded
        d = mk(float(k))
        _, p3 = C.decode_correspondences(mask, code, bb, 128, d)
        assert np.all(p3 == float(k))
        del d
    assert len(C._DEC_CACHE) <= C._DEC_CACHE_MAX


def test_fused_adam_multi_with_empty_tensors_inside_a_chunk():
    """zp_adam_multi packs up to 40 non-empty tensors per launch; empty tensors inside a chunk of 41+
    tensors must not make the next launch revisit (and double-update) a tensor."""
    from zebrapose_amd.optim import FusedAdam
    torch.manual_seed(3)
    sizes = [5, 0, 33, 0, 0, 7] * 9 + [11, 0, 2]
    ref = [torch.randn(n, dtype=torch.float32, requires_grad=True) for n in sizes]
    dev = [r.detach().clone().cuda().requires_grad_(True) for r in ref]
    o_ref = torch.optim.Adam(ref, lr=1e-2)
    o = FusedAdam(dev, lr=1e-2)
    for s in range(2):
        for r, d in zip(ref, dev):
            g = torch.randn(r.shape)
            r.grad = g.clone()
            d.grad = g.cuda()
        o_ref.step()
        o.step()
    torch.cuda.synchronize()
    for r, d in zip(ref, dev):
        np.testing.assert_allclose(d.detach().cpu().numpy(), r.detach().numpy(), rtol=1e-6, atol=1e-8)
