"""The oracle (oracle/ref_cpu.py) pinned against golden vectors captured from the real reference
(oracle/capture_fixtures.py imports /root/reference/zebrapose and runs it on CPU)."""
import numpy as np
import pytest
import torch

from oracle import ref_cpu


@pytest.fixture(scope="module")
def state(golden):
    bn = dict(golden("r34_bn_buffers.npz"))
    return lambda: ref_cpu.synthetic_state(34, 16, 0, bn)


def test_state_spec_matches_reference_keys(golden):
    import os
    from tests.conftest import GOLDEN
    want = open(os.path.join(GOLDEN, "state_keys_r34.txt")).read().splitlines()
    entries, aliases = ref_cpu.state_spec(34, 16)
    got = [f"{k} {list(s)}" for k, s, _ in entries]
    assert got == want
    assert len(aliases) == 96


def test_forward64_matches_reference(golden, state):
    f = golden("r34_fwd64.npz")
    with torch.no_grad():
        m, c = ref_cpu.forward(state(), torch.from_numpy(f["fwd64_x"]), 34)
    np.testing.assert_allclose(m.numpy(), f["fwd64_mask"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(c.numpy(), f["fwd64_code"], atol=1e-5, rtol=0)


def test_forward256_matches_reference(golden):
    """256x256, B=2, BN calibrated at 256x256 by the reference itself (capture_fwd256)."""
    f = golden("r34_fwd256.npz")
    sd = ref_cpu.synthetic_state(34, 16, 0, dict(golden("r34_bn_buffers256.npz")))
    with torch.no_grad():
        m, c = ref_cpu.forward(sd, torch.from_numpy(f["x"]), 34)
    np.testing.assert_allclose(m.numpy(), f["mask"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(c.numpy(), f["code"], atol=1e-5, rtol=0)


def test_forward_lowp_is_the_fp32_forward_plus_storage_rounding(golden):
    """forward_lowp restates forward with 16-bit storage: with an identity 'rounding' (f32) it must
    reproduce forward, and in bf16 / fp16 it must land in the conditioning band measured for this
    model (bf16 18.6% / fp16 3.0% rel-L2 at 256x256)."""
    f = golden("r34_fwd256.npz")
    sd = ref_cpu.synthetic_state(34, 16, 0, dict(golden("r34_bn_buffers256.npz")))
    x = torch.from_numpy(f["x"][:1])
    with torch.no_grad():
        m32, c32 = ref_cpu.forward_lowp(sd, x, 34, torch.float32)
        mb, cb = ref_cpu.forward_lowp(sd, x, 34, torch.bfloat16)
        mh, ch = ref_cpu.forward_lowp(sd, x, 34, torch.float16)
    np.testing.assert_allclose(c32.numpy(), f["code"][:1], atol=2e-4, rtol=0)
    np.testing.assert_allclose(m32.numpy(), f["mask"][:1], atol=2e-4, rtol=0)
    ref = f["code"][:1]
    for got, lo, hi in ((cb, 0.05, 0.30), (ch, 0.005, 0.06)):
        rel = np.linalg.norm(got.numpy() - ref) / np.linalg.norm(ref)
        assert lo <= rel <= hi, rel
    # stored activations are representable: every lp_conv output is exactly a bf16 value
    y = ref_cpu.lp_conv(x, sd["net.resnet.resnet.0.weight"], None, None, None, True, 2, 3)
    assert torch.equal(y, y.to(torch.bfloat16).float())


def test_gt_codes_oracle_matches_reference(golden):
    """A15: the reference's RGB_image_to_class_id_image + class_id_image_to_class_code_images
    (class_id_encoder_decoder.py:6-15, 43-63) vs oracle/crop_ref.crop_gt on 128x128 crops (a
    same-size square ROI: nearest resize is the identity, so only the colour -> code planes remain)."""
    from oracle import crop_ref
    f = golden("gt_codes.npz")
    for b in range(f["gt_bgr"].shape[0]):
        g = f["gt_bgr"][b]
        m = np.zeros(g.shape[:2], np.uint8)
        code, _, _ = crop_ref.crop_gt(g, m, m, np.array([0, 0, 128, 128]))
        np.testing.assert_array_equal(code, f["code"][b])


def test_add_adi_restatement_matches_reference(golden):
    """ADD / ADI (lib/pysixd/pose_error.py:297-336) restated in numpy / scipy against the values the
    reference's own functions returned (capture_add_adi)."""
    from scipy import spatial
    f = golden("add_adi.npz")
    pts = f["pts"].astype(np.float64)
    for b in range(f["add"].shape[0]):
        pe = (f["R_est"][b] @ pts.T + f["t_est"][b][:, None]).T
        pg = (f["R_gt"][b] @ pts.T + f["t_gt"][b][:, None]).T
        np.testing.assert_allclose(np.linalg.norm(pe - pg, axis=1).mean(), f["add"][b], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(spatial.cKDTree(pe).query(pg, k=1)[0].mean(), f["adi"][b], rtol=1e-12,
                                   atol=1e-12)


def test_train_step_matches_reference(golden, state):
    f = golden("r34_train_step.npz")
    sd = state()
    entries, aliases = ref_cpu.state_spec(34, 16)
    leaves = {}
    for k, s, kind in entries:
        if k in aliases or kind in ("bn_rm", "bn_rv", "bn_nbt"):
            continue
        sd[k].requires_grad_(True)
        leaves[k] = sd[k]
    for ak, ck in aliases.items():
        sd[ak] = sd[ck]
    x = torch.from_numpy(f["x"])
    m, c = ref_cpu.forward(sd, x, 34, train=True)
    np.testing.assert_allclose(m.detach().numpy(), f["mask_logits"], atol=1e-5)
    np.testing.assert_allclose(c.detach().numpy(), f["code_logits"], atol=1e-5)
    st = ref_cpu.HistLossState()
    loss, lb, lm = ref_cpu.train_step_loss(st, m, c, torch.from_numpy(f["gt_code"]), torch.from_numpy(f["gt_mask"]))
    assert lb.dtype == torch.float64
    np.testing.assert_allclose(lb.item(), float(f["loss_b"]), rtol=1e-9)
    np.testing.assert_allclose(lm.item(), float(f["loss_m"]), rtol=1e-6)
    np.testing.assert_allclose(st.histogram.numpy(), f["hist1"], rtol=0, atol=1e-12)
    loss.backward()
    for k in f:
        if k.startswith("grad:"):
            name = k[5:]
            g = leaves[name].grad.numpy()[:8]
            np.testing.assert_allclose(g, f[k], atol=1e-5 * max(1e-3, np.abs(f[k]).max()) + 1e-9, rtol=1e-3)
    for k in f:
        if k.startswith("after:"):
            np.testing.assert_allclose(sd[k[6:]].detach().numpy(), f[k], rtol=1e-5, atol=1e-7)
    # second BinaryCodeLoss call: histogram EMA (BinaryCodeNet.py:37-41)
    mask01 = torch.from_numpy(ref_cpu.threshold_np(m.detach().numpy()))
    lb2 = ref_cpu.binary_code_loss(st, c.detach(), mask01, torch.from_numpy(f["gt_code2"]))
    np.testing.assert_allclose(st.histogram.numpy(), f["hist2"], atol=1e-12)
    np.testing.assert_allclose(lb2.item(), float(f["loss_b2"]), rtol=1e-9)


def test_threshold_boundary_matches_reference(golden):
    d = golden("decode.npz")
    assert np.array_equal(ref_cpu.threshold_np(d["mask_logits"]).astype(np.uint8), d["mask_bits"])
    assert np.array_equal(ref_cpu.threshold_np(d["code_logits"]).astype(np.uint8), d["code_bits"])
    probe = np.array([8.940696716308594e-08, 8.94069742685133e-08, 0.0, -1e-8, np.nan], np.float32)
    assert ref_cpu.threshold_np(probe).tolist() == [0.0, 1.0, 0.0, 0.0, 0.0]


@pytest.mark.parametrize("ignore_bit", [0, 2])
def test_decode_matches_reference(golden, ignore_bit):
    d = golden("decode.npz")
    lut = d["lut"] if ignore_bit == 0 else ref_cpu.coarse_lut(d["lut"], 16, 16 - ignore_bit)
    if ignore_bit:
        np.testing.assert_array_equal(lut, d[f"lut_ib{ignore_bit}"])
    for b in range(d["mask_logits"].shape[0]):
        n, p2d, p3d, ids = ref_cpu.decode_crop(d["mask_logits"][b, 0], d["code_logits"][b], lut, d["bboxes"][b],
                                               ignore_bit=ignore_bit)
        assert n == int(d[f"ib{ignore_bit}_b{b}_count"])
        assert np.array_equal(ids, d[f"ib{ignore_bit}_b{b}_ids"])
        assert np.array_equal(p2d, d[f"ib{ignore_bit}_b{b}_p2d"])
        assert np.array_equal(p3d, d[f"ib{ignore_bit}_b{b}_p3d"])


def test_r50_state_spec_and_forward_match_reference(golden):
    """ResNet50_OS8 + ASPP_50 variant (resnet.py:206-227, aspp.py:117-225):
    key layout (488 keys, 144 aliases) and 64x64 forward against the captured reference."""
    import os
    from tests.conftest import GOLDEN
    want = open(os.path.join(GOLDEN, "state_keys_r50.txt")).read().splitlines()
    entries, aliases = ref_cpu.state_spec(50, 16)
    assert [f"{k} {list(s)}" for k, s, _ in entries] == want
    assert len(aliases) == 144
    f = golden("r50_fwd64.npz")
    sd = ref_cpu.synthetic_state(50, 16, 0, dict(golden("r50_bn_buffers.npz")))
    with torch.no_grad():
        m, c = ref_cpu.forward(sd, torch.from_numpy(f["fwd64_x"]), 50)
    np.testing.assert_allclose(m.numpy(), f["fwd64_mask"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(c.numpy(), f["fwd64_code"], atol=1e-5, rtol=0)


def test_r50_forward256_matches_reference(golden):
    """configs[4]'s network at its own 256x256 geometry (BN calibrated at 256x256 by the reference,
    oracle/capture_fixtures.py capture_r50_256): the oracle's R50 forward equals the reference's."""
    f = golden("r50_fwd256.npz")
    sd = ref_cpu.synthetic_state(50, 16, 0, dict(golden("r50_bn256_s0.npz")))
    with torch.no_grad():
        m, c = ref_cpu.forward(sd, torch.from_numpy(f["x"]), 50)
    np.testing.assert_allclose(m.numpy(), f["mask"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(c.numpy(), f["code"], atol=1e-5, rtol=0)


def test_v3_state_spec_and_forward_match_reference(golden):
    """BinaryCodeNet_Deeplab_v3: key layout and the 256x256 three-head forward
    of the oracle against the reference's own outputs (oracle/capture_fixtures.py capture_v3)."""
    import os
    from oracle import tv_layout
    from tests.conftest import GOLDEN
    entries, _ = tv_layout.state_spec("v3", 16)
    want = open(os.path.join(GOLDEN, "state_keys_r34v3.txt")).read().splitlines()
    assert [f"{k} {list(s)}" for k, s, _ in entries] == want
    f = golden("r34v3_fwd256.npz")
    sd = ref_cpu.synthetic_state("v3", 16, 0, dict(golden("r34v3_bn_buffers.npz")))
    with torch.no_grad():
        m, e, c = ref_cpu.forward_v3(sd, torch.from_numpy(f["x"]))
    np.testing.assert_array_equal(m.numpy(), f["mask"])
    np.testing.assert_array_equal(e.numpy(), f["entire"])
    np.testing.assert_array_equal(c.numpy(), f["code"])


def test_decode_loop_form_equals_vectorised(golden):
    """The CPU baseline's loop-form decode (the reference's per-pixel loop) gives the same outputs
    as the vectorised oracle and the reference fixture."""
    d = golden("decode.npz")
    ld = ref_cpu.lut_dict(d["lut"])
    for b in range(d["mask_logits"].shape[0]):
        n, p2d, p3d = ref_cpu.decode_crop_loop(d["mask_logits"][b, 0], d["code_logits"][b], ld, d["bboxes"][b])
        assert n == int(d[f"ib0_b{b}_count"])
        assert np.array_equal(p2d, d[f"ib0_b{b}_p2d"])
        assert np.array_equal(p3d, d[f"ib0_b{b}_p3d"])
