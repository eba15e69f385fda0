"""BinaryCodeNet_Deeplab_v3 (train_v5.py's network) through the HIP path
against the reference's own outputs (tests/golden/r34v3_*, oracle/capture_fixtures.py capture_v3):
the three-head forward in fp32 (and bf16 in the conditioning band, as for the main network) and
one fp32 training step (3 * loss_b + loss_mask + loss_entire_mask): losses, and gradients of the
v3 head, of the main head (which receives the entire-mask loss through the resampled mask
inputs) and of the shared encoder, with the budgets of test_gpu_parity.py."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
THR = np.float32(8.940696716308594e-08)


@pytest.fixture(scope="module")
def v3(golden):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import ref_cpu
    from zebrapose_amd.model.BinaryCodeNet_v3 import BinaryCodeNet_Deeplab_v3
    sd = ref_cpu.synthetic_state("v3", 16, 0, dict(golden("r34v3_bn_buffers.npz")))
    net = BinaryCodeNet_Deeplab_v3(34, 16, 2, concat=True, output_kernel_size=1, precision="fp32")
    net.load_state_dict(sd)
    return net.cuda().eval()


def test_v3_forward_fp32_matches_reference(v3, golden):
    f = golden("r34v3_fwd256.npz")
    v3.set_precision("fp32")
    with torch.no_grad():
        m, e, c = v3(torch.from_numpy(f["x"]).cuda())
    for got, key in ((m, "mask"), (e, "entire"), (c, "code")):
        ref = f[key]
        got = got.cpu().numpy()
        scale = np.abs(ref).max()
        err = np.abs(got - ref).max()
        print(f"v3 {key}: max|d| {err:.3g} scale {scale:.3g}")
        assert err <= 2e-3 + 1e-5 * scale, (key, err, scale)


def test_v3_forward_bf16_within_band(v3, golden):
    f = golden("r34v3_fwd256.npz")
    v3.set_precision("bf16")
    try:
        with torch.no_grad():
            m, e, c = v3(torch.from_numpy(f["x"]).cuda())
    finally:
        v3.set_precision("fp32")
    for got, key in ((m, "mask"), (e, "entire"), (c, "code")):
        ref = f[key]
        got = got.cpu().numpy()
        rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
        agree = ((got > THR) == (ref > THR))[np.abs(ref) > 0.25].mean()
        print(f"v3 bf16 {key}: rel-L2 {rel:.3g}, bits agree {agree:.4f} outside |ref| <= 0.25")
        # 256x256 with BN calibrated on two crops conditions worse than the 64x64 main-network
        # fixture (rel-L2 0.16 there); test_main_network_bf16_at_256 below is the main-network analogue
        # observed (r03): rel-L2 0.309 / 0.207 / 0.191, bits 0.944 / 0.970 / 0.969 (mask / entire /
        # code); bound = observed + ~25%
        assert rel <= 0.38 and agree >= 0.93, (key, rel, agree)


def test_main_network_bf16_at_256(golden):
    """The main network in bf16 on the reference's 256x256 fixture (BN calibrated at 256x256):
    in the conditioning band of this model (the bf16-emulating oracle sits at 18.6% rel-L2 from
    fp32; tests/test_gpu_bench_geometry.py checks bf16 teacher-forced layer by layer)."""
    from oracle import ref_cpu
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    f = golden("r34_fwd256.npz")
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="bf16")
    net.load_state_dict(ref_cpu.synthetic_state(34, 16, 0, dict(golden("r34_bn_buffers256.npz"))))
    net = net.cuda().eval()
    with torch.no_grad():
        m, c = net(torch.from_numpy(f["x"]).cuda())
    for got, key in ((m, "mask"), (c, "code")):
        ref = f[key]
        got = got.cpu().numpy()
        rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
        agree = ((got > THR) == (ref > THR))[np.abs(ref) > 0.25].mean()
        print(f"main bf16 @256 {key}: rel-L2 {rel:.3g}, bits agree {agree:.4f} outside |ref| <= 0.25")
        # observed (r03): rel-L2 0.255 / 0.188, bits 0.981 / 0.989 (mask / code); bound = observed + ~25%
        assert rel <= 0.32 and agree >= 0.97, (key, rel, agree)


def test_v3_rejects_other_input_sizes(v3):
    with pytest.raises(ValueError, match="256x256"):
        with torch.no_grad():
            v3(torch.zeros(1, 3, 128, 128, device="cuda"))


def test_v3_train_step_fp32_matches_reference(golden):
    from oracle import ref_cpu
    from zebrapose_amd import common_ops
    from zebrapose_amd.model.BinaryCodeNet_v3 import BinaryCodeLoss, BinaryCodeNet_Deeplab_v3, MaskLoss
    f = golden("r34v3_train_step.npz")
    sd = ref_cpu.synthetic_state("v3", 16, 0, dict(golden("r34v3_bn_buffers.npz")))
    net = BinaryCodeNet_Deeplab_v3(34, 16, 2, True, 1, precision="fp32")
    net.load_state_dict(sd)
    net = net.cuda().train()
    pm, pe, pc = net(torch.from_numpy(f["x"]).cuda())
    for got, key in ((pm, "mask_logits"), (pe, "entire_logits")):
        ref = f[key]
        err = np.abs(got.detach().cpu().numpy() - ref).max()
        assert err <= 3e-3 + 1e-5 * np.abs(ref).max(), (key, err)
    mask01 = torch.tensor(common_ops.from_output_to_class_mask(pm)).cuda()
    bcl, ml = BinaryCodeLoss("BCE", True, 2, True), MaskLoss()
    lb = bcl(pc, mask01, torch.from_numpy(f["gt_code"].astype(np.float64)).cuda())
    lm = ml(pm, torch.from_numpy(f["gt_mask"].astype(np.float32)).cuda())
    le = ml(pe, torch.from_numpy(f["gt_entire"].astype(np.float32)).cuda())
    np.testing.assert_allclose(lb.item(), float(f["loss_b"]), rtol=1e-4)
    np.testing.assert_allclose(lm.item(), float(f["loss_m"]), rtol=1e-4)
    np.testing.assert_allclose(le.item(), float(f["loss_e"]), rtol=1e-4)
    (3 * lb + lm + le).backward()
    named = dict(net.named_parameters())
    for k in f:
        if k.startswith("grad:"):
            name = k[5:]
            got = named[name].grad.cpu().numpy()[:8]
            ref = f[k]
            rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
            budget = 0.01 if name.endswith("conv_1x1_4.weight") or name.endswith("conv_1x1_4.bias") else 0.05
            print(f"v3 grad {name}: rel-L2 {rel:.3g}")
            assert rel <= budget, (name, rel)


def test_v3_bf16_teacher_forced(v3, golden):
    """bf16 v3 forward replayed op by op (as tests/test_gpu_bench_geometry.py does for the main
    network): every conv of the shared encoder / decoder and of the entire-mask head ASPP_v3
    (its concat inputs padded with zero channels) from the device's own stored 16-bit inputs,
    within 1 bf16 ulp (+ 2^-12 of the layer rms), and both f32 heads to accumulation order."""
    from oracle import ref_cpu
    from tests.test_gpu_bench_geometry import replay, _label, _nchw, _ulp_bf16
    f = golden("r34v3_fwd256.npz")
    v3.set_precision("bf16")
    eng = v3.net._engine
    eng.trace = []
    try:
        with torch.no_grad():
            m, e, c = v3(torch.from_numpy(f["x"]).cuda())
        torch.cuda.synchronize()
        trace = eng.trace
    finally:
        eng.trace = None
        v3.set_precision("fp32")
    n_conv = 0
    for i, rec in enumerate(trace):
        if rec[0] == "head" and rec[4] is None and rec[3][1] is None:  # the entire-mask head: f32, one channel
            unit, x, (ent, _) = rec[1], rec[2], rec[3]
            for b in range(ent.shape[0]):
                xin = _nchw(x, b)[:, :unit.cin_w]
                exp = ref_cpu.lp_conv(xin, unit.conv.weight.detach().float().cpu(), None,
                                      unit.conv.bias.detach().float().cpu(), None, False, dt=torch.bfloat16,
                                      out_f32=True)
                got = ent[b:b + 1].cpu()
                assert float((got - exp).abs().max()) <= 2e-5 * max(float(exp.abs().max()), 1.0), _label(rec, i)
            continue
        for b in range(m.shape[0]):
            exp, got = replay(rec, b, torch.bfloat16)
            assert exp.shape == got.shape, (_label(rec, i), exp.shape, got.shape)
            d = (got - exp).abs()
            if rec[0] == "head":
                assert float(d.max()) <= 2e-5 * max(float(exp.abs().max()), 1.0), _label(rec, i)
                continue
            rms = float(exp.pow(2).mean().sqrt())
            bad = d > _ulp_bf16(torch.maximum(exp.abs(), got.abs())) + 2.0 ** -12 * rms
            assert not bool(bad.any()), (_label(rec, i), int(bad.sum()))
            assert float((d > 0).float().mean()) <= 0.005, _label(rec, i)
        n_conv += rec[0] == "conv"
    assert n_conv >= 48 + 9, n_conv  # the main network's 48 + ASPP_v3's convs
