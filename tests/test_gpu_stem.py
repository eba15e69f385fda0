"""The two-plane stem (zp_stem_split, csrc/zp_stem.hip; reference model/resnet.py:195, torchvision
conv1 7x7 / stride 2 / pad 3, 3 -> 64, + BN + ReLU): one launch from the f32 image, persistent over
256-pixel tiles with the next tile's input region prefetched.  It reads either the NHWC copy
(zp_nchw_to_nhwc, the traced path) or -- ldx 0, the default eval path -- the reference's NCHW input
tensor directly; both must store the same bits, and both must be f32-accurate against a float64
conv (the two-plane storage bound of tests/test_gpu_x3.py: 2^-21 of the output scale plus the
exact-f32 product error).  Geometries: 64x64 (one tile per image), 128x128 and bs=33 at 256x256
(2112 tiles: more tiles than workgroups, a ragged last round)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,H", [(2, 64), (5, 128), (33, 256)])
def test_stem_nchw_equals_nhwc_and_is_f32_accurate(gpu, B, H):
    from zebrapose_amd import _lib as L
    from zebrapose_amd.engine import Act, Engine, NchwInput, Unit, joined
    from zebrapose_amd.model import layers as LY
    torch.manual_seed(9)
    conv = LY.Conv2d(3, 64, 7, 2, 3, 1, bias=False)
    bn = LY.BatchNorm2d(64)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_(0, 0.1)
        bn.running_mean.normal_(0, 0.1)
        bn.running_var.uniform_(0.5, 1.5)
    conv, bn = conv.to(gpu).eval(), bn.to(gpu).eval()
    unit = Unit(conv, bn, relu=True, cin_act=8)
    x = torch.randn(B, 3, H, H, device=gpu)
    eng = Engine(torch.nn.Module(), torch.float32, split="h2")
    OH = H // 2
    outs = {}
    for form in ("nchw", "nhwc"):
        if form == "nchw":
            xa = NchwInput(x.permute(0, 2, 3, 1), 0, 8)
        else:
            xin = torch.zeros(B, H, H, 8, device=gpu)
            L.call("zp_nchw_to_nhwc", x.data_ptr(), B, 3, H, H, 8, L.ZP_F32, xin.data_ptr(), L.stream_ptr())
            xa = Act(xin)
        oa = Act(eng._empty((B, OH, OH, 64), gpu))
        eng.stage_log = []
        eng.unit_fwd(unit, xa, oa, None)
        torch.cuda.synchronize()
        assert [r[1] for r in eng.stage_log] == ["k_stem_h2"], eng.stage_log
        outs[form] = oa.buf._base.clone()
    assert torch.equal(outs["nchw"], outs["nhwc"])
    got = joined(outs["nchw"][0]).permute(0, 3, 1, 2).double().cpu()
    w = conv.weight.detach().double().cpu()
    g, b, m, v = (t.detach().double().cpu() for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var))
    ref = F.conv2d(x.double().cpu(), w, None, 2, 3)
    ref = F.relu((ref - m.view(1, -1, 1, 1)) / torch.sqrt(v.view(1, -1, 1, 1) + 1e-5) * g.view(1, -1, 1, 1) + b.view(1, -1, 1, 1))
    f32 = F.relu(F.conv2d(x.cpu(), conv.weight.detach().cpu(), None, 2, 3).double()
                 .sub(m.view(1, -1, 1, 1)).div(torch.sqrt(v.view(1, -1, 1, 1) + 1e-5)).mul(g.view(1, -1, 1, 1)).add(b.view(1, -1, 1, 1)))
    scale = float(ref.abs().max())
    e, ef = float((got - ref).abs().max()), float((f32 - ref).abs().max())
    print(f"stem B={B} {H}x{H}: max |d| two-plane {e:.3g}, CPU f32 conv {ef:.3g} (scale {scale:.3g})")
    assert e <= 4.0 * ef + 2.0 ** -21 * scale, (e, ef, scale)


@pytest.mark.parametrize("knob", ["split_stem", "stem_direct"])
def test_stem_knobs_keep_fp32_eval_working(gpu, golden, knob):
    """nchw_stem (the NCHW input handed to the stem) and unit_fwd's zp_stem_split branch
    share one predicate.  With ZP_SPLIT_STEM=0 (the exact-f32 small-Cin stem) or ZP_STEM_DIRECT=0 (the
    im2col stem) the fp32 eval forward must still run -- from the NHWC copy -- and stay within the
    north star's 1e-3 of the default two-plane forward and of the reference's logits at 64x64."""
    from oracle import ref_cpu
    from zebrapose_amd import _lib as L
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    bn = dict(golden("r34_bn_buffers.npz"))
    sd = ref_cpu.synthetic_state(34, 16, 0, bn)
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="fp32")
    net.load_state_dict(sd)
    net = net.cuda().eval()
    f = golden("r34_fwd64.npz")
    x = torch.from_numpy(f["fwd64_x"]).cuda()
    with torch.no_grad():
        m0, c0 = (t.clone() for t in net(x))
        eng = net.net.eval_engine()
        assert eng.dt == L.ZP_F32H2
        setattr(eng, knob, False)
        m1, c1 = net(x)
    torch.cuda.synchronize()
    for a, b, ref in ((m0, m1, f["fwd64_mask"]), (c0, c1, f["fwd64_code"])):
        assert torch.isfinite(b).all()
        assert float((a - b).abs().max()) <= 1e-3, float((a - b).abs().max())
        # and the reference's own logits (the fixture), as tests/test_gpu_parity.py holds the default
        r = torch.from_numpy(ref).cuda()
        assert float(((b - r).abs() - 1e-4 * r.abs()).max()) <= 1e-3
