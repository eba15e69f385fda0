"""Weight-gradient kernel (zp_conv2d_wgrad) against torch fp32 on the SAME bf16-rounded operands:
with identical inputs the only difference left is f32 accumulation order, so the bound is tight
(rel L2 <= 2e-3, max |d| <= 1e-2 of the largest entry) -- unlike the network-level bf16 checks.
Covers every geometry class of the R34 backward: stem (Cin 3 padded to 8, 7x7 s2), 3x3 d1/d2/d4,
strided 3x3 and 1x1 downsample, dilated ASPP with most taps in padding, 1x1 head with Cout 17
(dy row pitch 32), transposed-conv phases, and grids large enough for several splits and pixel
rows that wrap across image rows and batch items inside one K step.  Round 6: the lean kernel at
stride 2 (W 32 / 64 / 128 output grids) and the ConvT weight gradient computed as the stride-2 conv
over dy with x as its output gradient (swap) as well as by the four phases."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

GEOMS = [
    # kind, cin(act), cin(weight), cout, k, s, p, d, H, B
    ("conv", 8, 3, 64, 7, 2, 3, 1, 64, 2),
    ("conv", 64, 64, 64, 3, 1, 1, 1, 32, 4),
    ("conv", 64, 64, 128, 3, 2, 1, 1, 32, 2),
    ("conv", 64, 64, 128, 1, 2, 0, 1, 32, 2),
    ("conv", 256, 256, 256, 3, 1, 4, 4, 16, 8),
    ("conv", 512, 512, 256, 3, 1, 18, 18, 16, 4),
    ("conv", 1280, 1280, 256, 1, 1, 0, 1, 8, 4),
    ("conv", 320, 320, 17, 1, 1, 0, 1, 32, 2),
    ("convT", 256, 256, 256, 3, 2, 1, 1, 8, 4),
    ("convT", 320, 320, 256, 3, 2, 1, 1, 16, 2),
    # (round 6) k_wgrad2 at stride 2 (output grid W 32 / 64 / 128), and the ConvT weight gradient as
    # the stride-2 conv over dy (Engine._convT_wgrad_swap) on that kernel: up1's and up2's ConvTs
    ("conv", 64, 64, 128, 3, 2, 1, 1, 64, 2),
    ("conv", 64, 64, 128, 1, 2, 0, 1, 64, 2),
    ("conv", 64, 64, 64, 3, 2, 1, 1, 128, 2),
    ("conv", 64, 64, 64, 3, 2, 1, 1, 256, 1),
    ("convT", 256, 256, 256, 3, 2, 1, 1, 32, 4),
    ("convT", 320, 320, 256, 3, 2, 1, 1, 64, 2),
    ("convT", 64, 64, 64, 3, 2, 1, 1, 128, 1),
]


# (geometry, swap): the ConvTs both ways -- as the stride-2 conv over dy and as four phases
CASES = [(g, True) for g in GEOMS] + [(g, False) for g in GEOMS if g[0] == "convT"]


@pytest.mark.parametrize("geom,swap", CASES, ids=[f"{g[0]}{g[1]}-{g[3]}k{g[4]}s{g[5]}d{g[7]}H{g[8]}"
                                                  + ("" if g[0] == "conv" else ("-swap" if sw else "-phases"))
                                                  for g, sw in CASES])
def test_wgrad_bf16(gpu, geom, swap):
    from zebrapose_amd.engine import Engine, Unit, Act
    from zebrapose_amd.model import layers as LY
    kind, cin, cw, cout, k, s, p, d, H, B = geom
    torch.manual_seed(3)
    if kind == "conv":
        conv = LY.Conv2d(cw, cout, k, s, p, d, bias=False)
    else:
        conv = LY.ConvTranspose2d(cw, cout, k, s, p, output_padding=1, bias=False)
    unit = Unit(conv, None, relu=False, cin_act=cin)
    OH, OW = unit.out_hw(H, H)
    x = torch.randn(B, cin, H, H).bfloat16().float()
    x[:, cw:] = 0  # padded input channels carry zeros, as the network's input kernel writes them
    ldy = 32 if cout == 17 else cout
    gy = torch.randn(B, ldy, OH, OW).bfloat16().float()
    gy[:, cout:] = 0
    xx = x[:, :cw].clone().requires_grad_(False)
    w = conv.weight.detach().clone().requires_grad_(True)
    if kind == "conv":
        y = F.conv2d(xx, w, None, s, p, d)
    else:
        y = F.conv_transpose2d(xx, w, None, 2, 1, 1)
    y.backward(gy[:, :cout])
    want = w.grad

    eng = Engine(torch.nn.Module(), torch.bfloat16)
    eng.convT_wgrad_swap = swap
    convg = conv.to(gpu)
    xa = Act(x.permute(0, 2, 3, 1).contiguous().to(gpu, torch.bfloat16))
    dya = Act(gy.permute(0, 2, 3, 1).contiguous().to(gpu, torch.bfloat16), 0, cout)
    dw = torch.empty_like(convg.weight)
    assert eng._convT_wgrad_swap(unit, xa, dya) == (kind == "convT" and swap)
    eng._wgrad(unit, xa, unit.fwd_plan(H, H), dya, dw)
    torch.cuda.synchronize()
    got = dw.cpu()
    rel = ((got - want).norm() / want.norm()).item()
    mx = (got - want).abs().max().item() / want.abs().max().item()
    assert rel <= 2e-3 and mx <= 1e-2, f"rel L2 {rel:.3g}, max {mx:.3g}"
