"""Host-side implicit-GEMM geometry (zebrapose_amd/geometry.py): the tap / phase plans, executed
by a small torch CPU interpreter, reproduce F.conv2d / F.conv_transpose2d and their data
gradients.  This pins the descriptors that every zp_conv2d / zp_conv2d_wgrad launch uses."""
import pytest
import torch
import torch.nn.functional as F

from zebrapose_amd import geometry as G


def run_plan(plan, x, wmat, OH, OW):
    """x [B,C,IH,IW]; wmat(ky, kx) -> [Cout, Cin]; returns [B, Cout, OH, OW]."""
    B, C, IH, IW = x.shape
    cout = wmat(0, 0).shape[0]
    out = torch.zeros(B, cout, OH, OW, dtype=x.dtype)
    for sb in plan.subs:
        for (ky, kx), (ty, tx) in zip(sb.taps, sb.offs):
            gy = torch.arange(plan.GH)
            gx = torch.arange(plan.GW)
            iy = gy * plan.sy + ty
            ix = gx * plan.sy + tx
            vy = (iy >= 0) & (iy < IH)
            vx = (ix >= 0) & (ix < IW)
            xs = torch.zeros(B, C, plan.GH, plan.GW, dtype=x.dtype)
            xs[:, :, vy.nonzero()[:, 0][:, None], vx.nonzero()[:, 0][None, :]] = \
                x[:, :, iy[vy][:, None], ix[vx][None, :]]
            contrib = torch.einsum("oc,bchw->bohw", wmat(ky, kx), xs)
            oy = gy * sb.oys + sb.oyo
            ox = gx * sb.oxs + sb.oxo
            out[:, :, oy[:, None], ox[None, :]] += contrib
    return out


CONVS = [(3, 1, 1, 1, 9), (3, 2, 1, 1, 10), (1, 2, 0, 1, 10), (3, 1, 2, 2, 9), (3, 1, 6, 6, 8), (3, 1, 18, 18, 8),
         (7, 2, 3, 1, 16), (1, 1, 0, 1, 5)]


@pytest.mark.parametrize("k,s,p,d,H", CONVS)
def test_conv_fwd_and_dgrad(k, s, p, d, H):
    torch.manual_seed(0)
    x = torch.randn(2, 3, H, H, dtype=torch.float64, requires_grad=True)
    w = torch.randn(4, 3, k, k, dtype=torch.float64)
    y = F.conv2d(x, w, None, s, p, d)
    plan = G.conv_fwd(H, H, k, s, p, d)
    got = run_plan(plan, x.detach(), lambda ky, kx: w[:, :, ky, kx], y.shape[2], y.shape[3])
    torch.testing.assert_close(got, y.detach())
    if s == 2 and H % 2:
        return  # phase decomposition needs even input sizes (all network shapes are)
    gy = torch.randn_like(y)
    y.backward(gy)
    dplan = G.conv_dgrad(H, H, k, s, p, d)
    dx = run_plan(dplan, gy, lambda ky, kx: w[:, :, ky, kx].t(), H, H)
    torch.testing.assert_close(dx, x.grad)


@pytest.mark.parametrize("H", [4, 8, 5])
def test_convT_fwd_and_dgrad(H):
    torch.manual_seed(1)
    x = torch.randn(2, 3, H, H, dtype=torch.float64, requires_grad=True)
    w = torch.randn(3, 4, 3, 3, dtype=torch.float64)  # [Cin, Cout, kh, kw]
    y = F.conv_transpose2d(x, w, None, 2, 1, 1)
    plan = G.convT_fwd(H, H)
    assert sum(len(s.taps) for s in plan.subs) == 9 and len(plan.subs) == 4
    got = run_plan(plan, x.detach(), lambda ky, kx: w[:, :, ky, kx].t(), y.shape[2], y.shape[3])
    torch.testing.assert_close(got, y.detach())
    gy = torch.randn_like(y)
    y.backward(gy)
    dplan = G.convT_dgrad(H, H)
    dx = run_plan(dplan, gy, lambda ky, kx: w[:, :, ky, kx], H, H)
    torch.testing.assert_close(dx, x.grad)


def test_out_size():
    assert G.out_size(256, 7, 2, 3) == 128
    assert G.out_size(128, 3, 2, 1) == 64
    assert G.out_size(32, 3, 1, 18, 18) == 32


def run_wgrad(plan, inp, dout):
    """The weight gradient a zp_conv2d_wgrad launch computes from a plan: for every sub and tap,
    dW[:, :, ky, kx] += sum over batch and grid of dout at the sub's output pixel (outer) inp at the
    tap's input pixel.  inp [B,C,IH,IW], dout [B,O,OH,OW] -> [O, C, kh, kw] (kh = kw = 3)."""
    B, C, IH, IW = inp.shape
    O = dout.shape[1]
    dw = torch.zeros(O, C, 3, 3, dtype=inp.dtype)
    for sb in plan.subs:
        gy = torch.arange(plan.GH)
        gx = torch.arange(plan.GW)
        oy = gy * sb.oys + sb.oyo
        ox = gx * sb.oxs + sb.oxo
        ds = dout[:, :, oy[:, None], ox[None, :]]
        for (ky, kx), (ty, tx) in zip(sb.taps, sb.offs):
            iy = gy * plan.sy + ty
            ix = gx * plan.sy + tx
            vy = (iy >= 0) & (iy < IH)
            vx = (ix >= 0) & (ix < IW)
            xs = torch.zeros(B, C, plan.GH, plan.GW, dtype=inp.dtype)
            xs[:, :, vy.nonzero()[:, 0][:, None], vx.nonzero()[:, 0][None, :]] = \
                inp[:, :, iy[vy][:, None], ix[vx][None, :]]
            dw[:, :, ky, kx] += torch.einsum("bohw,bchw->oc", ds, xs)
    return dw


@pytest.mark.parametrize("H", [4, 8])
def test_convT_wgrad_as_strided_conv_over_dy(H):
    """Round 6 (Engine._convT_wgrad_swap): the ConvTranspose2d(3, s2, p1, op1) weight gradient is the
    weight gradient of the stride-2 conv over dy (geometry.convT_dgrad's plan) whose output gradient
    is x -- with the two activations exchanged, in the ConvT weight's own [in][out][kh][kw] layout --
    and equally the four-phase form over x (convT_fwd's plan).  Both against torch's autograd."""
    torch.manual_seed(2)
    x = torch.randn(2, 3, H, H, dtype=torch.float64)
    w = torch.randn(3, 4, 3, 3, dtype=torch.float64, requires_grad=True)  # [Cin, Cout, kh, kw]
    y = F.conv_transpose2d(x, w, None, 2, 1, 1)
    gy = torch.randn_like(y)
    y.backward(gy)
    swap = run_wgrad(G.convT_dgrad(H, H), gy, x)          # [Cin, Cout, 3, 3] directly
    torch.testing.assert_close(swap, w.grad)
    phases = run_wgrad(G.convT_fwd(H, H), x, gy)          # [Cout, Cin, 3, 3]: the transposed layout
    torch.testing.assert_close(phases.transpose(0, 1), w.grad)


@pytest.mark.parametrize("k,s,p,H", [(3, 2, 1, 8), (1, 2, 0, 8), (3, 1, 1, 6)])
def test_conv_wgrad_from_plan(k, s, p, H):
    """The stride-1 / stride-2 conv weight gradient from conv_fwd's plan (the lean k_wgrad2 geometry,
    stride 2 since round 6) against torch's autograd."""
    torch.manual_seed(4)
    x = torch.randn(2, 3, H, H, dtype=torch.float64)
    w = torch.randn(4, 3, k, k, dtype=torch.float64, requires_grad=True)
    y = F.conv2d(x, w, None, s, p)
    gy = torch.randn_like(y)
    y.backward(gy)
    got = run_wgrad(G.conv_fwd(H, H, k, s, p), x, gy)
    torch.testing.assert_close(got[:, :, :k, :k], w.grad)
