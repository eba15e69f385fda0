"""Train-mode BatchNorm backward through the C-ABI (zp_bn_apply / zp_bn_bwd_reduce / zp_bn_bwd_apply):
the ReLU mask recomputed from the raw conv output (relu mode 2) must give bit-identical results to
the mask read from the stored activation (mode 1), and both match a torch fp32 restatement of
nn.BatchNorm2d + ReLU backward (torch/nn/modules/batchnorm.py semantics: batch statistics,
biased variance) within bf16 storage tolerance."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt", ["bf16", "f32"])
@pytest.mark.parametrize("P,Cc", [(4096, 64), (2048, 256), (1000, 512), (37, 8)])
def test_bn_backward_mask_from_raw_matches_stored_mask(dt, P, Cc):
    import zebrapose_amd._lib as L
    dev = torch.device("cuda", 0)
    tdt = torch.bfloat16 if dt == "bf16" else torch.float32
    code = L.dtype_code(tdt)
    g = torch.Generator(device="cpu").manual_seed(P + Cc)
    raw = (torch.randn(P, Cc, generator=g) * 2 + 0.3).to(tdt).to(dev)
    gout = torch.randn(P, Cc, generator=g).to(tdt).to(dev)
    gamma = (torch.rand(Cc, generator=g) + 0.5).to(dev)
    beta = (torch.randn(Cc, generator=g) * 0.5).to(dev)
    rf = raw.float()
    mean = rf.mean(0)
    invstd = torch.rsqrt(rf.var(0, unbiased=False) + 1e-5)
    scale = gamma * invstd
    shift = torch.addcmul(beta, -mean, scale)  # fma(-mean, scale, beta) up to rounding; kernel reads save
    save = torch.cat([mean, invstd, scale, shift]).contiguous()
    y = torch.empty_like(raw)
    st = L.stream_ptr()
    L.call("zp_bn_apply", raw.data_ptr(), P, Cc, scale.data_ptr(), shift.data_ptr(), None, 0, 0, 1, code, y.data_ptr(),
           Cc, 0, st)
    parts = L.lib.zp_bn_bwd_parts(P, Cc)
    outs = {}
    for mode in (1, 2):
        partials = torch.empty(2 * (parts + 1) * Cc, dtype=torch.float32, device=dev)
        dgamma = torch.empty(Cc, device=dev)
        dbeta = torch.empty(Cc, device=dev)
        yp = y.data_ptr() if mode == 1 else None
        L.call("zp_bn_bwd_reduce", gout.data_ptr(), Cc, 0, yp, Cc, 0, raw.data_ptr(), P, Cc, save.data_ptr(), mode,
               code, partials.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(), 0, st)
        dx = torch.empty_like(raw)
        L.call("zp_bn_bwd_apply", gout.data_ptr(), Cc, 0, yp, Cc, 0, raw.data_ptr(), P, Cc, save.data_ptr(),
               partials.data_ptr(), gamma.data_ptr(), mode, code, dx.data_ptr(), None, 0, 0, 0, st)
        torch.cuda.synchronize()
        outs[mode] = (dgamma.cpu(), dbeta.cpu(), dx.float().cpu())
    for a, b in zip(outs[1], outs[2]):
        assert torch.equal(a, b)
    # fp32 restatement: y = relu(xhat*gamma + beta); dL/dx through batch statistics
    xhat = (rf - mean) * invstd
    m = ((rf * scale + shift) > 0).float()
    gm = gout.float() * m
    db = gm.sum(0)
    dg = (gm * xhat).sum(0)
    dx_ref = gamma * invstd * (gm - db / P - xhat * dg / P)
    dgamma, dbeta, dx = outs[2]
    tol = 2e-2 if dt == "bf16" else 1e-4
    assert torch.allclose(dbeta, db.cpu(), rtol=1e-4, atol=1e-3)
    assert torch.allclose(dgamma, dg.cpu(), rtol=1e-4, atol=1e-3)
    err = float((dx - dx_ref.cpu()).norm() / dx_ref.norm())
    assert err < tol, err
    # the mask the kernel forms agrees with y > 0 wherever y is stored nonzero
    yk = y.float().cpu() > 0
    mk = (torch.addcmul(shift, rf, scale) > 0).cpu()  # fma form
    assert float((yk != mk).float().mean()) < 1e-3


@pytest.mark.parametrize("parts,C", [(8192, 64), (4100, 256), (200, 96), (512, 256), (1024, 2048)])
def test_bn_stat_merge_one_launch_equals_two(gpu, parts, C):
    """zp_bn_train_finalize's level-1 + level-2 statistics merge in ONE launch (zp_conv_tuning key 15;
    the last-arriving block of each channel group runs level 2 after an agent-scope counter hand-off)
    stores exactly the bits of the two-launch form (same parts, same fixed merge order), re-arms its
    counters (three calls in a row agree), and matches a float64 merge of the same partials (Chan's
    formula: the train-mode batch mean / biased variance, train_v6.py's BatchNorm2d in training).
    Up to 512 parts (200, 512) run the one-level merge (k_bn_stat_merge1) in both modes."""
    from zebrapose_amd import _lib as L
    g = torch.Generator().manual_seed(parts + C)
    cnt = torch.randint(1, 33, (parts, C), generator=g).float()
    mean = torch.randn(parts, C, generator=g) * 3 + 1
    m2 = torch.rand(parts, C, generator=g) * cnt * 2
    base = torch.cat([cnt, mean, m2]).contiguous()
    gamma, beta = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g)

    def run(mode):
        old = L.lib.zp_conv_tuning(15, mode)
        try:
            part = torch.empty(L.lib.zp_bn_finalize_floats(parts, C), device=gpu)
            part[:base.numel()] = base.reshape(-1).to(gpu)
            rm, rv = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
            nbt = torch.zeros(1, dtype=torch.int64, device=gpu)
            sc, sh = torch.empty(C, device=gpu), torch.empty(C, device=gpu)
            save = torch.empty(4 * C, device=gpu)
            L.call("zp_bn_train_finalize", part.data_ptr(), parts, C, int(cnt.sum()), 1e-5, 0.1,
                   gamma.to(gpu).data_ptr(), beta.to(gpu).data_ptr(), None, rm.data_ptr(), rv.data_ptr(), nbt.data_ptr(),
                   sc.data_ptr(), sh.data_ptr(), save.data_ptr(), L.stream_ptr())
            torch.cuda.synchronize()
            return [t.cpu() for t in (sc, sh, save, rm, rv, nbt)]
        finally:
            L.lib.zp_conv_tuning(15, old)
    two = run(0)
    ones = [run(1) for _ in range(3)]
    for one in ones:
        for a, b in zip(one, two):
            assert torch.equal(a, b)
    c64, m64, q64 = cnt.double(), mean.double(), m2.double()
    n = c64.sum(0)
    mu = (c64 * m64).sum(0) / n
    var = (q64.sum(0) + (c64 * (m64 - mu) ** 2).sum(0)) / n
    got_mean, got_inv = two[2][:C].double(), two[2][C:2 * C].double()
    assert torch.allclose(got_mean, mu, rtol=1e-6, atol=1e-6)
    assert torch.allclose(got_inv, 1.0 / torch.sqrt(var + 1e-5), rtol=1e-6)
    assert int(two[5][0]) == 1


def test_bn_stat_merge_concurrent_streams(gpu):
    """the one-launch merge's hand-off counters are per launch (ABI 4: in the caller's
    partials buffer, zeroed on the launch's stream).  Six finalizes of >512 parts enqueued round-robin
    on three streams without waiting, so their level-1 blocks interleave, each equal bit for bit to
    the same finalize run alone."""
    from zebrapose_amd import _lib as L
    C, parts = 256, 4100
    streams = [torch.cuda.Stream(device=gpu) for _ in range(3)]
    cases = []
    for i in range(6):
        g = torch.Generator().manual_seed(100 + i)
        cnt = torch.randint(1, 33, (parts, C), generator=g).float()
        base = torch.cat([cnt, torch.randn(parts, C, generator=g) * 3 + i, torch.rand(parts, C, generator=g) * cnt])
        cases.append((base.to(gpu), (torch.rand(C, generator=g) + 0.5).to(gpu), torch.randn(C, generator=g).to(gpu),
                      int(cnt.sum())))

    def launch(case, st):
        base, gamma, beta, count = case
        part = torch.empty(L.lib.zp_bn_finalize_floats(parts, C), device=gpu)
        part[:base.numel()].copy_(base.reshape(-1))
        out = [torch.zeros(C, device=gpu), torch.ones(C, device=gpu), torch.zeros(1, dtype=torch.int64, device=gpu),
               torch.empty(C, device=gpu), torch.empty(C, device=gpu), torch.empty(4 * C, device=gpu)]
        torch.cuda.synchronize()
        with torch.cuda.stream(st):
            L.call("zp_bn_train_finalize", part.data_ptr(), parts, C, count, 1e-5, 0.1, gamma.data_ptr(),
                   beta.data_ptr(), None, out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), out[3].data_ptr(),
                   out[4].data_ptr(), out[5].data_ptr(), st.cuda_stream)
        return part, out

    alone = []
    for c in cases:
        _, out = launch(c, streams[0])
        torch.cuda.synchronize()
        alone.append([t.cpu() for t in out])
    # concurrent: all buffers prepared first, then every launch enqueued before any wait
    prepared = []
    for c in cases:
        base, gamma, beta, count = c
        part = torch.empty(L.lib.zp_bn_finalize_floats(parts, C), device=gpu)
        part[:base.numel()].copy_(base.reshape(-1))
        prepared.append((part, [torch.zeros(C, device=gpu), torch.ones(C, device=gpu),
                                torch.zeros(1, dtype=torch.int64, device=gpu), torch.empty(C, device=gpu),
                                torch.empty(C, device=gpu), torch.empty(4 * C, device=gpu)], gamma, beta, count))
    torch.cuda.synchronize()
    for i, (part, out, gamma, beta, count) in enumerate(prepared):
        st = streams[i % 3]
        L.call("zp_bn_train_finalize", part.data_ptr(), parts, C, count, 1e-5, 0.1, gamma.data_ptr(), beta.data_ptr(),
               None, out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), out[3].data_ptr(), out[4].data_ptr(),
               out[5].data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    for (part, out, *_), ref in zip(prepared, alone):
        for a, b in zip(out, ref):
            assert torch.equal(a.cpu(), b)


@pytest.mark.parametrize("dt", ["bf16", "f16", "f32"])
@pytest.mark.parametrize("P,Cc,res,relu", [(4096, 64, False, 1), (2048, 256, True, 1), (1000, 512, True, 0),
                                           (37, 8, False, 1), (513, 2048, True, 1), (300, 24, True, 1),
                                           (129, 96, False, 0)])
def test_bn_apply_unrolled_equals_grid_stride(dt, P, Cc, res, relu, monkeypatch):
    """zp_bn_apply's k_bn_apply_u (C / N a power of two dividing 256: a fixed channel chunk per
    thread, 4 chunks in flight) against the grid-stride k_bn_apply (ZP_BN_APPLY_U=0, read per call):
    bit-identical, with and without the residual and ReLU, into a channel slice of a wider buffer;
    channel counts 24 / 96 (C / N not a power of two) take the grid-stride kernel either way.  Both
    match y = relu(x * scale + shift (+ res)) in f32 within the storage type's rounding."""
    import zebrapose_amd._lib as L
    dev = torch.device("cuda", 0)
    tdt = {"bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32}[dt]
    code = L.dtype_code(tdt)
    g = torch.Generator(device="cpu").manual_seed(P * 7 + Cc)
    x = torch.randn(P, Cc, generator=g).to(tdt).to(dev)
    r = torch.randn(P, 2 * Cc, generator=g).to(tdt).to(dev) if res else None
    scale = (torch.rand(Cc, generator=g) + 0.5).to(dev)
    shift = torch.randn(Cc, generator=g).to(dev)
    outs = []
    for knob in ("1", "0"):
        monkeypatch.setenv("ZP_BN_APPLY_U", knob)
        y = torch.full((P, 3 * Cc), 7.0, dtype=tdt, device=dev)
        L.call("zp_bn_apply", x.data_ptr(), P, Cc, scale.data_ptr(), shift.data_ptr(),
               None if r is None else r.data_ptr(), 2 * Cc, Cc if res else 0, relu, code, y.data_ptr(), 3 * Cc, Cc,
               L.stream_ptr())
        torch.cuda.synchronize()
        outs.append(y)
    assert torch.equal(outs[0], outs[1])
    y = outs[0]
    assert torch.all(y[:, :Cc] == 7.0) and torch.all(y[:, 2 * Cc:] == 7.0)  # outside the slice untouched
    ref = x.float() * scale + shift
    if res:
        ref = ref + r[:, Cc:2 * Cc].float()
    if relu:
        ref = ref.clamp_min(0.0)
    tol = {"bf16": 1e-2, "f16": 2e-3, "f32": 1e-6}[dt]
    torch.testing.assert_close(y[:, Cc:2 * Cc].float(), ref, rtol=tol, atol=tol)
