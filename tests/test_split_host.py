"""Host-side logic of the split-fp32 engine (no GPU needed): the split-K workspace query
(zp_conv2d_split_ws), the tuning knobs of the split kernels (zp_conv_tuning keys 7 / 8 / 9) and the
im2col entry point's argument checks."""
import ctypes

from zebrapose_amd import _lib as L


def _args(dtype, B, H, cin, cout, k=3, d=1):
    a = L.ConvArgs()
    a.dtype = dtype
    a.N, a.IH, a.IW, a.GH, a.GW, a.sy, a.sx = B, H, H, H, H, 1, 1
    a.Cin, a.Cout, a.ldx, a.k_pad, a.w_rows = cin, cout, cin, k * k * cin, ((cout + 127) // 128) * 128
    a.nsub = 1
    a.out_mode = L.ZP_OUT_NHWC
    s = a.sub[0]
    s.ntaps = k * k
    s.OH, s.OW, s.ldy = H, H, cout
    for t in range(k * k):
        s.ty[t], s.tx[t] = (t // k - k // 2) * d, (t % k - k // 2) * d
    return a


def test_split_k_workspace_query():
    # bs = 1, layer5 (512 -> 512, 3x3 d4 at 32 x 32): 64 workgroups over 144 K steps -> split
    a = _args(L.ZP_F32H2, 1, 32, 512, 512, d=4)
    nb = L.lib.zp_conv2d_split_ws(ctypes.byref(a))
    assert nb > 0 and nb % (32 * 32 * 512 * 4) == 0
    ns = nb // (32 * 32 * 512 * 4)
    assert 2 <= ns <= 16
    # the same layer at bs = 32: enough workgroups, no split; other dtypes never split
    assert L.lib.zp_conv2d_split_ws(ctypes.byref(_args(L.ZP_F32H2, 32, 32, 512, 512, d=4))) == 0
    assert L.lib.zp_conv2d_split_ws(ctypes.byref(_args(L.ZP_BF16, 1, 32, 512, 512, d=4))) == 0
    assert L.lib.zp_conv2d_split_ws(ctypes.byref(_args(L.ZP_F32X3, 1, 32, 512, 512, d=4))) == nb
    old = L.lib.zp_conv_tuning(9, 0)
    try:
        assert L.lib.zp_conv2d_split_ws(ctypes.byref(a)) == 0
    finally:
        L.lib.zp_conv_tuning(9, old)


def test_split_tuning_keys_round_trip():
    for key, val in ((7, 2), (8, 0), (9, 0)):
        old = L.lib.zp_conv_tuning(key, val)
        assert L.lib.zp_conv_tuning(key, old) == val
    assert L.lib.zp_conv_tuning(99, 0) == -1


def test_im2col_split_argument_checks():
    x = ctypes.c_void_p(0x1000)  # never dereferenced: the checks reject before any launch
    y = ctypes.c_void_p(0x2000)
    # kpad below k * k * C
    rc = L.lib.zp_im2col_split(x, 1, 16, 16, 8, 3, 7, 2, 3, 8, 8, 144, L.ZP_F32H2, y, None)
    assert rc == L.ZP_ERR_ARG if hasattr(L, "ZP_ERR_ARG") else rc == 1
    assert b"im2col" in L.lib.zp_last_error()
    # not a split dtype
    rc = L.lib.zp_im2col_split(x, 1, 16, 16, 8, 3, 7, 2, 3, 8, 8, 160, L.ZP_BF16, y, None)
    assert rc == 1 and b"split-fp32" in L.lib.zp_last_error()


def test_eval_batch_limit():
    """Engine.eval_batch_limit: the largest eval batch one pass keeps every conv
    input below 2 GiB -- the widest input is H/2 x W/2 x 384 channels of the engine's storage."""
    import torch
    from zebrapose_amd.engine import Engine
    m = torch.nn.Module()
    lim = {k: Engine(m, torch.float32, split=k).eval_batch_limit(256, 256) for k in ("h2", "x3")}
    lim["f32"] = Engine(m, torch.float32).eval_batch_limit(256, 256)
    lim["bf16"] = Engine(m, torch.bfloat16).eval_batch_limit(256, 256)
    assert lim == {"h2": 85, "x3": 56, "f32": 85, "bf16": 170}, lim
    e = Engine(m, torch.float32, split="h2")
    x = torch.zeros(128, 3, 256, 256)
    parts = e._chunks(x, train=False)
    assert [p.shape[0] for p in parts] == [64, 64]
    assert e._chunks(x, train=True) is None and e._chunks(x[:85], train=False) is None
