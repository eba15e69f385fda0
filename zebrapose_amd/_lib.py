"""ctypes binding of libzp.so (include/zp.h).

The library is the product: there is no fallback.  If ``libzp.so`` is missing or
a call fails, this module raises.  PyTorch is used only for device memory and the
current HIP stream (``torch.cuda.current_stream().cuda_stream``).
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (load torch's HIP runtime first; libzp binds to the same libamdhip64.so.7)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ZP_LIB", os.path.join(_HERE, "libzp.so"))

ZP_F32, ZP_BF16, ZP_F16, ZP_F32X3, ZP_F32H2 = 0, 1, 2, 3, 4
ZP_OUT_NHWC, ZP_OUT_HEAD_NCHW, ZP_OUT_NHWC_F32, ZP_OUT_NHWC_X3, ZP_OUT_NHWC_H2 = 0, 1, 2, 3, 4
MAX_TAPS, MAX_SUB = 64, 4

vp = C.c_void_p
i32 = C.c_int
i64 = C.c_longlong
f32 = C.c_float
f64 = C.c_double


class ConvSub(C.Structure):
    _fields_ = [("w", vp), ("scale", vp), ("shift", vp), ("y", vp), ("y2", vp),
                ("ldy", i32), ("cy0", i32), ("OH", i32), ("OW", i32),
                ("oys", i32), ("oyo", i32), ("oxs", i32), ("oxo", i32),
                ("ntaps", i32), ("kw", i32), ("dil", i32), ("pad", i32),
                ("ty", C.c_byte * MAX_TAPS), ("tx", C.c_byte * MAX_TAPS)]


class ConvArgs(C.Structure):
    _fields_ = [("dtype", i32), ("x", vp), ("ldx", i32), ("cx0", i32), ("IH", i32), ("IW", i32), ("Cin", i32),
                ("N", i32), ("GH", i32), ("GW", i32), ("sy", i32), ("sx", i32),
                ("Cout", i32), ("k_pad", i32), ("w_rows", i32),
                ("res", vp), ("ldr", i32), ("cr0", i32), ("relu", i32), ("out_mode", i32),
                ("stats", vp), ("nsub", i32), ("sub", ConvSub * MAX_SUB),
                ("bnr_x", vp), ("bnr_save", vp), ("bnr_part", vp)]


class WgradSub(C.Structure):
    _fields_ = [("dy", vp), ("lddy", i32), ("cdy0", i32), ("OH", i32), ("OW", i32),
                ("oys", i32), ("oyo", i32), ("oxs", i32), ("oxo", i32), ("ntaps", i32),
                ("ky", C.c_byte * MAX_TAPS), ("kx", C.c_byte * MAX_TAPS),
                ("ty", C.c_byte * MAX_TAPS), ("tx", C.c_byte * MAX_TAPS)]


class WgradArgs(C.Structure):
    _fields_ = [("dtype", i32), ("x", vp), ("ldx", i32), ("cx0", i32), ("IH", i32), ("IW", i32), ("Cin", i32),
                ("N", i32), ("GH", i32), ("GW", i32), ("sy", i32), ("sx", i32),
                ("Cout", i32), ("Cw", i32), ("kh", i32), ("kw", i32), ("transposed_w", i32),
                ("nsub", i32), ("sub", WgradSub * MAX_SUB), ("dw", vp), ("accumulate", i32)]


class HeadArgs(C.Structure):
    _fields_ = [("w", vp), ("k_pad", i32), ("bias", vp), ("cout", i32), ("x2", vp), ("ldx2", i32), ("cx20", i32),
                ("C2", i32), ("mask", vp), ("code", vp), ("ws", vp)]


class PackJob(C.Structure):
    _fields_ = [("src", vp), ("dst", vp), ("d0", i32), ("d1", i32), ("kh", i32), ("kw", i32),
                ("transposed", i32), ("ntaps", i32), ("cstride", i32), ("rows_pad", i32), ("k_pad", i32),
                ("dtype", i32), ("ky", C.c_byte * MAX_TAPS), ("kx", C.c_byte * MAX_TAPS)]


# name -> (restype, argtypes)
_SIGS = {
    "zp_abi_version": (i32, []),
    "zp_last_error": (C.c_char_p, []),
    "zp_conv2d": (i32, [C.POINTER(ConvArgs), vp]),
    "zp_conv_rows_pad": (i32, [i32]),
    "zp_conv2d_grid": (i32, [C.POINTER(ConvArgs)]),
    "zp_conv2d_stat_parts": (i32, [C.POINTER(ConvArgs)]),
    "zp_conv2d_bnr_parts": (i32, [C.POINTER(ConvArgs)]),
    "zp_conv2d_split_ws": (C.c_longlong, [C.POINTER(ConvArgs)]),
    "zp_pack_weight": (i32, [vp, i32, i32, i32, i32, i32, i32, C.POINTER(i32), C.POINTER(i32), i32, i32, vp, i32,
                             i32, vp]),
    "zp_conv2d_wgrad_ws_bytes": (i64, [C.POINTER(WgradArgs)]),
    "zp_conv2d_wgrad": (i32, [C.POINTER(WgradArgs), vp, vp]),
    "zp_bn_fold": (i32, [vp, vp, vp, vp, vp, f32, i32, vp, vp, vp]),
    "zp_bn_train_finalize": (i32, [vp, i32, i32, i64, f32, f32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "zp_bn_finalize_floats": (C.c_longlong, [i32, i32]),
    "zp_bn_apply": (i32, [vp, i32, i32, vp, vp, vp, i32, i32, i32, i32, vp, i32, i32, vp]),
    "zp_bn_bwd_parts": (i32, [i32, i32]),
    "zp_bn_bwd_reduce": (i32, [vp, i32, i32, vp, i32, i32, vp, i32, i32, vp, i32, i32, vp, vp, vp, i32, vp]),
    "zp_bn_bwd_totals": (i32, [vp, i32, i32, i32, vp, vp, i32, vp]),
    "zp_bn_bwd_apply": (i32, [vp, i32, i32, vp, i32, i32, vp, i32, i32, vp, vp, vp, i32, i32, vp, vp, i32, i32, i32,
                              vp]),
    "zp_nchw_to_nhwc": (i32, [vp, i32, i32, i32, i32, i32, i32, vp, vp]),
    "zp_maxpool3s2": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, vp, i32, i32, i32, i32, vp]),
    "zp_im2col_split": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp]),
    "zp_maxpool3s2_bwd": (i32, [vp, i32, i32, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, i32, i32, i32,
                                vp]),
    "zp_global_avgpool": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, vp, vp]),
    "zp_broadcast_hw": (i32, [vp, i32, i32, i32, vp, i32, i32, i32, i32, vp]),
    "zp_sum_hw": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, vp, vp]),
    "zp_add_broadcast_hw": (i32, [vp, f32, i32, i32, i32, vp, i32, i32, i32, i32, i32, vp]),
    "zp_copy_slice": (i32, [vp, i32, i32, i32, vp, i32, i32, i32, i32, i32, i32, vp]),
    "zp_head_grad_to_nhwc": (i32, [vp, vp, i32, i32, i32, i32, i32, i32, vp, vp]),
    "zp_mask_interp": (i32, [vp, i32, i32, i32, i32, i32, i32, vp, i32, i32, vp]),
    "zp_mask_interp_bwd": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, i32, vp]),
    "zp_code_loss_ws_bytes": (i64, [i32, i32, i32, i32]),
    "zp_code_loss": (i32, [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp]),
    "zp_code_loss_bwd": (i32, [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp]),
    "zp_mask_loss_ws_bytes": (i64, [i64]),
    "zp_mask_loss": (i32, [vp, vp, i64, vp, vp, vp]),
    "zp_mask_loss_bwd": (i32, [vp, vp, i64, vp, vp, vp]),
    "zp_threshold": (i32, [vp, i64, i32, vp, vp]),
    "zp_decode_ws_bytes": (i64, [i32, i32, i32]),
    "zp_decode": (i32, [vp, vp, i32, i32, i32, i32, i32, vp, vp, vp, i32, vp, vp, vp, vp, vp, vp]),
    "zp_lut_coarsen": (i32, [vp, i32, i32, vp, vp]),
    "zp_adam": (i32, [vp, vp, vp, vp, i64, f64, f64, f64, f64, i64, vp]),
    "zp_pack_weight_multi": (i32, [i32, vp, vp, i64, vp]),
    "zp_conv2d_config": (i32, [vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]),
    "zp_conv_tuning": (i32, [i32, i32]),
    "zp_pnp_ws_bytes": (i64, [i32, i32]),
    "zp_pnp_ransac": (i32, [i32, i32, vp, vp, vp, vp, i32, f64, f64, vp, vp, vp, vp, vp, vp]),
    "zp_pose_error_ws_bytes": (i64, [i32, i32, i32]),
    "zp_pose_error": (i32, [i32, vp, i32, vp, vp, vp, vp, i32, vp, vp, vp]),
    "zp_crop_image": (i32, [vp, i32, i32, i32, vp, vp, i32, i32, vp, vp]),
    "zp_crop_gt": (i32, [vp, vp, vp, i32, i32, i32, vp, vp, i32, i32, i32, vp, vp, vp, vp]),
    "zp_adam_multi": (i32, [i32, vp, vp, vp, vp, vp, f64, f64, f64, f64, i64, vp]),
    "zp_adam_multi_dev": (i32, [i32, vp, vp, vp, vp, vp, f64, f64, f64, f64, vp, vp]),
    "zp_split_range_flag": (i32, [vp]),
    "zp_stem_split": (i32, [vp, i32, i32, i32, i32, vp, i32, i32, vp, vp, i32, vp, i32, i32, i32, i32, vp]),
    "zp_conv2d_head_ok": (i32, [C.POINTER(ConvArgs)]),
    "zp_conv2d_head": (i32, [C.POINTER(ConvArgs), C.POINTER(HeadArgs), vp]),
    "zp_conv2d_head_ws": (C.c_longlong, [C.POINTER(ConvArgs)]),
}


class ZPError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libzp.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; "
                          f"g.build()'` (make -C zebrapose_amd/csrc).  There is no CPU fallback.")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.zp_abi_version() != 4:
        raise ImportError("libzp.so ABI version mismatch")
    return lib


lib = _load()


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib.zp_last_error().decode(errors="replace")
        raise ZPError(f"{what or 'libzp'} failed (rc={rc}): {msg}")


def call(name: str, *args):
    check(getattr(lib, name)(*args), name)


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


_RANGE_FLAGS = {}  # device index -> the word registered last (kept alive while registered)


def register_range_flag(t: torch.Tensor) -> None:
    """Register ``t`` (int32 [1] on a HIP device) with zp_split_range_flag (include/zp.h) for its
    device: every ZP_F32H2 store enqueued from now on raises it for a finite value beyond fp16's
    range.  The C side reads the pointer at enqueue time, so each Engine registers its own word
    before its launches (a captured hipGraph keeps the word of its capture).  The tensor is kept
    alive here while it is the registered one, so the registry never points at freed memory."""
    idx = t.device.index if t.device.index is not None else torch.cuda.current_device()
    if _RANGE_FLAGS.get(idx) is t:
        return
    with torch.cuda.device(idx):
        check(lib.zp_split_range_flag(t.data_ptr()), "zp_split_range_flag")
    _RANGE_FLAGS[idx] = t


def range_flag(device) -> torch.Tensor:
    """The word currently registered with zp_split_range_flag for ``device`` (int32 [1]); a fresh
    one is created and registered when there is none.  Engines use their own words
    (Engine.range_word); this is for direct callers of the C-ABI (tools, tests)."""
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    t = _RANGE_FLAGS.get(idx)
    if t is None:
        t = torch.zeros(1, dtype=torch.int32, device=f"cuda:{idx}")
        register_range_flag(t)
    return t


def dtype_code(dt) -> int:
    if dt == torch.float32:
        return ZP_F32
    if dt == torch.bfloat16:
        return ZP_BF16
    if dt == torch.float16:
        return ZP_F16
    raise ValueError(f"unsupported activation dtype {dt}")
