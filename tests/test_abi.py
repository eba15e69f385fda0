"""The C-ABI library loads (no GPU needed) and exports every function include/zp.h declares;
the ctypes structs match the C structs' sizes."""
import ctypes
import os
import re

from tests.conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "zp.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?(?:int|long long|char\s*\*|const char\s*\*)\s*\**\s*(zp_\w+)\s*\(",
                                 src, flags=re.M)))


def test_header_declares_functions():
    names = _declared()
    assert "zp_conv2d" in names and "zp_decode" in names and "zp_code_loss" in names
    assert len(names) >= 30


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(os.path.join(ROOT, "zebrapose_amd", "libzp.so"))
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    from zebrapose_amd import _lib
    assert set(_declared()) <= set(_lib._SIGS), set(_declared()) - set(_lib._SIGS)
    assert _lib.lib.zp_abi_version() == 4


def test_struct_layout():
    from zebrapose_amd import _lib
    # offsets the kernels rely on: sub[] array right after nsub, 8-byte aligned pointers
    assert ctypes.sizeof(_lib.ConvSub) % 8 == 0
    assert _lib.ConvArgs.sub.offset % 8 == 0
    # ABI 3: the fused BN backward reduce's three pointers follow sub[]
    assert _lib.ConvArgs.bnr_x.offset == _lib.ConvArgs.sub.offset + 4 * ctypes.sizeof(_lib.ConvSub)
    assert ctypes.sizeof(_lib.ConvArgs) == _lib.ConvArgs.bnr_x.offset + 3 * 8
    assert ctypes.sizeof(_lib.PackJob) == 16 + 10 * 4 + 2 * 64  # zp_pack_job (include/zp.h)


def test_host_side_validation_without_gpu():
    """Argument checks run on the host before any launch: a bad call fails cleanly (no GPU needed)."""
    from zebrapose_amd import _lib
    a = _lib.ConvArgs()
    a.dtype = 7
    rc = _lib.lib.zp_conv2d(ctypes.byref(a), None)
    assert rc == 1 and b"dtype" in _lib.lib.zp_last_error()
    assert _lib.lib.zp_conv_rows_pad(17) == 32 and _lib.lib.zp_conv_rows_pad(320) == 384
