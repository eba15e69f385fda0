"""Host-code AddressSanitizer build of the C-ABI (VERDICT r3 housekeeping).

``make -C zebrapose_amd/csrc asan`` compiles every libzp source with the host side instrumented
(``-Xarch_host -fsanitize=address``; the device side at -O0, since nothing here launches a kernel)
into libzp_asan.so, and tests/asan/abi_driver.cpp -- also instrumented -- calls the C-ABI entry
points whose work is host code: argument validation of invalid calls, workspace sizing, the
launch-configuration queries for the bench geometries (tile choice, split-K, fused-head
eligibility), tuning knobs.  No GPU is needed and none is used (GPU sanitizers are not run).  Any
out-of-bounds access or use-after-free in that host code aborts the driver with an ASan report."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "zebrapose_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
CLANG = "/opt/rocm/lib/llvm/bin/clang++"  # the driver is plain C++ (same ASan runtime as hipcc's)


@pytest.mark.timeout(900)
@pytest.mark.skipif(not (os.path.exists(HIPCC) and os.path.exists(CLANG)), reason="ROCm toolchain not installed")
def test_abi_host_code_under_asan(tmp_path):
    jobs = str(min(8, os.cpu_count() or 1))
    r = subprocess.run(["make", "-C", CSRC, f"-j{jobs}", "asan"], capture_output=True, text=True, timeout=840)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lib = os.path.join(ROOT, "zebrapose_amd", "libzp_asan.so")
    exe = str(tmp_path / "abi_driver")
    r = subprocess.run([CLANG, "-O1", "-g", "-std=c++17", "-fsanitize=address", "-fno-omit-frame-pointer",
                        "-x", "c++", os.path.join(ROOT, "tests", "asan", "abi_driver.cpp"), "-x", "none", lib,
                        "-o", exe, f"-Wl,-rpath,{os.path.dirname(lib)}"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    print(r.stdout, r.stderr[-3000:])
    assert "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    assert r.returncode == 0 and "abi_driver: ok" in r.stdout, (r.returncode, r.stdout, r.stderr[-2000:])
