"""Every kernel instantiation the host dispatch references is present in libzp.so (the host
compile pass can silently drop a kernel stub, which only shows up as an undefined symbol)."""
import os
import subprocess

from tests.conftest import ROOT


def test_no_undefined_kernel_stubs():
    out = subprocess.run(["nm", "-D", "--undefined-only", os.path.join(ROOT, "zebrapose_amd", "libzp.so")],
                         capture_output=True, text=True, check=True).stdout
    bad = [l for l in out.splitlines() if "device_stub" in l or "_ZN2zp" in l]
    assert not bad, bad
