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


def test_mfma_kernels_do_not_spill(tmp_path):
    """The MFMA kernels run at 1-2 waves per SIMD with most registers holding accumulators: a
    scratch spill halves their speed (seen once: 112 spilled VGPRs in the 256-channel conv tile
    after an innocuous-looking change).  Compile the device code to assembly and check every
    k_conv / k_wgrad_lds instantiation for private segment (scratch) use."""
    import re
    src = os.path.join(ROOT, "zebrapose_amd", "csrc", "zp_conv.hip")
    asm = tmp_path / "zp_conv.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    src, "-o", str(asm)], check=True, capture_output=True)
    text = asm.read_text()
    blocks = re.findall(r"\.name:\s+(\S+)\n(.*?)(?=\n  - |\n\.end_amdgpu_metadata)", text, re.S)
    checked = 0
    for name, body in blocks:
        if "k_conv" not in name and "k_wgrad_lds" not in name:
            continue
        checked += 1
        priv = int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", body).group(1))
        spill = int(re.search(r"\.vgpr_spill_count:\s+(\d+)", body).group(1))
        assert priv == 0 and spill == 0, f"{name}: scratch {priv} B, {spill} spilled VGPRs"
    assert checked >= 10, checked
