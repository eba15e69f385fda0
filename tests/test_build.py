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
    after an innocuous-looking change; 333 in the first wide split tile, from a sunk correction
    flush).  Compile the device code of every conv source to assembly (with the Makefile's per-file
    flags) and check every k_conv* / k_wgrad_lds / k_stem instantiation for private segment (scratch)
    use -- except the timing-only ablation builds of k_conv3w (ABL != 0)."""
    import re
    srcs = {"zp_conv.hip": [], "zp_conv3.hip": [], "zp_conv3w.hip": ["-fno-slp-vectorize"], "zp_stem.hip": []}
    procs = []
    for f, extra in srcs.items():
        asm = tmp_path / (f + ".s")
        procs.append((asm, subprocess.Popen(
            ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S", *extra,
             os.path.join(ROOT, "zebrapose_amd", "csrc", f), "-o", str(asm)],
            stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    checked = 0
    for asm, p in procs:
        out, _ = p.communicate(timeout=900)
        assert p.returncode == 0, out.decode()[-2000:]
        text = asm.read_text()
        blocks = re.findall(r"\.name:\s+(\S+)\n(.*?)(?=\n  - |\n\.end_amdgpu_metadata)", text, re.S)
        for name, body in blocks:
            if "k_conv" not in name and "k_wgrad_lds" not in name and "k_stem" not in name:
                continue
            if re.search(r"k_conv3wILi[1-9]", name):  # diagnostic ablation builds
                continue
            checked += 1
            priv = int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", body).group(1))
            spill = int(re.search(r"\.vgpr_spill_count:\s+(\d+)", body).group(1))
            assert priv == 0 and spill == 0, f"{name}: scratch {priv} B, {spill} spilled VGPRs"
    assert checked >= 20, checked
