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


LLVM = "/opt/rocm/lib/llvm/bin"
CSRC = os.path.join(ROOT, "zebrapose_amd", "csrc")
LIB = os.path.join(ROOT, "zebrapose_amd", "libzp.so")


def _kernel_metadata_from_lib(tmp_path):
    """(name, scratch bytes, spilled VGPRs) of every gfx950 kernel in the built libzp.so: its
    .hip_fatbin holds one offload bundle per translation unit; each is unbundled and its code
    object's metadata note read."""
    import re
    fat = tmp_path / "fat.bin"
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", LIB, str(tmp_path / "lib.o")], check=True,
                   capture_output=True)
    data = fat.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    assert starts, "no offload bundle in libzp.so"
    out = []
    for i, s in enumerate(starts):
        part, co = tmp_path / f"b{i}.bin", tmp_path / f"b{i}.co"
        part.write_bytes(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}", f"--output={co}"],
                       check=True, capture_output=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(co)], check=True, capture_output=True,
                               text=True).stdout
        for body in re.split(r"\n  - (?=\.)", notes)[1:]:
            name = re.search(r"^    \.name:\s+(\S+)", body, re.M)
            priv = re.search(r"^    \.private_segment_fixed_size:\s+(\d+)", body, re.M)
            spill = re.search(r"^    \.vgpr_spill_count:\s+(\d+)", body, re.M)
            if name and priv and spill:
                out.append((name.group(1), int(priv.group(1)), int(spill.group(1))))
    return out


def _kernel_metadata_from_sources(tmp_path):
    """The same from the sources: device code of every conv source compiled to assembly with the
    Makefile's per-file flags."""
    import re
    srcs = {"zp_conv.hip": [], "zp_conv3.hip": [], "zp_conv3w.hip": ["-fno-slp-vectorize"], "zp_stem.hip": []}
    procs = []
    for f, extra in srcs.items():
        asm = tmp_path / (f + ".s")
        procs.append((asm, subprocess.Popen(
            ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S", *extra,
             os.path.join(CSRC, f), "-o", str(asm)],
            stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    out = []
    for asm, p in procs:
        log, _ = p.communicate(timeout=900)
        assert p.returncode == 0, log.decode()[-2000:]
        text = asm.read_text()
        for name, body in re.findall(r"\.name:\s+(\S+)\n(.*?)(?=\n  - |\n\.end_amdgpu_metadata)", text, re.S):
            priv = int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", body).group(1))
            spill = int(re.search(r"\.vgpr_spill_count:\s+(\d+)", body).group(1))
            out.append((name, priv, spill))
    return out


def test_mfma_kernels_do_not_spill(tmp_path):
    """The MFMA kernels run at 1-2 waves per SIMD with most registers holding accumulators: a
    scratch spill halves their speed (seen once: 112 spilled VGPRs in the 256-channel conv tile
    after an innocuous-looking change; 333 in the first wide split tile, from a sunk correction
    flush).  Every k_conv* / k_wgrad* / k_stem instantiation must use no private segment (scratch)
    -- except the timing-only ablation builds of k_conv3w (ABL != 0).  Read from the built
    libzp.so's code objects when it is newer than every source (seconds; build() has just made
    it), else from the sources compiled to assembly (minutes)."""
    import glob
    import re
    srcs = glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h")) + \
        [os.path.join(CSRC, "Makefile")]
    fresh = os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(f) for f in srcs)
    meta = _kernel_metadata_from_lib(tmp_path) if fresh else _kernel_metadata_from_sources(tmp_path)
    checked = 0
    for name, priv, spill in meta:
        if "k_conv" not in name and "k_wgrad" not in name and "k_stem" not in name:
            continue
        if re.search(r"k_conv3wILi[1-9]", name):  # diagnostic ablation builds
            continue
        checked += 1
        assert priv == 0 and spill == 0, f"{name}: scratch {priv} B, {spill} spilled VGPRs"
    assert checked >= 20, checked
