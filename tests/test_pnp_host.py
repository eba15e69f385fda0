"""The device EPnP math of csrc/zp_pnp.hip (its __host__ __device__ functions, compiled for the CPU
by tools/pnp_host_check.hip) against oracle/pnp_ref.py's epnp() on the same inlier sets: the final
RANSAC refinement is a well-posed least-squares problem, so the two agree to 1e-9 (relative).
No GPU needed."""
import os
import struct
import subprocess

import numpy as np
import pytest

from oracle import pnp_ref
from tests.conftest import ROOT

K = np.array([[572.4114, 0.0, 325.2611], [0.0, 573.57043, 242.04899], [0.0, 0.0, 1.0]])


@pytest.fixture(scope="module")
def host_check(tmp_path_factory):
    exe = tmp_path_factory.mktemp("pnp") / "pnp_host_check"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "--offload-arch=gfx950",
                    os.path.join(ROOT, "tools", "pnp_host_check.hip"), "-o", str(exe)], check=True,
                   capture_output=True)
    return str(exe)


def _rodrigues(w):
    th = np.linalg.norm(w)
    k = w / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx


@pytest.mark.parametrize("n,noise", [(6, 0.0), (40, 0.5), (419, 0.5), (5000, 1.0)])
def test_epnp_refinement_matches_oracle(host_check, tmp_path, n, noise):
    rng = np.random.default_rng(n)
    R = _rodrigues(rng.normal(0, 0.6, 3))
    t = np.array([20.0, -35.0, 750.0])
    pw = rng.uniform(-60, 60, (n, 3)).astype(np.float32)
    Xc = pw.astype(np.float64) @ R.T + t
    uv = np.stack([K[0, 0] * Xc[:, 0] / Xc[:, 2] + K[0, 2], K[1, 1] * Xc[:, 1] / Xc[:, 2] + K[1, 2]], 1)
    uv = np.round(uv + rng.normal(0, noise, uv.shape)).astype(np.float32)
    inl = np.arange(n, dtype=np.int32)
    sub = np.zeros((1, 5), np.int32)
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(fin, "wb") as f:
        f.write(struct.pack("ii", n, 1))
        f.write(np.array([K[0, 0], K[1, 1], K[0, 2], K[1, 2]]).tobytes())
        f.write(pw.tobytes())
        f.write(uv.tobytes())
        f.write(sub.tobytes())
        f.write(struct.pack("i", n))
        f.write(inl.tobytes())
    subprocess.run([host_check, str(fin), str(fout)], check=True, capture_output=True)
    out = np.fromfile(fout, dtype=np.float64)[12:]
    Rr, tr = pnp_ref.epnp(pw, uv, K)
    np.testing.assert_allclose(out[:9].reshape(3, 3), Rr, atol=1e-9)
    np.testing.assert_allclose(out[9:], tr, rtol=1e-9, atol=1e-9 * np.abs(tr).max())
