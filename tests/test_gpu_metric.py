"""ADD / ADI on the device against the reference formulas (lib/pysixd/pose_error.py:297-336:
numpy f64 transforms, scipy cKDTree nearest neighbour for ADI)."""
import numpy as np
import pytest
from scipy import spatial

pytestmark = pytest.mark.gpu


def _rot(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


@pytest.mark.parametrize("n", [1, 777, 5000])
def test_add_adi_match_reference_formulas(gpu, n):
    from zebrapose_amd.metric import pose_errors, Calculate_ADD_Error_BOP, Calculate_ADI_Error_BOP, ADD, ADI
    rng = np.random.default_rng(n)
    pts = rng.uniform(-60, 60, (n, 3)).astype(np.float32)
    B = 5
    Rg = np.stack([_rot(rng) for _ in range(B)])
    tg = rng.uniform(-50, 50, (B, 3)) + np.array([0, 0, 800])
    Re = np.stack([r @ _rot(np.random.default_rng(k)) if k % 2 else r for k, r in enumerate(Rg)])
    te = tg + rng.normal(0, 5, (B, 3))
    add = pose_errors(pts, Re, te, Rg, tg, ADD).cpu().numpy()
    adi = pose_errors(pts, Re, te, Rg, tg, ADI).cpu().numpy()
    p64 = pts.astype(np.float64)
    for b in range(B):
        pe = (Re[b] @ p64.T + te[b][:, None]).T
        pg = (Rg[b] @ p64.T + tg[b][:, None]).T
        want_add = np.linalg.norm(pe - pg, axis=1).mean()
        want_adi = spatial.cKDTree(pe).query(pg, k=1)[0].mean()
        assert abs(add[b] - want_add) <= 1e-9 * max(1.0, want_add)
        assert abs(adi[b] - want_adi) <= 1e-9 * max(1.0, want_adi)
    # reference-signature drop-ins (metric.py:8-18)
    assert abs(Calculate_ADD_Error_BOP(Rg[1], tg[1], Re[1], te[1], pts) - add[1]) < 1e-12
    assert abs(Calculate_ADI_Error_BOP(Rg[1], tg[1], Re[1], te[1], pts) - adi[1]) < 1e-12


def test_add_adi_match_reference_fixture(gpu, golden):
    """ADD / ADI against the values the reference's own lib/pysixd/pose_error.add / adi returned
    (tests/golden/add_adi.npz: identical pose, rotated, translated, 180-degree flip, random, 1 um)."""
    from zebrapose_amd.metric import pose_errors, ADD, ADI
    f = golden("add_adi.npz")
    add = pose_errors(f["pts"], f["R_est"], f["t_est"], f["R_gt"], f["t_gt"], ADD).cpu().numpy()
    adi = pose_errors(f["pts"], f["R_est"], f["t_est"], f["R_gt"], f["t_gt"], ADI).cpu().numpy()
    np.testing.assert_allclose(add, f["add"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(adi, f["adi"], rtol=1e-9, atol=1e-12)
