"""CPU restatement of the reference's PnP step -- TEST INFRASTRUCTURE ONLY (the product never
imports this module).

Reference call (binary_code_helper/CNN_output_to_pose.py:152-156):
    cv2.solvePnPRansac(Points_3D f32, Original_Points_2D f32, K, distCoeffs=None,
                       reprojectionError=2, iterationsCount=150, flags=cv2.SOLVEPNP_EPNP)
OpenCV is a third-party dependency that is not in this image (no cv2 module, no source in
/root/reference), so this file restates the published algorithms the call runs, following
OpenCV 4.x:
  * ptsetreg.cpp  RANSACPointSetRegistrator::run -- cv::RNG(0xffffffff...) subsets drawn by
    getSubset (redraw duplicates), goodCount > max(maxGood, modelPoints - 1) keeps a model and
    shrinks the iteration budget with RANSACUpdateNumIters(confidence = 0.99)
  * solvepnp.cpp  solvePnPRansac: modelPoints = 5, EPnP hypotheses, inlier <=> float squared
    reprojection error <= reprojectionError^2, final EPnP over all inliers
  * epnp.cpp      Lepetit, Moreno-Noguer & Fua (IJCV 2009)
PARITY UNPINNED against OpenCV itself (no cv2 here, and the reference holds no PnP fixtures); this
restatement is written independently of the HIP kernels (numpy SVD / lstsq) and pins them.
"""
from __future__ import annotations

import math

import numpy as np

MASK64 = (1 << 64) - 1


def cv_rng_subsets(n, iters, model_points=5):
    """ptsetreg.cpp getSubset with cv::RNG(-1): idx[iters][model_points]."""
    st = MASK64
    out = np.zeros((iters, model_points), dtype=np.int64)
    for it in range(iters):
        i = 0
        while i < model_points:
            while True:
                st = ((st & 0xffffffff) * 4164903690 + (st >> 32)) & MASK64
                v = (st & 0xffffffff) % n
                if v not in out[it, :i]:
                    break
            out[it, i] = v
            i += 1
    return out


def ransac_update_num_iters(p, ep, model_points, max_iters):
    p = min(max(p, 0.0), 1.0)
    ep = min(max(ep, 0.0), 1.0)
    num = max(1.0 - p, np.finfo(np.float64).tiny)
    denom = 1.0 - (1.0 - ep) ** model_points
    if denom < np.finfo(np.float64).tiny:
        return 0
    num, denom = math.log(num), math.log(denom)
    return max_iters if (denom >= 0 or -num >= max_iters * (-denom)) else int(np.rint(num / denom))


def epnp(pw, uv, K):
    """epnp.cpp compute_pose: pw [n,3], uv [n,2] pixels, K 3x3 -> (R 3x3, t 3)."""
    fu, fv, uc, vc = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    pw = np.asarray(pw, dtype=np.float64)
    uv = np.asarray(uv, dtype=np.float64)
    n = len(pw)
    c0 = pw.mean(0)
    d = pw - c0
    _, dc, uct = np.linalg.svd(d.T @ d)
    # canonical principal-axis signs (largest-magnitude component positive): EPnP's algebraic
    # error depends on them, and OpenCV's cvSVD sign convention is not reproducible here
    sgn = np.sign(uct[np.arange(3), np.abs(uct).argmax(1)])
    uct = uct * np.where(sgn == 0, 1.0, sgn)[:, None]
    k = np.sqrt(np.maximum(dc, 0) / n)
    cws = np.vstack([c0, c0 + k[:, None] * uct])
    cc = (cws[1:] - c0).T
    ci = np.linalg.pinv(cc)
    al = np.empty((n, 4))
    al[:, 1:] = d @ ci.T
    al[:, 0] = 1 - al[:, 1:].sum(1)
    M = np.zeros((2 * n, 12))
    M[0::2, 0::3] = al * fu
    M[0::2, 2::3] = al * (uc - uv[:, :1])
    M[1::2, 1::3] = al * fv
    M[1::2, 2::3] = al * (vc - uv[:, 1:])
    _, _, ut = np.linalg.svd(M.T @ M)
    v = [ut[11], ut[10], ut[9], ut[8]]
    pairs = [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]
    dv = [[vi[3 * a:3 * a + 3] - vi[3 * b:3 * b + 3] for a, b in pairs] for vi in v]
    L = np.zeros((6, 10))
    for j in range(6):
        a0, a1, a2, a3 = dv[0][j], dv[1][j], dv[2][j], dv[3][j]
        L[j] = [a0 @ a0, 2 * a0 @ a1, a1 @ a1, 2 * a0 @ a2, 2 * a1 @ a2, a2 @ a2, 2 * a0 @ a3, 2 * a1 @ a3,
                2 * a2 @ a3, a3 @ a3]
    rho = np.array([np.sum((cws[a] - cws[b]) ** 2) for a, b in pairs])

    def lsq(A, b):
        return np.linalg.lstsq(A, b, rcond=None)[0]

    def gauss_newton(betas):
        betas = np.array(betas, dtype=np.float64)
        for _ in range(5):
            b0, b1, b2, b3 = betas
            A = np.stack([2 * L[:, 0] * b0 + L[:, 1] * b1 + L[:, 3] * b2 + L[:, 6] * b3,
                          L[:, 1] * b0 + 2 * L[:, 2] * b1 + L[:, 4] * b2 + L[:, 7] * b3,
                          L[:, 3] * b0 + L[:, 4] * b1 + 2 * L[:, 5] * b2 + L[:, 8] * b3,
                          L[:, 6] * b0 + L[:, 7] * b1 + L[:, 8] * b2 + 2 * L[:, 9] * b3], 1)
            quad = (L[:, 0] * b0 * b0 + L[:, 1] * b0 * b1 + L[:, 2] * b1 * b1 + L[:, 3] * b0 * b2 + L[:, 4] * b1 * b2
                    + L[:, 5] * b2 * b2 + L[:, 6] * b0 * b3 + L[:, 7] * b1 * b3 + L[:, 8] * b2 * b3
                    + L[:, 9] * b3 * b3)
            betas = betas + lsq(A, rho - quad)
        return betas

    cands = []
    b4 = lsq(L[:, [0, 1, 3, 6]], rho)  # approx 1
    s = math.sqrt(abs(b4[0]))
    cands.append([s, *(-b4[1:] / s)] if b4[0] < 0 else [s, *(b4[1:] / s)])
    b3 = lsq(L[:, :3], rho)  # approx 2
    if b3[0] < 0:
        bb = [math.sqrt(-b3[0]), math.sqrt(-b3[2]) if b3[2] < 0 else 0.0]
    else:
        bb = [math.sqrt(b3[0]), math.sqrt(b3[2]) if b3[2] > 0 else 0.0]
    if b3[1] < 0:
        bb[0] = -bb[0]
    cands.append([bb[0], bb[1], 0.0, 0.0])
    b5 = lsq(L[:, :5], rho)  # approx 3
    if b5[0] < 0:
        bb = [math.sqrt(-b5[0]), math.sqrt(-b5[2]) if b5[2] < 0 else 0.0]
    else:
        bb = [math.sqrt(b5[0]), math.sqrt(b5[2]) if b5[2] > 0 else 0.0]
    if b5[1] < 0:
        bb[0] = -bb[0]
    cands.append([bb[0], bb[1], b5[3] / bb[0], 0.0])

    best = None
    for betas in cands:
        betas = gauss_newton(betas)
        ccs = sum(betas[i] * v[i] for i in range(4)).reshape(4, 3)
        pcs = al @ ccs
        if pcs[0, 2] < 0:  # solve_for_sign
            ccs, pcs = -ccs, -pcs
        pc0, pw0 = pcs.mean(0), pw.mean(0)
        abt = (pcs - pc0).T @ (pw - pw0)
        U, _, Vt = np.linalg.svd(abt)
        R = U @ Vt
        if np.linalg.det(R) < 0:
            R[2] = -R[2]
        t = pc0 - R @ pw0
        Xc = pw @ R.T + t
        iz = 1.0 / Xc[:, 2]
        ue = uc + fu * Xc[:, 0] * iz
        ve = vc + fv * Xc[:, 1] * iz
        err = np.sqrt((uv[:, 0] - ue) ** 2 + (uv[:, 1] - ve) ** 2).sum() / n
        if best is None or err < best[0]:  # N = 1; if (err2 < err1) N = 2; if (err3 < errN) N = 3
            best = (err, R, t)
    return best[1], best[2]


def ransac_err(R, t, pw_f32, uv_f32, K):
    """PnPRansacCallback::computeError: f64 projection stored as f32, f32 squared distance."""
    Xc = pw_f32.astype(np.float64) @ R.T + t
    z = np.where(Xc[:, 2] != 0, 1.0 / np.where(Xc[:, 2] != 0, Xc[:, 2], 1.0), 1.0)
    pu = (Xc[:, 0] * z * K[0, 0] + K[0, 2]).astype(np.float32)
    pv = (Xc[:, 1] * z * K[1, 1] + K[1, 2]).astype(np.float32)
    du = uv_f32[:, 0] - pu
    dv = uv_f32[:, 1] - pv
    return du * du + dv * dv


def solve_pnp_ransac(pw, uv, K, iterations=150, reprojection_error=2.0, confidence=0.99):
    """-> dict(success, R, t, best, inliers, good[iterations]) for one crop."""
    pw = np.asarray(pw, dtype=np.float32)
    uv = np.asarray(uv, dtype=np.float32)
    n = len(pw)
    mp = 5
    if n < mp:
        return {"success": False}
    subsets = cv_rng_subsets(n, iterations, mp)
    thr2 = np.float32(reprojection_error * reprojection_error)
    niters, maxgood, best, best_model = iterations, 0, -1, None
    good = np.full(iterations, -1)
    it = 0
    while it < niters:
        idx = subsets[it]
        R, t = epnp(pw[idx], uv[idx], K)
        if np.all(np.isfinite(R)) and np.all(np.isfinite(t)):
            g = int((ransac_err(R, t, pw, uv, K) <= thr2).sum())
            good[it] = g
            if g > max(maxgood, mp - 1):
                best, maxgood, best_model = it, g, (R, t)
                niters = ransac_update_num_iters(confidence, (n - g) / n, mp, niters)
        it += 1
    if best < 0:
        return {"success": False, "good": good}
    inl = ransac_err(best_model[0], best_model[1], pw, uv, K) <= thr2
    R, t = epnp(pw[inl], uv[inl], K)
    return {"success": True, "R": R, "t": t, "best": best, "inliers": int(inl.sum()), "good": good,
            "hyp": best_model}
