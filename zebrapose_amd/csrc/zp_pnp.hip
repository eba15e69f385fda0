// Batched RANSAC-EPnP on the device: the pose step that consumes the decode's
// 2D-3D correspondences.  Reference call: binary_code_helper/CNN_output_to_pose.py:152-156,
//   cv2.solvePnPRansac(P3D f32, P2D f32, K, None, reprojectionError=2, iterationsCount=150,
//                      flags=cv2.SOLVEPNP_EPNP)   (confidence: OpenCV default 0.99)
// followed by cv2.Rodrigues.  OpenCV is a third-party dependency absent from the image; this file
// restates the published algorithms it runs (OpenCV 4.x):
//   ptsetreg.cpp  RANSACPointSetRegistrator::run / getSubset / RANSACUpdateNumIters, cv::RNG(-1)
//   solvepnp.cpp  solvePnPRansac: 5-point EPnP hypotheses (PnPRansacCallback), squared float
//                 reprojection error <= thr^2, final EPnP over all inliers
//   epnp.cpp      Lepetit, Moreno-Noguer, Fua 2009: control points, barycentric coordinates,
//                 M^T M null space, beta approximations 1/2/3 + 5 Gauss-Newton steps, Procrustes
// Subsets come from OpenCV's own generator sequence, so for the same correspondences the
// hypotheses are the ones OpenCV draws; all geometry is f64.
//
// Kernels (one launch each, stream-ordered, no host sync):
//   k_pnp_subsets  thread per crop: cv::RNG draws -> idx[b][it][5]
//   k_pnp_hyp      thread per (crop, iteration): EPnP on the 5-point subset -> model[b][it]
//   k_pnp_score    block per (crop, iteration): inlier count over all correspondences
//   k_pnp_select   thread per crop: the sequential RANSAC scan (adaptive iteration count)
//   k_pnp_refine   block per crop: EPnP over the best model's inliers (block reductions)
#include <math.h>
#include <stdlib.h>
#include "zp_common.h"

// the linear algebra and EPnP pieces are host + device code (tools/pnp_host_check.hip runs them
// on the CPU against oracle/pnp_ref.py)
#define ZP_HD __host__ __device__

namespace zp {

// ------------------------------------------------------------------ small dense linear algebra
// cyclic Jacobi eigen-decomposition of a symmetric n x n matrix (row-major, destroyed);
// evals descending, evecs rows = eigenvectors (the CV_SVD_U_T convention for a PSD matrix)
template <int N>
ZP_HD void sym_eig(double* A, double* evals, double* evecs) {
  double V[N * N];
  for (int i = 0; i < N * N; ++i) V[i] = (i / N == i % N) ? 1.0 : 0.0;
  // rotate while an off-diagonal entry is not negligible against ITS OWN diagonal pair
  // (|a_pq| <= 1e-17 sqrt|a_pp a_qq|): the small eigenpairs -- EPnP's null space -- then come out
  // to relative precision, not only to precision relative to the largest eigenvalue
  for (int sweep = 0; sweep < 60; ++sweep) {
    bool rotated = false;
    for (int p = 0; p < N - 1; ++p)
      for (int q = p + 1; q < N; ++q) {
        const double apq = A[p * N + q];
        if (fabs(apq) <= 1e-17 * sqrt(fabs(A[p * N + p] * A[q * N + q])) || apq == 0.0) continue;
        rotated = true;
        const double theta = (A[q * N + q] - A[p * N + p]) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < N; ++k) {  // columns p, q
          const double akp = A[k * N + p], akq = A[k * N + q];
          A[k * N + p] = c * akp - s * akq;
          A[k * N + q] = s * akp + c * akq;
        }
        for (int k = 0; k < N; ++k) {  // rows p, q
          const double apk = A[p * N + k], aqk = A[q * N + k];
          A[p * N + k] = c * apk - s * aqk;
          A[q * N + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < N; ++k) {
          const double vkp = V[k * N + p], vkq = V[k * N + q];
          V[k * N + p] = c * vkp - s * vkq;
          V[k * N + q] = s * vkp + c * vkq;
        }
      }
    if (!rotated) break;
  }
  int ord[N];
  for (int i = 0; i < N; ++i) ord[i] = i;
  for (int i = 0; i < N; ++i)  // selection sort, descending
    for (int j = i + 1; j < N; ++j)
      if (A[ord[j] * N + ord[j]] > A[ord[i] * N + ord[i]]) {
        const int t = ord[i];
        ord[i] = ord[j];
        ord[j] = t;
      }
  for (int i = 0; i < N; ++i) {
    evals[i] = A[ord[i] * N + ord[i]];
    for (int k = 0; k < N; ++k) evecs[i * N + k] = V[k * N + ord[i]];
  }
}

// min-norm least squares x = argmin |A x - b| for A (R x C), R >= C, via the pseudo-inverse of
// A^T A (cvSolve(..., CV_SVD) semantics for the well-posed systems EPnP builds)
template <int R, int C>
ZP_HD void lsq(const double* A, const double* b, double* x) {
  double AtA[C * C], Atb[C], ev[C], evec[C * C];
  for (int i = 0; i < C; ++i) {
    Atb[i] = 0;
    for (int r = 0; r < R; ++r) Atb[i] += A[r * C + i] * b[r];
    for (int j = 0; j < C; ++j) {
      double s = 0;
      for (int r = 0; r < R; ++r) s += A[r * C + i] * A[r * C + j];
      AtA[i * C + j] = s;
    }
  }
  // Cholesky of A^T A (cheap, registers); only a (numerically) singular system takes the
  // eigen-decomposition pseudo-inverse below
  {
    double Lc[C * C];
    bool pd = true;
    double dmax = 0;
    for (int i = 0; i < C; ++i) dmax = fmax(dmax, AtA[i * C + i]);
    for (int i = 0; i < C && pd; ++i)
      for (int j = 0; j <= i; ++j) {
        double s = AtA[i * C + j];
        for (int k = 0; k < j; ++k) s -= Lc[i * C + k] * Lc[j * C + k];
        if (i == j) {
          if (!(s > 1e-13 * dmax)) {
            pd = false;
            break;
          }
          Lc[i * C + i] = sqrt(s);
        } else {
          Lc[i * C + j] = s / Lc[j * C + j];
        }
      }
    if (pd) {
      double y[C];
      for (int i = 0; i < C; ++i) {
        double s = Atb[i];
        for (int k = 0; k < i; ++k) s -= Lc[i * C + k] * y[k];
        y[i] = s / Lc[i * C + i];
      }
      for (int i = C - 1; i >= 0; --i) {
        double s = y[i];
        for (int k = i + 1; k < C; ++k) s -= Lc[k * C + i] * x[k];
        x[i] = s / Lc[i * C + i];
      }
      return;
    }
  }
  sym_eig<C>(AtA, ev, evec);
  const double tol = ev[0] * 1e-15;
  for (int i = 0; i < C; ++i) x[i] = 0;
  for (int k = 0; k < C; ++k) {
    if (ev[k] <= tol) continue;
    double p = 0;
    for (int i = 0; i < C; ++i) p += evec[k * C + i] * Atb[i];
    p /= ev[k];
    for (int i = 0; i < C; ++i) x[i] += p * evec[k * C + i];
  }
}

// R = U V^T from the SVD of the 3x3 ABt (Procrustes, epnp.cpp estimate_R_and_t); the
// det < 0 fix negates R's last row exactly as epnp.cpp does
ZP_HD void procrustes(const double* abt, double* Rm) {
  double AtA[9], ev[3], V[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s = 0;
      for (int k = 0; k < 3; ++k) s += abt[k * 3 + i] * abt[k * 3 + j];
      AtA[i * 3 + j] = s;
    }
  sym_eig<3>(AtA, ev, V);  // rows of V: right singular vectors, descending
  double U[9];             // columns u_k = ABt v_k / s_k
  for (int k = 0; k < 3; ++k) {
    double u[3];
    for (int i = 0; i < 3; ++i) u[i] = abt[i * 3 + 0] * V[k * 3 + 0] + abt[i * 3 + 1] * V[k * 3 + 1] + abt[i * 3 + 2] * V[k * 3 + 2];
    double n = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
    if (k == 2 && n <= 1e-12 * (sqrt(fabs(ev[0])) + 1e-300)) {  // rank 2: u2 = u0 x u1
      const double ax = U[0], ay = U[3], az = U[6], bx = U[1], by = U[4], bz = U[7];
      u[0] = ay * bz - az * by;
      u[1] = az * bx - ax * bz;
      u[2] = ax * by - ay * bx;
      n = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
    }
    for (int i = 0; i < 3; ++i) U[i * 3 + k] = n > 0 ? u[i] / n : 0.0;
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Rm[i * 3 + j] = U[i * 3 + 0] * V[0 * 3 + j] + U[i * 3 + 1] * V[1 * 3 + j] + U[i * 3 + 2] * V[2 * 3 + j];
  const double det = Rm[0] * Rm[4] * Rm[8] + Rm[1] * Rm[5] * Rm[6] + Rm[2] * Rm[3] * Rm[7] - Rm[2] * Rm[4] * Rm[6] -
                     Rm[1] * Rm[3] * Rm[8] - Rm[0] * Rm[5] * Rm[7];
  if (det < 0) {
    Rm[6] = -Rm[6];
    Rm[7] = -Rm[7];
    Rm[8] = -Rm[8];
  }
}

// ------------------------------------------------------------------ EPnP pieces (epnp.cpp)
struct Cam {
  double fu, fv, uc, vc;
};

// control points from the points' mean and scatter matrix (choose_control_points) and the
// inverse of CC = [c1-c0 c2-c0 c3-c0] (compute_barycentric_coordinates, SVD pseudo-inverse)
ZP_HD void epnp_control(const double* mean, const double* scatter, double n, double* cws, double* ccinv) {
  double S[9], dc[3], uct[9];
  for (int i = 0; i < 9; ++i) S[i] = scatter[i];
  sym_eig<3>(S, dc, uct);
  // EPnP's algebraic error depends on which way each principal axis points (c0 +- k u), so the
  // sign is fixed canonically: largest-magnitude component positive (OpenCV's cvSVD sign
  // convention cannot be reproduced without OpenCV; oracle/pnp_ref.py applies the same rule)
  for (int i = 0; i < 3; ++i) {
    int m = 0;
    for (int j = 1; j < 3; ++j)
      if (fabs(uct[i * 3 + j]) > fabs(uct[i * 3 + m])) m = j;
    if (uct[i * 3 + m] < 0)
      for (int j = 0; j < 3; ++j) uct[i * 3 + j] = -uct[i * 3 + j];
  }
  for (int j = 0; j < 3; ++j) cws[j] = mean[j];
  double kk[3], kmax = 0;
  for (int i = 0; i < 3; ++i) {
    kk[i] = sqrt(fmax(dc[i], 0.0) / n);
    kmax = fmax(kmax, kk[i]);
    for (int j = 0; j < 3; ++j) cws[(i + 1) * 3 + j] = mean[j] + kk[i] * uct[i * 3 + j];
  }
  // CC(i, j) = k_j uct[j][i]  ->  CC^+ = diag(1 / k) Uct
  for (int j = 0; j < 3; ++j)
    for (int i = 0; i < 3; ++i) ccinv[j * 3 + i] = kk[j] > 1e-12 * kmax ? uct[j * 3 + i] / kk[j] : 0.0;
}

ZP_HD inline void epnp_alphas(const double* pw, const double* cws, const double* ci, double* a) {
  const double d0 = pw[0] - cws[0], d1 = pw[1] - cws[1], d2 = pw[2] - cws[2];
  for (int j = 0; j < 3; ++j) a[1 + j] = ci[3 * j] * d0 + ci[3 * j + 1] * d1 + ci[3 * j + 2] * d2;
  a[0] = 1.0 - a[1] - a[2] - a[3];
}

// the point's two rows of M, added into the upper triangle of M^T M (78 entries, row-major
// i <= j packed as in tri_index)
ZP_HD inline int tri_index(int i, int j) { return i * 12 - i * (i - 1) / 2 + (j - i); }
ZP_HD inline void epnp_accum(const double* a, double u, double v, const Cam& K, double* mtm) {
  double m1[12], m2[12];
  for (int j = 0; j < 4; ++j) {
    m1[3 * j] = a[j] * K.fu;
    m1[3 * j + 1] = 0.0;
    m1[3 * j + 2] = a[j] * (K.uc - u);
    m2[3 * j] = 0.0;
    m2[3 * j + 1] = a[j] * K.fv;
    m2[3 * j + 2] = a[j] * (K.vc - v);
  }
  for (int i = 0; i < 12; ++i)
    for (int j = i; j < 12; ++j) mtm[tri_index(i, j)] += m1[i] * m1[j] + m2[i] * m2[j];
}

// null space -> three candidate control-point sets in the camera frame (betas approximations
// 1/2/3, each refined by 5 Gauss-Newton steps): ccs[3][4][3]
// v4: the eigenvectors of the 4 smallest eigenvalues of M^T M, smallest first (epnp.cpp's
// ut rows 11, 10, 9, 8)
ZP_HD void epnp_betas_null(const double* v4, const double* cws, double* ccs_out) {
  const double* v[4] = {v4, v4 + 12, v4 + 24, v4 + 36};
  double dv[4][6][3];
  for (int i = 0; i < 4; ++i) {
    int a = 0, b = 1;
    for (int j = 0; j < 6; ++j) {
      for (int k = 0; k < 3; ++k) dv[i][j][k] = v[i][3 * a + k] - v[i][3 * b + k];
      if (++b > 3) {
        ++a;
        b = a + 1;
      }
    }
  }
  auto dot3 = [](const double* x, const double* y) { return x[0] * y[0] + x[1] * y[1] + x[2] * y[2]; };
  double L[60];
  for (int j = 0; j < 6; ++j) {
    double* r = L + 10 * j;
    r[0] = dot3(dv[0][j], dv[0][j]);
    r[1] = 2.0 * dot3(dv[0][j], dv[1][j]);
    r[2] = dot3(dv[1][j], dv[1][j]);
    r[3] = 2.0 * dot3(dv[0][j], dv[2][j]);
    r[4] = 2.0 * dot3(dv[1][j], dv[2][j]);
    r[5] = dot3(dv[2][j], dv[2][j]);
    r[6] = 2.0 * dot3(dv[0][j], dv[3][j]);
    r[7] = 2.0 * dot3(dv[1][j], dv[3][j]);
    r[8] = 2.0 * dot3(dv[2][j], dv[3][j]);
    r[9] = dot3(dv[3][j], dv[3][j]);
  }
  auto d2 = [&](int a, int b) {
    const double x = cws[3 * a] - cws[3 * b], y = cws[3 * a + 1] - cws[3 * b + 1], z = cws[3 * a + 2] - cws[3 * b + 2];
    return x * x + y * y + z * z;
  };
  const double rho[6] = {d2(0, 1), d2(0, 2), d2(0, 3), d2(1, 2), d2(1, 3), d2(2, 3)};
  for (int N = 1; N <= 3; ++N) {
    double betas[4] = {0, 0, 0, 0};
    if (N == 1) {  // find_betas_approx_1: B11 B12 B13 B14
      double A[24], b4[4];
      for (int i = 0; i < 6; ++i) {
        A[i * 4 + 0] = L[i * 10 + 0];
        A[i * 4 + 1] = L[i * 10 + 1];
        A[i * 4 + 2] = L[i * 10 + 3];
        A[i * 4 + 3] = L[i * 10 + 6];
      }
      lsq<6, 4>(A, rho, b4);
      if (b4[0] < 0) {
        betas[0] = sqrt(-b4[0]);
        betas[1] = -b4[1] / betas[0];
        betas[2] = -b4[2] / betas[0];
        betas[3] = -b4[3] / betas[0];
      } else {
        betas[0] = sqrt(b4[0]);
        betas[1] = b4[1] / betas[0];
        betas[2] = b4[2] / betas[0];
        betas[3] = b4[3] / betas[0];
      }
    } else if (N == 2) {  // find_betas_approx_2: B11 B12 B22
      double A[18], b3[3];
      for (int i = 0; i < 6; ++i)
        for (int k = 0; k < 3; ++k) A[i * 3 + k] = L[i * 10 + k];
      lsq<6, 3>(A, rho, b3);
      if (b3[0] < 0) {
        betas[0] = sqrt(-b3[0]);
        betas[1] = (b3[2] < 0) ? sqrt(-b3[2]) : 0.0;
      } else {
        betas[0] = sqrt(b3[0]);
        betas[1] = (b3[2] > 0) ? sqrt(b3[2]) : 0.0;
      }
      if (b3[1] < 0) betas[0] = -betas[0];
    } else {  // find_betas_approx_3: B11 B12 B22 B13 B23
      double A[30], b5[5];
      for (int i = 0; i < 6; ++i)
        for (int k = 0; k < 5; ++k) A[i * 5 + k] = L[i * 10 + k];
      lsq<6, 5>(A, rho, b5);
      if (b5[0] < 0) {
        betas[0] = sqrt(-b5[0]);
        betas[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0;
      } else {
        betas[0] = sqrt(b5[0]);
        betas[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0;
      }
      if (b5[1] < 0) betas[0] = -betas[0];
      betas[2] = b5[3] / betas[0];
    }
    for (int it = 0; it < 5; ++it) {  // gauss_newton
      double A[24], bb[6], X[4];
      const double b0 = betas[0], b1 = betas[1], b2 = betas[2], b3 = betas[3];
      for (int i = 0; i < 6; ++i) {
        const double* r = L + 10 * i;
        A[i * 4 + 0] = 2 * r[0] * b0 + r[1] * b1 + r[3] * b2 + r[6] * b3;
        A[i * 4 + 1] = r[1] * b0 + 2 * r[2] * b1 + r[4] * b2 + r[7] * b3;
        A[i * 4 + 2] = r[3] * b0 + r[4] * b1 + 2 * r[5] * b2 + r[8] * b3;
        A[i * 4 + 3] = r[6] * b0 + r[7] * b1 + r[8] * b2 + 2 * r[9] * b3;
        bb[i] = rho[i] - (r[0] * b0 * b0 + r[1] * b0 * b1 + r[2] * b1 * b1 + r[3] * b0 * b2 + r[4] * b1 * b2 +
                          r[5] * b2 * b2 + r[6] * b0 * b3 + r[7] * b1 * b3 + r[8] * b2 * b3 + r[9] * b3 * b3);
      }
      lsq<6, 4>(A, bb, X);
      for (int k = 0; k < 4; ++k) betas[k] += X[k];
    }
    double* ccs = ccs_out + (N - 1) * 12;  // compute_ccs
    for (int k = 0; k < 12; ++k) ccs[k] = 0.0;
    for (int i = 0; i < 4; ++i)
      for (int k = 0; k < 12; ++k) ccs[k] += betas[i] * v[i][k];
  }
}

ZP_HD void epnp_betas(const double* mtm_tri, const double* cws, double* ccs_out) {
  double MtM[144], D[12], ut[144];
  for (int i = 0; i < 12; ++i)
    for (int j = i; j < 12; ++j) MtM[i * 12 + j] = MtM[j * 12 + i] = mtm_tri[tri_index(i, j)];
  sym_eig<12>(MtM, D, ut);
  double v4[48];
  for (int i = 0; i < 4; ++i)
    for (int k = 0; k < 12; ++k) v4[12 * i + k] = ut[12 * (11 - i) + k];
  epnp_betas_null(v4, cws, ccs_out);
}

// compute_R_and_t from the camera-frame control points, given the sufficient statistics of the
// points: a0 = alphas of the FIRST point (solve_for_sign), Aw[j] = sum_i alpha_ij pw_i,
// sa[j] = sum_i alpha_ij, pw0 = mean of pw, n
ZP_HD void epnp_pose(double* ccs, const double* a0, const double* Aw, const double* sa, const double* pw0, double n,
                          double* Rm, double* t) {
  double z0 = 0;
  for (int j = 0; j < 4; ++j) z0 += a0[j] * ccs[3 * j + 2];
  if (z0 < 0)
    for (int k = 0; k < 12; ++k) ccs[k] = -ccs[k];
  double pc0[3] = {0, 0, 0};
  for (int j = 0; j < 4; ++j)
    for (int k = 0; k < 3; ++k) pc0[k] += sa[j] * ccs[3 * j + k];
  for (int k = 0; k < 3; ++k) pc0[k] /= n;
  // ABt = sum_i (pc_i - pc0)(pw_i - pw0)^T = sum_j ccs_j Aw_j^T - n pc0 pw0^T
  double abt[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      double s = 0;
      for (int j = 0; j < 4; ++j) s += ccs[3 * j + r] * Aw[3 * j + c];
      abt[r * 3 + c] = s - n * pc0[r] * pw0[c];
    }
  procrustes(abt, Rm);
  for (int r = 0; r < 3; ++r) t[r] = pc0[r] - (Rm[r * 3] * pw0[0] + Rm[r * 3 + 1] * pw0[1] + Rm[r * 3 + 2] * pw0[2]);
}

ZP_HD inline double reproj_dist(const double* Rm, const double* t, const double* pw, double u, double v,
                                              const Cam& K) {
  const double Xc = Rm[0] * pw[0] + Rm[1] * pw[1] + Rm[2] * pw[2] + t[0];
  const double Yc = Rm[3] * pw[0] + Rm[4] * pw[1] + Rm[5] * pw[2] + t[1];
  const double inv = 1.0 / (Rm[6] * pw[0] + Rm[7] * pw[1] + Rm[8] * pw[2] + t[2]);
  const double ue = K.uc + K.fu * Xc * inv, ve = K.vc + K.fv * Yc * inv;
  return sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
}

// squared reprojection error the way PnPRansacCallback::computeError measures it: projection in
// f64 stored as f32 (projectPoints output), difference and square in f32
ZP_HD inline float ransac_err(const double* Rm, const double* t, const float* pw, float u, float v,
                                            const Cam& K) {
  const double X = pw[0], Y = pw[1], Z = pw[2];
  const double Xc = Rm[0] * X + Rm[1] * Y + Rm[2] * Z + t[0];
  const double Yc = Rm[3] * X + Rm[4] * Y + Rm[5] * Z + t[1];
  const double Zc = Rm[6] * X + Rm[7] * Y + Rm[8] * Z + t[2];
  const double inv = Zc != 0 ? 1.0 / Zc : 1.0;  // projectPoints: x = X * (1 / Z); u = x * fx + cx
  const float pu = (float)(Xc * inv * K.fu + K.uc), pv = (float)(Yc * inv * K.fv + K.vc);
  const float du = u - pu, dv = v - pv;
  return du * du + dv * dv;
}

// ------------------------------------------------------------------ kernels
struct PnpArgs {
  int B, HW, iters, model_points;
  const int* counts;   // [B]
  const int* xy;       // [B][HW][2] original-image pixels
  const float* xyz;    // [B][HW][3]
  const double* K;     // [B][4] (fu, fv, uc, vc)
  float thr2;          // reprojection error^2 (f32, as findInliers)
  double confidence;
  int* idx;            // [B][iters][5]
  int* nsub;           // [B] subsets drawn (0: RANSAC cannot run)
  double* model;       // [B][iters][12] (R row-major, t)
  int* mvalid;         // [B][iters]
  int* good;           // [B][iters]
  int* best;           // [B] best iteration (-1 none)
  int* maxgood;        // [B] the running RANSAC scan: inliers of the best model so far
  int* niters;         // [B] its current iteration bound (RANSACUpdateNumIters)
  int it0, it1;        // the chunk of iterations a hyp / score / select launch covers
  double* R;           // [B][9]
  double* T;           // [B][3]
  int* success;        // [B]
  int* ninl;           // [B]
};

// cv::RNG(0xffffffffffffffff): state = (u64)(u32)state * 4164903690 + (state >> 32); next() = (u32)state;
// uniform(0, n) = next() % n.  getSubset: redraw an index already in the subset; every subset
// accepted (PnPRansacCallback has no checkSubset).
__global__ void k_pnp_subsets(const PnpArgs a) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  const int n = a.counts[b];
  if (n < a.model_points) {
    a.nsub[b] = 0;
    return;
  }
  unsigned long long st = 0xffffffffffffffffull;
  int* out = a.idx + (size_t)b * a.iters * 5;
  for (int it = 0; it < a.iters; ++it) {
    int cur[5];
    for (int i = 0; i < 5; ++i) {
      int v;
      for (;;) {
        st = (unsigned long long)(unsigned)st * 4164903690ull + (unsigned)(st >> 32);
        v = (int)((unsigned)st % (unsigned)n);
        bool dup = false;
#pragma unroll
        for (int j = 0; j < 5; ++j) dup |= (j < i) && cur[j] == v;
        if (!dup) break;
      }
#pragma unroll
      for (int j = 0; j < 5; ++j)
        if (j == i) cur[j] = v;
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) out[it * 5 + i] = cur[i];
  }
  a.nsub[b] = a.iters;
}

__device__ __forceinline__ void load_pt(const PnpArgs& a, int b, int i, double* pw, double* u, double* v) {
  const float* p = a.xyz + ((size_t)b * a.HW + i) * 3;
  const int* q = a.xy + ((size_t)b * a.HW + i) * 2;
  pw[0] = p[0];
  pw[1] = p[1];
  pw[2] = p[2];
  *u = (double)(float)q[0];
  *v = (double)(float)q[1];
}

// EPnP pose of m <= 5 correspondences (one RANSAC hypothesis); false if not finite
ZP_HD bool epnp_small(int m, const double (*pw)[3], const double* uu, const double* vv, const Cam& K, double* outR,
                      double* outT) {
  double mean[3] = {0, 0, 0};
  for (int i = 0; i < m; ++i)
    for (int k = 0; k < 3; ++k) mean[k] += pw[i][k];
  for (int k = 0; k < 3; ++k) mean[k] /= m;
  double sc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < m; ++i)
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) sc[r * 3 + c] += (pw[i][r] - mean[r]) * (pw[i][c] - mean[c]);
  double cws[12], ci[9];
  epnp_control(mean, sc, (double)m, cws, ci);
  double mtm[78];
  for (int k = 0; k < 78; ++k) mtm[k] = 0;
  double al[5][4], Aw[12], sa[4] = {0, 0, 0, 0};
  for (int k = 0; k < 12; ++k) Aw[k] = 0;
  for (int i = 0; i < m; ++i) {
    epnp_alphas(pw[i], cws, ci, al[i]);
    epnp_accum(al[i], uu[i], vv[i], K, mtm);
    for (int j = 0; j < 4; ++j) {
      sa[j] += al[i][j];
      for (int k = 0; k < 3; ++k) Aw[3 * j + k] += al[i][j] * pw[i][k];
    }
  }
  double ccs[36];
  epnp_betas(mtm, cws, ccs);
  double bestE = 0;
  for (int N = 0; N < 3; ++N) {
    double Rm[9], t[3];
    epnp_pose(ccs + 12 * N, al[0], Aw, sa, mean, (double)m, Rm, t);
    double e = 0;
    for (int i = 0; i < m; ++i) e += reproj_dist(Rm, t, pw[i], uu[i], vv[i], K);
    e /= m;
    if (N == 0 || e < bestE) {  // epnp.cpp: N = 1; if (err2 < err1) N = 2; if (err3 < errN) N = 3
      bestE = e;
      for (int k = 0; k < 9; ++k) outR[k] = Rm[k];
      for (int k = 0; k < 3; ++k) outT[k] = t[k];
    }
  }
  bool ok = isfinite(bestE);
  for (int k = 0; k < 9; ++k) ok = ok && isfinite(outR[k]);
  for (int k = 0; k < 3; ++k) ok = ok && isfinite(outT[k]);
  return ok;
}

// Parallel cyclic Jacobi on the symmetric 12x12 A (LDS), eigenvectors accumulated in V (LDS,
// columns): threads 0..63 of the block work (6 disjoint rotations per round, circle-method
// pairing, 11 rounds per sweep), every thread of the block takes part in the barriers.
__device__ void par_jacobi12(double* A, double* V, double (*cs)[2], int* rotated) {
  const int lane = threadIdx.x;
  const bool worker = lane < 64;
  if (worker)
    for (int e = lane; e < 144; e += 64) V[e] = (e / 12 == e % 12) ? 1.0 : 0.0;
  __syncthreads();
  for (int sweep = 0; sweep < 40; ++sweep) {
    if (lane == 0) *rotated = 0;
    __syncthreads();
    for (int r = 0; r < 11; ++r) {
      if (lane < 6) {
        const int p = lane == 0 ? 11 : (r + lane) % 11;
        const int q = lane == 0 ? r : (r - lane + 11) % 11;
        const double apq = A[p * 12 + q], app = A[p * 12 + p], aqq = A[q * 12 + q];
        double c = 1.0, sn = 0.0;
        if (!(fabs(apq) <= 1e-17 * sqrt(fabs(app * aqq)) || apq == 0.0)) {
          const double theta = (aqq - app) / (2.0 * apq);
          const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
          c = 1.0 / sqrt(t * t + 1.0);
          sn = t * c;
          *rotated = 1;
        }
        cs[lane][0] = c;
        cs[lane][1] = sn;
      }
      __syncthreads();
      if (worker)
        for (int job = lane; job < 72; job += 64) {  // rows p, q of the 6 pairs
          const int k = job / 12, j = job % 12;
          const int p = k == 0 ? 11 : (r + k) % 11, q = k == 0 ? r : (r - k + 11) % 11;
          const double c = cs[k][0], sn = cs[k][1];
          const double ap = A[p * 12 + j], aq = A[q * 12 + j];
          A[p * 12 + j] = c * ap - sn * aq;
          A[q * 12 + j] = sn * ap + c * aq;
        }
      __syncthreads();
      if (worker)
        for (int job = lane; job < 72; job += 64) {  // columns p, q, and V
          const int k = job / 12, i = job % 12;
          const int p = k == 0 ? 11 : (r + k) % 11, q = k == 0 ? r : (r - k + 11) % 11;
          const double c = cs[k][0], sn = cs[k][1];
          const double ap = A[i * 12 + p], aq = A[i * 12 + q];
          A[i * 12 + p] = c * ap - sn * aq;
          A[i * 12 + q] = sn * ap + c * aq;
          const double vp = V[i * 12 + p], vq = V[i * 12 + q];
          V[i * 12 + p] = c * vp - sn * vq;
          V[i * 12 + q] = sn * vp + c * vq;
        }
      __syncthreads();
    }
    if (!*rotated) break;
  }
}

// the 4 eigenvectors of the smallest eigenvalues (diagonal of the rotated A), smallest first
__device__ void null4(const double* A, const double* V, double* v4) {
  int ord[12];
  for (int i = 0; i < 12; ++i) ord[i] = i;
  for (int i = 0; i < 12; ++i)
    for (int j = i + 1; j < 12; ++j)
      if (A[ord[j] * 12 + ord[j]] > A[ord[i] * 12 + ord[i]]) {
        const int t = ord[i];
        ord[i] = ord[j];
        ord[j] = t;
      }
  for (int i = 0; i < 4; ++i)
    for (int k = 0; k < 12; ++k) v4[12 * i + k] = V[k * 12 + ord[11 - i]];
}

// One wave per hypothesis: lane 0 builds M^T M from the 5-point subset, the 64 lanes run a
// parallel cyclic Jacobi on it (6 disjoint rotations per round, circle-method pairing, 11 rounds
// per sweep) with the matrix in LDS, lane 0 finishes EPnP from the 4-vector null space.  (A
// thread-per-hypothesis version spent ~8 ms of serial scratch traffic in the 12x12 Jacobi.)
__global__ void __launch_bounds__(64) k_pnp_hyp(const PnpArgs a) {
  const int b = blockIdx.y, it = a.it0 + blockIdx.x, lane = threadIdx.x;
  // early termination: the scan of the chunks before this one already bounds the crop's RANSAC
  // loop below this iteration (the bound only shrinks), so it is never evaluated
  if (it >= a.niters[b]) return;
  __shared__ double A[144], V[144], cs[6][2];
  __shared__ double pw[5][3], uu[5], vv[5], cws[12], al[5][4], Aw[12], sa[4], mean[3];
  __shared__ int skip, rotated;
  const size_t mi = (size_t)b * a.iters + it;
  const Cam K{a.K[b * 4], a.K[b * 4 + 1], a.K[b * 4 + 2], a.K[b * 4 + 3]};
  const int m = a.model_points;
  if (lane == 0) {
    skip = a.nsub[b] == 0;
    if (!skip) {
      const int* id = a.idx + mi * 5;
      for (int i = 0; i < m; ++i) load_pt(a, b, id[i], pw[i], &uu[i], &vv[i]);
      double mn[3] = {0, 0, 0}, sc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, ci[9], mtm[78];
      for (int i = 0; i < m; ++i)
        for (int k = 0; k < 3; ++k) mn[k] += pw[i][k];
      for (int k = 0; k < 3; ++k) mean[k] = mn[k] / m;
      for (int i = 0; i < m; ++i)
        for (int r = 0; r < 3; ++r)
          for (int c = 0; c < 3; ++c) sc[r * 3 + c] += (pw[i][r] - mean[r]) * (pw[i][c] - mean[c]);
      double cw[12];
      epnp_control(mean, sc, (double)m, cw, ci);
      for (int k = 0; k < 12; ++k) cws[k] = cw[k];
      for (int k = 0; k < 78; ++k) mtm[k] = 0;
      for (int k = 0; k < 12; ++k) Aw[k] = 0;
      for (int j = 0; j < 4; ++j) sa[j] = 0;
      for (int i = 0; i < m; ++i) {
        double p[3] = {pw[i][0], pw[i][1], pw[i][2]}, al_i[4];
        epnp_alphas(p, cw, ci, al_i);
        epnp_accum(al_i, uu[i], vv[i], K, mtm);
        for (int j = 0; j < 4; ++j) {
          al[i][j] = al_i[j];
          sa[j] += al_i[j];
          for (int k = 0; k < 3; ++k) Aw[3 * j + k] += al_i[j] * p[k];
        }
      }
      for (int i = 0; i < 12; ++i)
        for (int j = i; j < 12; ++j) A[i * 12 + j] = A[j * 12 + i] = mtm[tri_index(i, j)];
    }
  }
  __syncthreads();
  if (skip) {
    if (lane == 0) a.mvalid[mi] = 0;
    return;
  }
  par_jacobi12(A, V, cs, &rotated);
  if (lane != 0) return;
  double v4[48], cw[12];
  null4(A, V, v4);
  for (int k = 0; k < 12; ++k) cw[k] = cws[k];
  double ccs[36];
  epnp_betas_null(v4, cw, ccs);
  double a0[4] = {al[0][0], al[0][1], al[0][2], al[0][3]}, aw[12], s4[4] = {sa[0], sa[1], sa[2], sa[3]};
  double mn[3] = {mean[0], mean[1], mean[2]};
  for (int k = 0; k < 12; ++k) aw[k] = Aw[k];
  double* md = a.model + mi * 12;
  double bestE = 0;
  for (int N = 0; N < 3; ++N) {
    double Rm[9], t[3];
    epnp_pose(ccs + 12 * N, a0, aw, s4, mn, (double)m, Rm, t);
    double e = 0;
    for (int i = 0; i < m; ++i) {
      const double p[3] = {pw[i][0], pw[i][1], pw[i][2]};
      e += reproj_dist(Rm, t, p, uu[i], vv[i], K);
    }
    e /= m;
    if (N == 0 || e < bestE) {
      bestE = e;
      for (int k = 0; k < 9; ++k) md[k] = Rm[k];
      for (int k = 0; k < 3; ++k) md[9 + k] = t[k];
    }
  }
  bool ok = isfinite(bestE);
  for (int k = 0; k < 12; ++k) ok = ok && isfinite(md[k]);
  a.mvalid[mi] = ok ? 1 : 0;
}

__global__ void __launch_bounds__(256) k_pnp_score(const PnpArgs a) {
  const int b = blockIdx.y, it = a.it0 + blockIdx.x;
  if (it >= a.niters[b]) return;
  __shared__ int red[256];
  const size_t mi = (size_t)b * a.iters + it;
  const int n = a.counts[b];
  int c = 0;
  if (a.nsub[b] != 0 && a.mvalid[mi]) {
    const Cam K{a.K[b * 4], a.K[b * 4 + 1], a.K[b * 4 + 2], a.K[b * 4 + 3]};
    const double* md = a.model + mi * 12;
    double Rm[9], t[3];
    for (int k = 0; k < 9; ++k) Rm[k] = md[k];
    for (int k = 0; k < 3; ++k) t[k] = md[9 + k];
    for (int i = threadIdx.x; i < n; i += 256) {
      const float* p = a.xyz + ((size_t)b * a.HW + i) * 3;
      const int* q = a.xy + ((size_t)b * a.HW + i) * 2;
      c += ransac_err(Rm, t, p, (float)q[0], (float)q[1], K) <= a.thr2;
    }
  }
  red[threadIdx.x] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) a.good[mi] = red[0];
}

// RANSACUpdateNumIters (ptsetreg.cpp)
__device__ int update_num_iters(double p, double ep, int model_points, int max_iters) {
  p = fmax(p, 0.0);
  p = fmin(p, 1.0);
  ep = fmax(ep, 0.0);
  ep = fmin(ep, 1.0);
  double num = fmax(1.0 - p, 2.2250738585072014e-308);
  double denom = 1.0 - pow(1.0 - ep, (double)model_points);
  if (denom < 2.2250738585072014e-308) return 0;
  num = log(num);
  denom = log(denom);
  return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : (int)rint(num / denom);
}

// the sequential RANSAC scan (ptsetreg.cpp RANSACPointSetRegistrator::run), continued over
// iterations [it0, it1) from the state the previous chunks left (it0 == 0: fresh state)
__global__ void k_pnp_select(const PnpArgs a) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  const int n = a.counts[b];
  int best = a.it0 == 0 ? -1 : a.best[b];
  int niters = a.it0 == 0 ? a.iters : a.niters[b];
  int maxgood = a.it0 == 0 ? 0 : a.maxgood[b];
  if (a.nsub[b] != 0) {
    for (int it = a.it0; it < niters && it < a.it1; ++it) {
      const size_t mi = (size_t)b * a.iters + it;
      if (!a.mvalid[mi]) continue;
      const int g = a.good[mi];
      if (g > max(maxgood, a.model_points - 1)) {
        best = it;
        maxgood = g;
        niters = update_num_iters(a.confidence, (double)(n - g) / n, a.model_points, niters);
      }
    }
  } else {
    niters = 0;
  }
  a.best[b] = best;
  a.maxgood[b] = maxgood;
  a.niters[b] = niters;
}

__global__ void k_pnp_scan_init(const PnpArgs a) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  a.niters[b] = a.nsub[b] != 0 ? a.iters : 0;
}

// final EPnP over the best model's inliers; block per crop (4 waves), f64 block reductions:
// wave butterfly, then the 4 wave partials in a fixed order (deterministic)
template <int NV>
__device__ void block_sum(double (&v)[NV], double* sh) {
  // sh: [NV][4]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int k = 0; k < NV; ++k) {
    double x = v[k];
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
    if (lane == 0) sh[k * 4 + w] = x;
  }
  __syncthreads();
  for (int k = 0; k < NV; ++k) v[k] = ((sh[k * 4] + sh[k * 4 + 1]) + sh[k * 4 + 2]) + sh[k * 4 + 3];
  __syncthreads();
}

__global__ void __launch_bounds__(256) k_pnp_refine(const PnpArgs a) {
  const int b = blockIdx.x;
  __shared__ double sh[94 * 4];
  __shared__ double cws[12], ci[9], a0[4], ccs[36], cand[3][12];
  __shared__ int first, nin;
  const int n = a.counts[b];
  const int best = a.best[b];
  if (best < 0) {
    if (threadIdx.x == 0) {
      a.success[b] = 0;
      a.ninl[b] = 0;
      for (int k = 0; k < 9; ++k) a.R[b * 9 + k] = 0;
      for (int k = 0; k < 3; ++k) a.T[b * 3 + k] = 0;
    }
    return;
  }
  const Cam K{a.K[b * 4], a.K[b * 4 + 1], a.K[b * 4 + 2], a.K[b * 4 + 3]};
  const double* md = a.model + ((size_t)b * a.iters + best) * 12;
  double Rb[9], tb[3];
  for (int k = 0; k < 9; ++k) Rb[k] = md[k];
  for (int k = 0; k < 3; ++k) tb[k] = md[9 + k];
  auto inlier = [&](int i) {
    const float* p = a.xyz + ((size_t)b * a.HW + i) * 3;
    const int* q = a.xy + ((size_t)b * a.HW + i) * 2;
    return ransac_err(Rb, tb, p, (float)q[0], (float)q[1], K) <= a.thr2;
  };
  // pass 1: count, first inlier, mean
  if (threadIdx.x == 0) first = 0x7fffffff;
  __syncthreads();
  double s1[4] = {0, 0, 0, 0};
  int myfirst = 0x7fffffff;
  for (int i = threadIdx.x; i < n; i += 256) {
    if (!inlier(i)) continue;
    double pw[3], u, v;
    load_pt(a, b, i, pw, &u, &v);
    s1[0] += 1;
    for (int k = 0; k < 3; ++k) s1[1 + k] += pw[k];
    myfirst = min(myfirst, i);
  }
  atomicMin(&first, myfirst);
  block_sum<4>(s1, sh);
  const double cnt = s1[0];
  const double mean[3] = {s1[1] / cnt, s1[2] / cnt, s1[3] / cnt};
  // pass 2: scatter matrix
  double s2[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = threadIdx.x; i < n; i += 256) {
    if (!inlier(i)) continue;
    double pw[3], u, v;
    load_pt(a, b, i, pw, &u, &v);
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) s2[r * 3 + c] += (pw[r] - mean[r]) * (pw[c] - mean[c]);
  }
  block_sum<9>(s2, sh);
  if (threadIdx.x == 0) {
    nin = (int)cnt;
    epnp_control(mean, s2, cnt, cws, ci);
    double pw[3], u, v;
    load_pt(a, b, first, pw, &u, &v);
    epnp_alphas(pw, cws, ci, a0);
  }
  __syncthreads();
  // pass 3: M^T M (78), Aw (12), sum alphas (4)
  double s3[94];
  for (int k = 0; k < 94; ++k) s3[k] = 0;
  for (int i = threadIdx.x; i < n; i += 256) {
    if (!inlier(i)) continue;
    double pw[3], u, v, al[4];
    load_pt(a, b, i, pw, &u, &v);
    epnp_alphas(pw, cws, ci, al);
    epnp_accum(al, u, v, K, s3);
    for (int j = 0; j < 4; ++j) {
      s3[78 + j] += al[j];
      for (int k = 0; k < 3; ++k) s3[82 + 3 * j + k] += al[j] * pw[k];
    }
  }
  block_sum<94>(s3, sh);
  __shared__ double Aj[144], Vj[144], csj[6][2];
  __shared__ int rotj;
  if (threadIdx.x == 0)
    for (int i = 0; i < 12; ++i)
      for (int j = i; j < 12; ++j) Aj[i * 12 + j] = Aj[j * 12 + i] = s3[tri_index(i, j)];
  __syncthreads();
  par_jacobi12(Aj, Vj, csj, &rotj);
  if (threadIdx.x == 0) {
    double v4[48];
    null4(Aj, Vj, v4);
    epnp_betas_null(v4, cws, ccs);
    for (int N = 0; N < 3; ++N) {
      double Rm[9], t[3];
      epnp_pose(ccs + 12 * N, a0, s3 + 82, s3 + 78, mean, cnt, Rm, t);
      for (int k = 0; k < 9; ++k) cand[N][k] = Rm[k];
      for (int k = 0; k < 3; ++k) cand[N][9 + k] = t[k];
    }
  }
  __syncthreads();
  // pass 4: mean reprojection distance of the three candidates (epnp.cpp reprojection_error)
  double s4[3] = {0, 0, 0};
  for (int i = threadIdx.x; i < n; i += 256) {
    if (!inlier(i)) continue;
    double pw[3], u, v;
    load_pt(a, b, i, pw, &u, &v);
    for (int N = 0; N < 3; ++N) s4[N] += reproj_dist(cand[N], cand[N] + 9, pw, u, v, K);
  }
  block_sum<3>(s4, sh);
  if (threadIdx.x == 0) {
    int N = 0;
    if (s4[1] < s4[0]) N = 1;
    if (s4[2] < s4[N]) N = 2;
    bool ok = true;
    for (int k = 0; k < 12; ++k) ok = ok && isfinite(cand[N][k]);
    for (int k = 0; k < 9; ++k) a.R[b * 9 + k] = ok ? cand[N][k] : Rb[k];
    for (int k = 0; k < 3; ++k) a.T[b * 3 + k] = ok ? cand[N][9 + k] : tb[k];
    a.success[b] = 1;
    a.ninl[b] = nin;
  }
}

}  // namespace zp

using namespace zp;

extern "C" long long zp_pnp_ws_bytes(int B, int iters) {
  if (B <= 0 || iters <= 0) return -1;
  const long long bi = (long long)B * iters;
  return bi * 5 * 4 + (long long)B * 4 + bi * 12 * 8 + bi * 4 + bi * 4 + (long long)B * 4 * 3 + 256;
}

extern "C" int zp_pnp_ransac(int B, int HW, const int* counts, const int* xy, const float* xyz, const double* K,
                             int iters, double reproj_err, double confidence, double* R, double* T, int* success,
                             int* inliers, void* ws, void* stream) {
  ZP_CHECK_ARG(B > 0 && HW > 0 && counts && xy && xyz && K && R && T && success && inliers && ws,
               "zp_pnp_ransac: bad args");
  ZP_CHECK_ARG(iters > 0 && iters <= 100000 && reproj_err > 0 && confidence >= 0 && confidence <= 1,
               "zp_pnp_ransac: iters %d / threshold / confidence", iters);
  PnpArgs a{};
  a.B = B;
  a.HW = HW;
  a.iters = iters;
  a.model_points = 5;
  a.counts = counts;
  a.xy = xy;
  a.xyz = xyz;
  a.K = K;
  a.thr2 = (float)(reproj_err * reproj_err);
  a.confidence = confidence;
  char* p = (char*)ws;
  const size_t bi = (size_t)B * iters;
  a.model = (double*)p;      p += bi * 12 * 8;
  a.idx = (int*)p;           p += bi * 5 * 4;
  a.mvalid = (int*)p;        p += bi * 4;
  a.good = (int*)p;          p += bi * 4;
  a.nsub = (int*)p;          p += (size_t)B * 4;
  a.best = (int*)p;          p += (size_t)B * 4;
  a.maxgood = (int*)p;       p += (size_t)B * 4;
  a.niters = (int*)p;
  a.R = R;
  a.T = T;
  a.success = success;
  a.ninl = inliers;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_pnp_subsets, dim3((B + 63) / 64), dim3(64), 0, st, a);
  ZP_LAUNCH_CHECK("zp_pnp_ransac subsets");
  hipLaunchKernelGGL(k_pnp_scan_init, dim3((B + 63) / 64), dim3(64), 0, st, a);
  // hypotheses in two chunks, each followed by the scan over it: the first FIRST iterations, then
  // the rest.  A crop whose adaptive bound (RANSACUpdateNumIters) fell to <= FIRST skips the second
  // chunk (its workgroups return at once), so the device work follows OpenCV's early termination
  // (a 70%-inlier scene stops after ~25 iterations); the result is the one-pass scan's, bit for bit.
  // Worst case (random correspondences, no termination): one extra round of launches.
  // ZP_PNP_FIRST overrides FIRST (0: one chunk).
  const char* ev = getenv("ZP_PNP_FIRST");
  const int first = ev ? atoi(ev) : 32;
  for (int c0 = 0; c0 < iters;) {
    a.it0 = c0;
    a.it1 = (c0 == 0 && first > 0) ? min(iters, first) : iters;
    c0 = a.it1;
    hipLaunchKernelGGL(k_pnp_hyp, dim3(a.it1 - a.it0, B), dim3(64), 0, st, a);
    ZP_LAUNCH_CHECK("zp_pnp_ransac hypotheses");
    hipLaunchKernelGGL(k_pnp_score, dim3(a.it1 - a.it0, B), dim3(256), 0, st, a);
    ZP_LAUNCH_CHECK("zp_pnp_ransac score");
    hipLaunchKernelGGL(k_pnp_select, dim3((B + 63) / 64), dim3(64), 0, st, a);
    ZP_LAUNCH_CHECK("zp_pnp_ransac select");
  }
  hipLaunchKernelGGL(k_pnp_refine, dim3(B), dim3(256), 0, st, a);
  ZP_LAUNCH_CHECK("zp_pnp_ransac refine");
  return ZP_OK;
}
