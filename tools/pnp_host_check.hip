// Host-side check of the device EPnP math (zp_pnp.hip's ZP_HD functions run on the CPU):
//   tools/pnp_host_check <in.bin> <out.bin>
// in:  int n, int m_hyp; double K[4]; float pw[n][3]; float uv[n][2]; int idx[m_hyp][5];
//      int nin; int inl[nin]
// out: double hyp[m_hyp][12]; double refined[12]
// (tests/test_pnp_host.py compares against oracle/pnp_ref.py; no GPU involved)
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "../zebrapose_amd/csrc/zp_pnp.hip"
namespace zp {
void set_error(const char*, ...) {}  // the library's error slot lives in zp_misc.hip
}

int main(int argc, char** argv) {
  if (argc != 3) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  int n, mh;
  double Kv[4];
  if (fread(&n, 4, 1, f) != 1 || fread(&mh, 4, 1, f) != 1 || fread(Kv, 8, 4, f) != 4) return 3;
  std::vector<float> pw(3 * n), uv(2 * n);
  std::vector<int> idx(5 * mh);
  if (fread(pw.data(), 4, 3 * n, f) != (size_t)3 * n || fread(uv.data(), 4, 2 * n, f) != (size_t)2 * n) return 3;
  if (fread(idx.data(), 4, 5 * mh, f) != (size_t)5 * mh) return 3;
  int nin;
  if (fread(&nin, 4, 1, f) != 1) return 3;
  std::vector<int> inl(nin);
  if (fread(inl.data(), 4, nin, f) != (size_t)nin) return 3;
  fclose(f);
  const zp::Cam K{Kv[0], Kv[1], Kv[2], Kv[3]};
  std::vector<double> out(12 * mh + 12);
  for (int h = 0; h < mh; ++h) {
    double p[5][3], u[5], v[5];
    for (int i = 0; i < 5; ++i) {
      const int j = idx[5 * h + i];
      for (int k = 0; k < 3; ++k) p[i][k] = pw[3 * j + k];
      u[i] = uv[2 * j];
      v[i] = uv[2 * j + 1];
    }
    zp::epnp_small(5, p, u, v, K, &out[12 * h], &out[12 * h + 9]);
  }
  // refinement over the given inliers, same sufficient statistics as k_pnp_refine
  double mean[3] = {0, 0, 0}, sc[9] = {0};
  for (int q = 0; q < nin; ++q)
    for (int k = 0; k < 3; ++k) mean[k] += pw[3 * inl[q] + k];
  for (int k = 0; k < 3; ++k) mean[k] /= nin;
  for (int q = 0; q < nin; ++q)
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) sc[r * 3 + c] += (pw[3 * inl[q] + r] - mean[r]) * (pw[3 * inl[q] + c] - mean[c]);
  double cws[12], ci[9], a0[4], s3[94] = {0};
  zp::epnp_control(mean, sc, (double)nin, cws, ci);
  for (int q = 0; q < nin; ++q) {
    const int j = inl[q];
    double p[3] = {pw[3 * j], pw[3 * j + 1], pw[3 * j + 2]}, al[4];
    zp::epnp_alphas(p, cws, ci, al);
    if (q == 0)
      for (int k = 0; k < 4; ++k) a0[k] = al[k];
    zp::epnp_accum(al, uv[2 * j], uv[2 * j + 1], K, s3);
    for (int jj = 0; jj < 4; ++jj) {
      s3[78 + jj] += al[jj];
      for (int k = 0; k < 3; ++k) s3[82 + 3 * jj + k] += al[jj] * p[k];
    }
  }
  double ccs[36], cand[3][12], e[3] = {0, 0, 0};
  zp::epnp_betas(s3, cws, ccs);
  for (int N = 0; N < 3; ++N) zp::epnp_pose(ccs + 12 * N, a0, s3 + 82, s3 + 78, mean, (double)nin, cand[N], cand[N] + 9);
  for (int q = 0; q < nin; ++q) {
    const int j = inl[q];
    double p[3] = {pw[3 * j], pw[3 * j + 1], pw[3 * j + 2]};
    for (int N = 0; N < 3; ++N) e[N] += zp::reproj_dist(cand[N], cand[N] + 9, p, uv[2 * j], uv[2 * j + 1], K);
  }
  int N = 0;
  if (e[1] < e[0]) N = 1;
  if (e[2] < e[N]) N = 2;
  for (int k = 0; k < 12; ++k) out[12 * mh + k] = cand[N][k];
  fprintf(stderr, "refine candidates err %.9g %.9g %.9g -> %d\n", e[0] / nin, e[1] / nin, e[2] / nin, N);
  FILE* g = fopen(argv[2], "wb");
  fwrite(out.data(), 8, out.size(), g);
  fclose(g);
  return 0;
}
