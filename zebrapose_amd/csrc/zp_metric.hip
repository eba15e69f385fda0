// ADD / ADI pose errors on the device, batched over crops.
// Reference: metric.py:8-18 (Calculate_ADD_Error_BOP / Calculate_ADI_Error_BOP) ->
// bop_toolkit pose_error.add / adi, restated in lib/pysixd/pose_error.py:297-336:
//   ADD = mean_i || (R_e p_i + t_e) - (R_g p_i + t_g) ||
//   ADI = mean_i min_j || (R_g p_i + t_g) - (R_e p_j + t_e) ||   (cKDTree nearest neighbour)
// f64 throughout (the reference transforms in numpy f64).  ADI is an exact brute-force nearest
// neighbour search: one block per (crop, 256 ground-truth points), estimated points streamed
// through LDS in tiles.
#include <math.h>
#include "zp_common.h"

namespace zp {

__device__ __forceinline__ void xform(const double* R, const double* t, const float* p, double* o) {
  const double x = p[0], y = p[1], z = p[2];
  o[0] = R[0] * x + R[1] * y + R[2] * z + t[0];
  o[1] = R[3] * x + R[4] * y + R[5] * z + t[1];
  o[2] = R[6] * x + R[7] * y + R[8] * z + t[2];
}

// partial sums per (crop, block) -> ws[b][blk]; reduced in a fixed order by k_metric_final
__global__ void __launch_bounds__(256) k_add(const float* __restrict__ pts, int n, const double* __restrict__ Re,
                                             const double* __restrict__ te, const double* __restrict__ Rg,
                                             const double* __restrict__ tg, double* __restrict__ ws) {
  const int b = blockIdx.y;
  __shared__ double red[256];
  double s = 0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    double a[3], g[3];
    xform(Re + 9 * b, te + 3 * b, pts + 3 * (size_t)i, a);
    xform(Rg + 9 * b, tg + 3 * b, pts + 3 * (size_t)i, g);
    const double dx = a[0] - g[0], dy = a[1] - g[1], dz = a[2] - g[2];
    s += sqrt(dx * dx + dy * dy + dz * dz);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) ws[(size_t)b * gridDim.x + blockIdx.x] = red[0];
}

constexpr int ADI_TILE = 1024;
__global__ void __launch_bounds__(256) k_adi(const float* __restrict__ pts, int n, const double* __restrict__ Re,
                                             const double* __restrict__ te, const double* __restrict__ Rg,
                                             const double* __restrict__ tg, double* __restrict__ ws) {
  const int b = blockIdx.y;
  __shared__ double tile[3][ADI_TILE];
  __shared__ double red[256];
  const int i = blockIdx.x * 256 + threadIdx.x;
  double g[3] = {0, 0, 0};
  if (i < n) xform(Rg + 9 * b, tg + 3 * b, pts + 3 * (size_t)i, g);
  double best = INFINITY;
  for (int j0 = 0; j0 < n; j0 += ADI_TILE) {
    __syncthreads();
    for (int j = threadIdx.x; j < ADI_TILE; j += 256) {
      double e[3] = {INFINITY, INFINITY, INFINITY};
      if (j0 + j < n) xform(Re + 9 * b, te + 3 * b, pts + 3 * (size_t)(j0 + j), e);
      tile[0][j] = e[0];
      tile[1][j] = e[1];
      tile[2][j] = e[2];
    }
    __syncthreads();
    const int m = min(ADI_TILE, n - j0);
    for (int j = 0; j < m; ++j) {
      const double dx = g[0] - tile[0][j], dy = g[1] - tile[1][j], dz = g[2] - tile[2][j];
      best = fmin(best, dx * dx + dy * dy + dz * dz);
    }
  }
  red[threadIdx.x] = i < n ? sqrt(best) : 0.0;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) ws[(size_t)b * gridDim.x + blockIdx.x] = red[0];
}

__global__ void k_metric_final(const double* __restrict__ ws, int parts, int n, double* __restrict__ out, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double s = 0;
  for (int k = 0; k < parts; ++k) s += ws[(size_t)b * parts + k];
  out[b] = s / n;
}

}  // namespace zp

using namespace zp;

extern "C" long long zp_pose_error_ws_bytes(int B, int n, int mode) {
  if (B <= 0 || n <= 0) return -1;
  const int parts = mode == ZP_METRIC_ADI ? (n + 255) / 256 : min(64, (n + 255) / 256);
  return (long long)B * parts * 8;
}

extern "C" int zp_pose_error(int B, const float* pts, int n, const double* R_est, const double* t_est,
                             const double* R_gt, const double* t_gt, int mode, double* out, void* ws, void* stream) {
  ZP_CHECK_ARG(B > 0 && n > 0 && pts && R_est && t_est && R_gt && t_gt && out && ws, "zp_pose_error: bad args");
  ZP_CHECK_ARG(mode == ZP_METRIC_ADD || mode == ZP_METRIC_ADI, "zp_pose_error: mode %d", mode);
  hipStream_t st = (hipStream_t)stream;
  int parts;
  if (mode == ZP_METRIC_ADI) {
    parts = (n + 255) / 256;
    hipLaunchKernelGGL(k_adi, dim3(parts, B), dim3(256), 0, st, pts, n, R_est, t_est, R_gt, t_gt, (double*)ws);
  } else {
    parts = min(64, (n + 255) / 256);
    hipLaunchKernelGGL(k_add, dim3(parts, B), dim3(256), 0, st, pts, n, R_est, t_est, R_gt, t_gt, (double*)ws);
  }
  ZP_LAUNCH_CHECK("zp_pose_error");
  hipLaunchKernelGGL(k_metric_final, dim3((B + 63) / 64), dim3(64), 0, st, (const double*)ws, parts, n, out, B);
  ZP_LAUNCH_CHECK("zp_pose_error final");
  return ZP_OK;
}
