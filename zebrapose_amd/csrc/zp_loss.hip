// Training losses of ZebraPose on gfx950 (f64 where the reference is f64).
//
// Reference (lyltc1/ZebraPose, model/BinaryCodeNet.py):
//   HammingLoss :100-109   h_new[i] = sum |round(sigmoid(code_i)) - round(gt_i)| * m / (sum m + 1)
//   BinaryCodeLoss :34-67  EMA h <- 0.05 h_new + 0.95 h (first call: h = h_new);
//                          w = exp(3 * min(h, 0.51 - h));  z = m * code   (m: f64 host mask bits)
//   BinaryLossWeighted :76-81  loss_b = sum_i w_i * mean_{b,y,x} BCEWithLogits(z, gt)_i / sum_i w_i
//   MaskLoss :89-93        loss_m = mean |sigmoid(mask) - gt_mask|   (f32)
//   train_v6.py:325-335    m = from_output_to_class_mask(mask) (f64 0/1), loss = 3 loss_b + loss_m
// m and gt arrive as f64 in the reference, so loss_b and d loss_b / d code are f64 computations;
// the per-bit sums are accumulated in f64 (deterministic two-pass block reduction).
#include <math.h>
#include "zp_common.h"

namespace zp {

constexpr float kHalf = 8.940696716308594e-08f;  // CPU fp32 sigmoid(x) > 0.5  <=>  x > kHalf
constexpr int LOSS_MAXL = 32;

__device__ __forceinline__ double bce_logits(double x, double t) {
  // ATen: (1 - t) * x - log_sigmoid(x),  log_sigmoid(x) = min(x, 0) - log1p(exp(-|x|))
  double ls = fmin(x, 0.0) - log1p(exp(-fabs(x)));
  return (1.0 - t) * x - ls;
}

__device__ __forceinline__ double block_sum(double v, double* sh) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return sh[0] + sh[1] + sh[2] + sh[3];
}

__device__ __forceinline__ double mask_value(const double* m01, const float* mlog, long e) {
  if (m01) {
    double v = rint(m01[e]);  // round().clamp(0, 1) (HammingLoss :102; half-to-even like torch.round)
    return v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v);
  }
  return mlog[e] > kHalf ? 1.0 : 0.0;
}

__device__ __forceinline__ double gt_value(const void* gt, int gt_f64, size_t idx) {
  if (gt_f64) return ((const double*)gt)[idx];
  return ((const uint8_t*)gt)[idx] ? 1.0 : 0.0;
}

// per block: [0..L) hamming, [L..2L) bce, [2L] mask sum
__device__ __forceinline__ double wave_sum(double v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

__global__ void __launch_bounds__(256) k_code_partials(const float* __restrict__ clog, const double* __restrict__ m01,
                                                       const float* __restrict__ mlog, const void* __restrict__ gt,
                                                       int gt_f64, int B, int L, int HW, int mask_code,
                                                       double* __restrict__ part) {
  // (round 5) every value is wave-summed into its own LDS slot per wave and the 2L+1 block sums are
  // taken after one barrier (the per-value block_sum paid two barriers each, 66 per block); the sums
  // and their order (wave xor tree, then waves 0+1+2+3) are block_sum's, so the partials are unchanged
  __shared__ double sh[4][2 * LOSS_MAXL + 1];
  const long N = (long)B * HW;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const int nv = 2 * L + 1;
  const int w = threadIdx.x >> 6;
  const bool lead = (threadIdx.x & 63) == 0;
  double m = 0, mraw = 0;
  long b = 0, p = 0;
  const bool ok = e < N;
  if (ok) {
    b = e / HW;
    p = e - b * HW;
    m = mask_value(m01, mlog, e);                 // HammingLoss: mask.round().clamp(0, 1)
    mraw = m01 ? m01[e] : m;                      // BinaryCodeLoss :47-48 multiplies by the raw mask
  }
  constexpr int LB = 8;  // bits per batch: their loads are issued before any use
  for (int i0 = 0; i0 < L; i0 += LB) {
    float zb[LB];
    double gb[LB];
#pragma unroll
    for (int k = 0; k < LB; ++k) {
      const int i = i0 + k;
      const size_t idx = ((size_t)b * L + i) * HW + p;
      zb[k] = (ok && i < L) ? clog[idx] : 0.f;
      gb[k] = (ok && i < L) ? gt_value(gt, gt_f64, idx) : 0.0;
    }
#pragma unroll
    for (int k = 0; k < LB; ++k) {
      const int i = i0 + k;
      if (i >= L) break;
      double h = 0, c = 0;
      if (ok) {
        const float z = zb[k];
        const double graw = gb[k];
        double t2 = rint(graw);
        t2 = t2 < 0.0 ? 0.0 : (t2 > 1.0 ? 1.0 : t2);
        double bit = z > kHalf ? 1.0 : 0.0;
        h = fabs(bit - t2) * m;
        double zz = mask_code ? mraw * (double)z : (double)z;
        c = bce_logits(zz, graw);
      }
      h = wave_sum(h);
      c = wave_sum(c);
      if (lead) {
        sh[w][i] = h;
        sh[w][L + i] = c;
      }
    }
  }
  m = wave_sum(m);
  if (lead) sh[w][2 * L] = m;
  __syncthreads();
  const int j = threadIdx.x;
  if (j < nv) part[(size_t)blockIdx.x * nv + j] = sh[0][j] + sh[1][j] + sh[2][j] + sh[3][j];
}

// column sums of the per-block partials: one block per column (same summation order as a
// single block walking the columns, so the result is unchanged and deterministic)
__global__ void __launch_bounds__(256) k_code_colsum(const double* __restrict__ part, int nblk, int nv,
                                                     double* __restrict__ tot) {
  __shared__ double sh[4];
  const int j = blockIdx.x;
  double s = 0;
  for (int k = threadIdx.x; k < nblk; k += 256) s += part[(size_t)k * nv + j];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) tot[j] = s;
}

// per-bit work (EMA histogram, weight exp) on lane i < L, the sums serially on lane 0 in bit order
// (the reference's summation order)
__global__ void __launch_bounds__(64) k_code_finalize(const double* __restrict__ tot, int B, int L, int HW,
                                                      int use_hist, double* __restrict__ hist,
                                                      double* __restrict__ out, double* __restrict__ coef) {
  __shared__ double sw[LOSS_MAXL], shn[LOSS_MAXL];
  const int i = threadIdx.x;
  const double msum = tot[2 * L];
  const bool first = hist[L] == 0.0;
  if (i < L) {
    const double hn = tot[i] / (msum + 1.0);
    shn[i] = hn;
    if (use_hist) {
      const double h = first ? hn : hn * 0.05 + hist[i] * 0.95;
      hist[i] = h;
      sw[i] = exp(fmin(h, 0.51 - h) * 3.0);
    } else {
      sw[i] = 1.0;
    }
  }
  __syncthreads();
  if (i == 0) {
    const double N = (double)B * HW;
    double wsum = 0, hmean = 0, lb = 0;
    for (int k = 0; k < L; ++k) {
      hmean += shn[k];
      wsum += sw[k];
    }
    if (use_hist) hist[L] = 1.0;
    for (int k = 0; k < L; ++k) lb += (tot[L + k] / N) * sw[k];
    out[0] = lb / wsum;
    out[1] = hmean / L;
    shn[0] = wsum;  // hn no longer needed
  }
  __syncthreads();
  if (i < L) coef[i] = sw[i] / shn[0] / ((double)B * HW);
}

__global__ void k_code_grad(const float* __restrict__ clog, const double* __restrict__ m01,
                            const float* __restrict__ mlog, const void* __restrict__ gt, int gt_f64, int B, int L,
                            int HW, int mask_code, const double* __restrict__ coef, const double* __restrict__ gs,
                            float* __restrict__ dcode) {
  const long N = (long)B * HW;
  const double scale = gs ? gs[0] : 1.0;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < N; e += (long)gridDim.x * blockDim.x) {
    long b = e / HW, p = e - b * HW;
    const double m = mask_code ? (m01 ? m01[e] : (mlog[e] > kHalf ? 1.0 : 0.0)) : 1.0;
    for (int i = 0; i < L; ++i) {
      size_t idx = ((size_t)b * L + i) * HW + p;
      double z = m * (double)clog[idx];
      double t = gt_value(gt, gt_f64, idx);
      double sgm = 1.0 / (1.0 + exp(-z));
      dcode[idx] = (float)(scale * coef[i] * (sgm - t) * m);
    }
  }
}

__global__ void __launch_bounds__(256) k_mask_partials(const float* __restrict__ x, const float* __restrict__ g, long n,
                                                       double* __restrict__ part) {
  __shared__ double sh[4];
  double s = 0;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    float sg = 1.f / (1.f + expf(-x[e]));
    s += fabsf(sg - g[e]);
  }
  s = block_sum(s, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_mask_finalize(const double* __restrict__ part, int nblk, long n,
                                                       float* __restrict__ out) {
  __shared__ double sh[4];
  double s = 0;
  for (int k = threadIdx.x; k < nblk; k += 256) s += part[k];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) out[0] = (float)(s / (double)n);
}

__global__ void k_mask_grad(const float* __restrict__ x, const float* __restrict__ g, long n, const float* __restrict__ gs,
                            float* __restrict__ dx) {
  const float scale = gs ? gs[0] : 1.f;
  const float invn = 1.f / (float)n;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    float s = 1.f / (1.f + expf(-x[e]));
    float d = s - g[e];
    float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
    dx[e] = scale * sgn * invn * ((1.f - s) * s);  // l1_loss backward, then sigmoid backward
  }
}

static int mask_blocks(long n) {
  long b = (n + 255) / 256;
  return (int)(b > 1024 ? 1024 : (b < 1 ? 1 : b));
}

}  // namespace zp

using namespace zp;

extern "C" long long zp_code_loss_ws_bytes(int B, int L, int H, int W) {
  long long N = (long long)B * H * W;
  return ((N + 255) / 256) * (2LL * L + 1) * 8 + (2LL * LOSS_MAXL + 1) * 8 + 64;
}

extern "C" int zp_code_loss(const float* code_logits, const double* mask01, const float* mask_logits, const void* gt,
                            int gt_f64, int B, int L, int H, int W, int use_hist, int mask_code, double* hist_state,
                            double* out, double* coef, void* ws, void* stream) {
  ZP_CHECK_ARG(code_logits && gt && hist_state && out && coef && ws && (mask01 || mask_logits || !mask_code),
               "zp_code_loss: null pointer");
  ZP_CHECK_ARG(B > 0 && L >= 1 && L <= LOSS_MAXL && H > 0 && W > 0, "zp_code_loss: bad sizes");
  const int HW = H * W;
  const long N = (long)B * HW;
  const int nblk = (int)((N + 255) / 256);
  hipStream_t st = (hipStream_t)stream;
  double* part = (double*)ws;
  hipLaunchKernelGGL(k_code_partials, dim3(nblk), dim3(256), 0, st, code_logits, mask01, mask_logits, gt, gt_f64, B, L,
                     HW, mask_code, part);
  ZP_LAUNCH_CHECK("zp_code_loss partials");
  const int nv = 2 * L + 1;
  double* tot = part + (size_t)nblk * nv;
  hipLaunchKernelGGL(k_code_colsum, dim3(nv), dim3(256), 0, st, (const double*)part, nblk, nv, tot);
  ZP_LAUNCH_CHECK("zp_code_loss colsum");
  hipLaunchKernelGGL(k_code_finalize, dim3(1), dim3(64), 0, st, (const double*)tot, B, L, HW, use_hist, hist_state,
                     out, coef);
  ZP_LAUNCH_CHECK("zp_code_loss finalize");
  return ZP_OK;
}

extern "C" int zp_code_loss_bwd(const float* code_logits, const double* mask01, const float* mask_logits, const void* gt,
                                int gt_f64, int B, int L, int H, int W, int mask_code, const double* coef,
                                const double* grad_scale, float* dcode, void* stream) {
  ZP_CHECK_ARG(code_logits && gt && coef && dcode && (mask01 || mask_logits || !mask_code),
               "zp_code_loss_bwd: null pointer");
  const long N = (long)B * H * W;
  long g = (N + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(k_code_grad, dim3((int)g), dim3(256), 0, (hipStream_t)stream, code_logits, mask01, mask_logits, gt,
                     gt_f64, B, L, H * W, mask_code, coef, grad_scale, dcode);
  ZP_LAUNCH_CHECK("zp_code_loss_bwd");
  return ZP_OK;
}

extern "C" long long zp_mask_loss_ws_bytes(long long n) { return (long long)mask_blocks((long)n) * 8 + 64; }

extern "C" int zp_mask_loss(const float* x, const float* g, long long n, float* out, void* ws, void* stream) {
  ZP_CHECK_ARG(x && g && out && ws && n > 0, "zp_mask_loss: bad args");
  const int nb = mask_blocks((long)n);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_mask_partials, dim3(nb), dim3(256), 0, st, x, g, (long)n, (double*)ws);
  ZP_LAUNCH_CHECK("zp_mask_loss partials");
  hipLaunchKernelGGL(k_mask_finalize, dim3(1), dim3(256), 0, st, (const double*)ws, nb, (long)n, out);
  ZP_LAUNCH_CHECK("zp_mask_loss finalize");
  return ZP_OK;
}

extern "C" int zp_mask_loss_bwd(const float* x, const float* g, long long n, const float* grad_scale, float* dx,
                                void* stream) {
  ZP_CHECK_ARG(x && g && dx && n > 0, "zp_mask_loss_bwd: bad args");
  long gb = (n + 255) / 256;
  if (gb > 8192) gb = 8192;
  hipLaunchKernelGGL(k_mask_grad, dim3((int)gb), dim3(256), 0, (hipStream_t)stream, x, g, (long)n, grad_scale, dx);
  ZP_LAUNCH_CHECK("zp_mask_loss_bwd");
  return ZP_OK;
}
