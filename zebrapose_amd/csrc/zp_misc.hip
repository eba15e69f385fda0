// Memory-bound kernels of the ZebraPose hot path on gfx950: weight packing, batch-norm
// (eval fold, train statistics / apply / backward), pooling, layout conversion, slice
// copies, and the Adam step.  All NHWC, 16-byte vectorised (8 bf16 / 4 f32 per access).
#include <stdarg.h>
#include <stdio.h>
#include <math.h>
#include <type_traits>
#include "zp_common.h"

namespace zp {

static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// 16-byte vector of dtype T
template <typename T> struct V16;
template <> struct V16<bf16_t> {
  static constexpr int N = 8;
  static __device__ __forceinline__ void load(const bf16_t* p, float* f) {
    uint4 u = *(const uint4*)p;
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = __uint_as_float(w[i] << 16);
      f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ void store(bf16_t* p, const float* f) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
    *(uint4*)p = make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <> struct V16<f16_t> {
  static constexpr int N = 8;
  static __device__ __forceinline__ void load(const f16_t* p, float* f) {
    const f16x8 h = *(const f16x8*)p;
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = (float)h[i];
  }
  static __device__ __forceinline__ void store(f16_t* p, const float* f) {
    f16x8 h;
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = (f16_t)f[i];
    *(f16x8*)p = h;
  }
};
template <> struct V16<float> {
  static constexpr int N = 4;
  static __device__ __forceinline__ void load(const float* p, float* f) {
    float4 v = *(const float4*)p;
    f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
  }
  static __device__ __forceinline__ void store(float* p, const float* f) { *(float4*)p = make_float4(f[0], f[1], f[2], f[3]); }
};

static inline int grid_for(long n, int block = 256, int cap = 8192) {
  long g = (n + block - 1) / block;
  if (g < 1) g = 1;
  return (int)(g > cap ? cap : g);
}

// ------------------------------------------------------------------ weight packing
struct PackArgs {
  const float* src;
  void* dst;
  int d0, d1, kh, kw, transposed, ntaps, cstride, rows_pad, k_pad;
  signed char ky[ZP_MAX_TAPS], kx[ZP_MAX_TAPS];
};

template <typename T>
__global__ void k_pack(const PackArgs a) {
  const long total = (long)a.rows_pad * a.k_pad;
  const int rows = a.transposed ? a.d1 : a.d0;
  const int chans = a.transposed ? a.d0 : a.d1;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    int r = (int)(e / a.k_pad), k = (int)(e - (long)r * a.k_pad);
    int t = k / a.cstride, c = k - t * a.cstride;
    float v = 0.f;
    if (r < rows && t < a.ntaps && c < chans) {
      int ky = a.ky[t], kx = a.kx[t];
      size_t idx = a.transposed ? (((size_t)c * a.d1 + r) * a.kh + ky) * a.kw + kx
                                : (((size_t)r * a.d1 + c) * a.kh + ky) * a.kw + kx;
      v = a.src[idx];
    }
    ((T*)a.dst)[e] = Elem<T>::cvt(v);
  }
}

// split-fp32 packing (ZP_F32X3 / ZP_F32H2): the same element map as k_pack, the f32 weight split
// into NPL planes [NPL][rows_pad][k_pad] (SplitF32<NPL>)
template <int NPL>
__global__ void k_pack_split(const PackArgs a, unsigned* rflag) {
  const long total = (long)a.rows_pad * a.k_pad;
  bool bad = false;
  const int rows = a.transposed ? a.d1 : a.d0;
  const int chans = a.transposed ? a.d0 : a.d1;
  unsigned short* d = (unsigned short*)a.dst;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    int r = (int)(e / a.k_pad), k = (int)(e - (long)r * a.k_pad);
    int t = k / a.cstride, c = k - t * a.cstride;
    float v = 0.f;
    if (r < rows && t < a.ntaps && c < chans) {
      int ky = a.ky[t], kx = a.kx[t];
      size_t idx = a.transposed ? (((size_t)c * a.d1 + r) * a.kh + ky) * a.kw + kx
                                : (((size_t)r * a.d1 + c) * a.kh + ky) * a.kw + kx;
      v = a.src[idx];
    }
    unsigned short q[NPL];
    SplitF32<NPL>::split(v, q);
    if constexpr (NPL == 2) bad |= h2w_overflow(v);
#pragma unroll
    for (int p = 0; p < NPL; ++p) d[e + p * total] = q[p];
  }
  if constexpr (NPL == 2) raise_range_flag(rflag, bad);
}

// one launch for many pack jobs: blockIdx.y = job (read once, uniform), threads over the job's
// (row, channel) pairs; each thread reads its pair's kh x kw taps (contiguous in the checkpoint
// layout, so a wave reads one contiguous span) and writes them at k = t * cstride + c (adjacent
// threads -> adjacent k: coalesced 2-byte stores), then the pair's share of the k_pad tail (zeros).
// Same result as zp_pack_weight per job.
__device__ __forceinline__ void pack_store(const zp_pack_job& a, int d, float v, unsigned* rflag) {
  if (a.dtype == ZP_F32X3) {  // three planes of rows_pad * k_pad
    const size_t ps = (size_t)a.rows_pad * a.k_pad;
    unsigned short q[3];
    SplitF32<3>::split(v, q);
    for (int p = 0; p < 3; ++p) ((unsigned short*)a.dst)[d + p * ps] = q[p];
  } else if (a.dtype == ZP_F32H2) {  // two planes
    const size_t ps = (size_t)a.rows_pad * a.k_pad;
    unsigned short q[2];
    SplitF32<2>::split(v, q);
    for (int p = 0; p < 2; ++p) ((unsigned short*)a.dst)[d + p * ps] = q[p];
    raise_range_flag(rflag, h2w_overflow(v));
  } else if (a.dtype == ZP_BF16) ((bf16_t*)a.dst)[d] = f2bf(v);
  else if (a.dtype == ZP_F16) ((f16_t*)a.dst)[d] = (f16_t)v;
  else ((float*)a.dst)[d] = v;
}

// Tiled form for kh x kw <= 9 (every job but the 7x7 stem): a block stages a tile of PK_R packed
// rows x PK_C channels x the kh*kw taps in LDS with reads contiguous in the checkpoint layout (rows
// of [c][tap] for a forward packing, [r][tap] runs per channel for a transposed / data-gradient one),
// then writes each packed row's (tap, channel) run as consecutive 2-byte stores.  The per-pair form
// below it read the transposed layouts one scattered 36-byte run per lane (r02 PMC: 1.3 GB moved per
// 116 MB of weights).
constexpr int PK_R = 8, PK_C = 64, PK_ROW = PK_C * 9 + 1;  // +1: the transposed fill hits distinct banks
// KHW / NT: the job's kh * kw and tap count as compile-time constants (9 / 9: a full 3x3 forward packing;
// 9 / -9: the reversed taps of a 3x3 data-gradient packing; 1 / 1: the 1x1s), or 0 for the runtime
// values (ConvT phase sub-problems); with them a tile's loads are all issued before its LDS writes
// (one memory round trip per tile instead of one per element batch)
template <int KHW, int NT>
__device__ __forceinline__ void pack_tiled(const zp_pack_job& a, const int* toff, float* tile, unsigned* rflag) {
  const int rows = a.transposed ? a.d1 : a.d0;
  const int chans = a.transposed ? a.d0 : a.d1;
  const int khw = KHW ? KHW : a.kh * a.kw;
  const int ntaps = NT > 0 ? NT : (NT < 0 ? -NT : a.ntaps);
  const int ct = (a.cstride + PK_C - 1) / PK_C, rt = (a.rows_pad + PK_R - 1) / PK_R;
  const int kt = ntaps * a.cstride, nld = PK_R * PK_C * khw;
  for (int tl = blockIdx.x; tl < rt * ct; tl += gridDim.x) {
    const int r0 = (tl / ct) * PK_R, c0 = (tl % ct) * PK_C;
    auto elem = [&](int e, int& li) -> float {  // source element e of the tile -> its value, LDS index
      const int k = e % khw, q = e / khw;
      int rl, cl;
      if (a.transposed) {  // src[c][r][tap]: runs of consecutive r per channel
        rl = q % PK_R;
        cl = q / PK_R;
      } else {  // src[r][c][tap]: runs of consecutive c per row
        cl = q % PK_C;
        rl = q / PK_C;
      }
      const int r = r0 + rl, c = c0 + cl;
      li = rl * PK_ROW + cl * 9 + k;
      return (r < rows && c < chans) ? a.src[(a.transposed ? ((size_t)c * a.d1 + r) : ((size_t)r * a.d1 + c)) * khw + k]
                                     : 0.f;
    };
    if constexpr (KHW > 0) {
      constexpr int PER = (PK_R * PK_C * KHW + 255) / 256;
      float v[PER];
      int li[PER];
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int e = threadIdx.x + 256 * u;
        v[u] = e < nld ? elem(e, li[u]) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < PER; ++u)
        if (threadIdx.x + 256 * u < nld) tile[li[u]] = v[u];
    } else {
      for (int e = threadIdx.x; e < nld; e += blockDim.x) {
        int li;
        const float v = elem(e, li);
        tile[li] = v;
      }
    }
    __syncthreads();
    const int cw = min(PK_C, a.cstride - c0);
    for (int e = threadIdx.x; e < PK_R * ntaps * PK_C; e += blockDim.x) {
      const int cl = e % PK_C, q = e / PK_C, t = q % ntaps, rl = q / ntaps;
      const int r = r0 + rl;
      const int tk = NT == 9 && KHW == 9 ? t : (NT == -9 && KHW == 9 ? 8 - t : (NT == 1 && KHW == 1 ? 0 : toff[t]));
      if (cl < cw && r < a.rows_pad) pack_store(a, r * a.k_pad + t * a.cstride + c0 + cl, tile[rl * PK_ROW + cl * 9 + tk], rflag);
    }
    if (c0 == 0)  // the row's k_pad tail
      for (int e = threadIdx.x; e < PK_R * (a.k_pad - kt); e += blockDim.x) {
        const int rl = e / (a.k_pad - kt), kk = kt + e % (a.k_pad - kt);
        if (r0 + rl < a.rows_pad) pack_store(a, (r0 + rl) * a.k_pad + kk, 0.f, rflag);
      }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) k_pack_multi(const zp_pack_job* __restrict__ jobs, unsigned* rflag, int forms) {
  const zp_pack_job& a = jobs[blockIdx.y];
  // tap offsets in LDS (a private copy of the job's tap arrays would live in scratch)
  __shared__ int toff[ZP_MAX_TAPS];
  __shared__ float tile[PK_R * PK_ROW];
  if ((int)threadIdx.x < a.ntaps) toff[threadIdx.x] = a.ky[threadIdx.x] * a.kw + a.kx[threadIdx.x];
  __syncthreads();
  const int rows = a.transposed ? a.d1 : a.d0;
  const int chans = a.transposed ? a.d0 : a.d1;
  if (a.kh * a.kw <= 9) {
    bool ident = true, rev = true;
    for (int t = 0; t < a.ntaps; ++t) {
      ident = ident && a.ky[t] * a.kw + a.kx[t] == t;
      rev = rev && a.ky[t] * a.kw + a.kx[t] == a.ntaps - 1 - t;
    }
    if (!forms) pack_tiled<0, 0>(a, toff, tile, rflag);  // (A/B: ZP_PACK_FORMS=0)
    else if (ident && a.kh * a.kw == 9 && a.ntaps == 9) pack_tiled<9, 9>(a, toff, tile, rflag);
    else if (rev && a.kh * a.kw == 9 && a.ntaps == 9) pack_tiled<9, -9>(a, toff, tile, rflag);
    else if (ident && a.kh * a.kw == 1 && a.ntaps == 1) pack_tiled<1, 1>(a, toff, tile, rflag);
    else pack_tiled<0, 0>(a, toff, tile, rflag);
    return;
  }
  const int pairs = a.rows_pad * a.cstride;
  const int kt = a.ntaps * a.cstride, khw = a.kh * a.kw;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < pairs; q += gridDim.x * blockDim.x) {
    const int r = q / a.cstride, c = q - r * a.cstride;
    const bool live = r < rows && c < chans;
    const float* sp = a.src + (a.transposed ? ((size_t)c * a.d1 + r) : ((size_t)r * a.d1 + c)) * khw;
    const int o = r * a.k_pad + c;
    if (a.ntaps <= 9) {  // all loads in flight before the stores
      float v[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) v[t] = (live && t < a.ntaps) ? sp[toff[t]] : 0.f;
#pragma unroll
      for (int t = 0; t < 9; ++t)
        if (t < a.ntaps) pack_store(a, o + t * a.cstride, v[t], rflag);
    } else {
      for (int t = 0; t < a.ntaps; ++t) pack_store(a, o + t * a.cstride, live ? sp[toff[t]] : 0.f, rflag);
    }
    for (int kk = kt + c; kk < a.k_pad; kk += a.cstride) pack_store(a, r * a.k_pad + kk, 0.f, rflag);
  }
}

// ------------------------------------------------------------------ batch norm
__global__ void k_bn_fold(const float* g, const float* b, const float* m, const float* v, const float* bias, float eps,
                          int C, float* scale, float* shift) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  // PyTorch CPU eval: alpha = weight / sqrt(var + eps); out = in * alpha + (bias - mean * alpha)
  float inv = 1.f / sqrtf(v[c] + eps);
  float s = g[c] * inv;
  float sh = b[c] - m[c] * s;
  if (bias) sh += bias[c] * s;
  scale[c] = s;
  shift[c] = sh;
}

// Level 1 of the statistics merge: block (channel group, j) merges parts [j*R, (j+1)*R) with
// Chan's formula (f64 inside the block) and writes the merged (count, mean, M2) back in place into
// part j*R -- only this block reads that range, so the in-place write is race-free.  Level 2
// (k_bn_train_finalize) then reads every R-th part.  Two levels keep both kernels short: the
// conv epilogue emits one part per wave-half (8192 parts at 128x128, bs 32).
constexpr int BN_MERGE_R = 64;
__global__ void k_bn_stat_merge(float* __restrict__ part, int parts, int C) {
  __shared__ double sh[3][8][33];
  const int cl = threadIdx.x & 31, pl = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  const int k0 = blockIdx.y * BN_MERGE_R, k1 = min(parts, k0 + BN_MERGE_R);
  double n = 0, s = 0;
  if (c < C)
    for (int k = k0 + pl; k < k1; k += 8) {
      double nk = part[(size_t)k * C + c];
      n += nk;
      s += nk * (double)part[((size_t)parts + k) * C + c];
    }
  sh[0][pl][cl] = n;
  sh[1][pl][cl] = s;
  __syncthreads();
  double ntot = 0, stot = 0;
  for (int k = 0; k < 8; ++k) {
    ntot += sh[0][k][cl];
    stot += sh[1][k][cl];
  }
  const double mean = ntot > 0 ? stot / ntot : 0.0;
  double q = 0;
  if (c < C)
    for (int k = k0 + pl; k < k1; k += 8) {
      double nk = part[(size_t)k * C + c];
      double dm = (double)part[((size_t)parts + k) * C + c] - mean;
      q += (double)part[((size_t)2 * parts + k) * C + c] + nk * dm * dm;
    }
  sh[2][pl][cl] = q;
  __syncthreads();  // every read of this range precedes the write-back below
  if (pl != 0 || c >= C) return;
  for (int k = 1; k < 8; ++k) q += sh[2][k][cl];
  part[(size_t)k0 * C + c] = (float)ntot;
  part[((size_t)parts + k0) * C + c] = (float)mean;
  part[((size_t)2 * parts + k0) * C + c] = (float)q;
}

// Level 2 (one block = 32 channels x 8 part lanes; reads parts 0, R, 2R, ... (R = stride)):
// partials [0] count, [1] mean, [2] M2 (centred) per part, merged with Chan's formula in f64:
// n = sum n_k, mean = sum n_k mean_k / n, M2 = sum M2_k + sum n_k (mean_k - mean)^2; then the
// train-mode scale / shift, the saved statistics and the running-statistics update
struct BnFin {
  float eps, mom;
  const float *gamma, *beta, *bias;
  float *rm, *rv;
  int64_t* nbt;
  float *scale, *shift, *save;
};
__device__ __forceinline__ void bn_finalize_block(const float* __restrict__ part, int parts, int stride, int C, int cgrp,
                                                  const BnFin& f, double (&sh)[3][8][33]) {
  const int cl = threadIdx.x & 31, pl = threadIdx.x >> 5;
  const int c = cgrp * 32 + cl;
  double n = 0, s = 0;
  if (c < C)
    for (int k = pl * stride; k < parts; k += 8 * stride) {
      double nk = part[(size_t)k * C + c];
      n += nk;
      s += nk * (double)part[((size_t)parts + k) * C + c];
    }
  sh[0][pl][cl] = n;
  sh[1][pl][cl] = s;
  __syncthreads();
  double ntot = 0, stot = 0;
  for (int k = 0; k < 8; ++k) {
    ntot += sh[0][k][cl];
    stot += sh[1][k][cl];
  }
  const double mean = ntot > 0 ? stot / ntot : 0.0;
  double q = 0;
  if (c < C)
    for (int k = pl * stride; k < parts; k += 8 * stride) {
      double nk = part[(size_t)k * C + c];
      double dm = (double)part[((size_t)parts + k) * C + c] - mean;
      q += (double)part[((size_t)2 * parts + k) * C + c] + nk * dm * dm;
    }
  sh[2][pl][cl] = q;
  __syncthreads();
  if (pl != 0 || c >= C) return;
  for (int k = 1; k < 8; ++k) q += sh[2][k][cl];
  const double cntd = ntot;
  double var = cntd > 0 ? q / cntd : 0.0;
  if (var < 0) var = 0;
  float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
  float sc = f.gamma[c] * invstd;
  const float shv = __builtin_fmaf(-(float)mean, sc, f.beta[c]);
  f.scale[c] = sc;
  f.shift[c] = shv;
  f.save[c] = (float)mean;
  f.save[C + c] = invstd;
  f.save[2 * C + c] = sc;  // the backward recomputes the ReLU mask from the raw conv output
  f.save[3 * C + c] = shv;
  double mt = mean + (f.bias ? (double)f.bias[c] : 0.0);
  double unb = cntd > 1 ? var * cntd / (cntd - 1.0) : var;
  f.rm[c] = (float)((1.0 - f.mom) * f.rm[c] + f.mom * mt);
  f.rv[c] = (float)((1.0 - f.mom) * f.rv[c] + f.mom * unb);
  if (c == 0 && f.nbt) f.nbt[0] += 1;
}

__global__ void k_bn_train_finalize(const float* __restrict__ part, int parts, int stride, int C, const BnFin f) {
  __shared__ double sh[3][8][33];
  bn_finalize_block(part, parts, stride, C, blockIdx.x, f, sh);
}

// Levels 1 and 2 in one launch (round 5; VERDICT r4 #4: the training step ran ~55 merge + ~55
// finalize launches of 5-7 us).  Block (channel group x, part range y) merges its range in place as
// k_bn_stat_merge does; then the blocks of a channel group hand off through an agent-scope counter
// (cdna_hip_programming.md Guideline 16, counter form: every wave drains its stores, the block's
// barrier, one lane's release fence + drain, relaxed agent fetch_add); the block that draws the last
// ticket acquires (fence, drain, barrier) and runs level 2 over the merged parts, then re-arms the
// counter for the next launch.  Correct for any placement of the blocks over XCDs; the parts are
// merged in the same fixed order as the two-launch form, so results are bit-identical to it.
__global__ void __launch_bounds__(256) k_bn_stat_merge_fin(float* __restrict__ part, int parts, int C,
                                                           unsigned* __restrict__ cnt, const BnFin f) {
  __shared__ double sh[3][8][33];
  __shared__ int last;
  const int cl = threadIdx.x & 31, pl = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  const int k0 = blockIdx.y * BN_MERGE_R, k1 = min(parts, k0 + BN_MERGE_R);
  double n = 0, s = 0;
  if (c < C)
    for (int k = k0 + pl; k < k1; k += 8) {
      double nk = part[(size_t)k * C + c];
      n += nk;
      s += nk * (double)part[((size_t)parts + k) * C + c];
    }
  sh[0][pl][cl] = n;
  sh[1][pl][cl] = s;
  __syncthreads();
  double ntot = 0, stot = 0;
  for (int k = 0; k < 8; ++k) {
    ntot += sh[0][k][cl];
    stot += sh[1][k][cl];
  }
  const double mean = ntot > 0 ? stot / ntot : 0.0;
  double q = 0;
  if (c < C)
    for (int k = k0 + pl; k < k1; k += 8) {
      double nk = part[(size_t)k * C + c];
      double dm = (double)part[((size_t)parts + k) * C + c] - mean;
      q += (double)part[((size_t)2 * parts + k) * C + c] + nk * dm * dm;
    }
  sh[2][pl][cl] = q;
  __syncthreads();  // every read of this range precedes the write-back below
  if (pl == 0 && c < C) {
    for (int k = 1; k < 8; ++k) q += sh[2][k][cl];
    part[(size_t)k0 * C + c] = (float)ntot;
    part[((size_t)parts + k0) * C + c] = (float)mean;
    part[((size_t)2 * parts + k0) * C + c] = (float)q;
  }
  // hand-off: publish this block's merged part, count it; the last block of the group continues
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(cnt + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int l = prev == gridDim.y - 1;
    if (l) {
      __hip_atomic_store(cnt + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    last = l;
  }
  __syncthreads();
  if (!last) return;
  bn_finalize_block(part, parts, BN_MERGE_R, C, blockIdx.x, f, sh);
}

// One level for up to BN_MERGE1_MAX parts (round 5; with the strip tile's per-tile parts most layers
// of the bs 32 training step have 128): block = 8 channels x 128 part lanes, a lane's (at most 4) parts loaded once; the two passes of
// Chan's merge (n, sum n_k mean_k -> mean; sum M2_k + n_k (mean_k - mean)^2) read registers, each
// followed by a fixed pairwise tree over the 128 lanes in f64 (deterministic); then the finalize of
// bn_finalize_block.  One launch without the two-level form's counter hand-off, whose release /
// acquire fences and two dependent global passes per level held every merge near 10 us.
constexpr int BN_MERGE1_MAX = 512;
__global__ void __launch_bounds__(1024) k_bn_stat_merge1(const float* __restrict__ part, int parts, int C, const BnFin f) {
  __shared__ double sh[2][128][9];
  const int cl = threadIdx.x & 7, pl = threadIdx.x >> 3;
  const int c = blockIdx.x * 8 + cl;
  constexpr int U = BN_MERGE1_MAX / 128;
  float pn[U], pm[U], pq[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int k = pl + 128 * u;
    const bool in = c < C && k < parts;
    pn[u] = in ? part[(size_t)k * C + c] : 0.f;
    pm[u] = in ? part[((size_t)parts + k) * C + c] : 0.f;
    pq[u] = in ? part[((size_t)2 * parts + k) * C + c] : 0.f;
  }
  double n = 0, s = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    n += (double)pn[u];
    s += (double)pn[u] * (double)pm[u];
  }
  sh[0][pl][cl] = n;
  sh[1][pl][cl] = s;
  __syncthreads();
  for (int w = 64; w > 0; w >>= 1) {
    if (pl < w) {
      sh[0][pl][cl] += sh[0][pl + w][cl];
      sh[1][pl][cl] += sh[1][pl + w][cl];
    }
    __syncthreads();
  }
  const double ntot = sh[0][0][cl], stot = sh[1][0][cl];
  const double mean = ntot > 0 ? stot / ntot : 0.0;
  double q = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const double dm = (double)pm[u] - mean;
    q += (double)pq[u] + (double)pn[u] * dm * dm;  // (parts past the end: all three zero)
  }
  __syncthreads();  // every lane has read the pass-1 totals
  sh[0][pl][cl] = q;
  __syncthreads();
  for (int w = 64; w > 0; w >>= 1) {
    if (pl < w) sh[0][pl][cl] += sh[0][pl + w][cl];
    __syncthreads();
  }
  if (pl != 0 || c >= C) return;
  q = sh[0][0][cl];
  const double cntd = ntot;
  double var = cntd > 0 ? q / cntd : 0.0;
  if (var < 0) var = 0;
  float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
  float sc = f.gamma[c] * invstd;
  const float shv = __builtin_fmaf(-(float)mean, sc, f.beta[c]);
  f.scale[c] = sc;
  f.shift[c] = shv;
  f.save[c] = (float)mean;
  f.save[C + c] = invstd;
  f.save[2 * C + c] = sc;
  f.save[3 * C + c] = shv;
  double mt = mean + (f.bias ? (double)f.bias[c] : 0.0);
  double unb = cntd > 1 ? var * cntd / (cntd - 1.0) : var;
  f.rm[c] = (float)((1.0 - f.mom) * f.rm[c] + f.mom * mt);
  f.rv[c] = (float)((1.0 - f.mom) * f.rv[c] + f.mom * unb);
  if (c == 0 && f.nbt) f.nbt[0] += 1;
}

// the fused merge's hand-off counters (one per channel group) live in the caller's partials buffer,
// past the [3][parts][C] statistics (ABI 4, zp_bn_finalize_floats), and are zeroed on the launch's
// stream before the merge: every launch has its own, whatever stream or hipGraph it runs in (ADVICE
// r5: one static array per device was shared by concurrent launches on different streams)
static int g_bn_fused = -1;  // zp_conv_tuning key 15: 1 the one-launch merge, 0 two launches (-1: ZP_BN_FUSED or 1)
int bn_fused_mode(int v) {
  const int old = g_bn_fused;
  g_bn_fused = v;
  return old;
}

// N consecutive per-channel floats (16-byte aligned: c and C are multiples of N)
template <int N>
__device__ __forceinline__ void load_chan(const float* __restrict__ p, float* v) {
#pragma unroll
  for (int i = 0; i < N; i += 4) {
    const float4 q = *(const float4*)(p + i);
    v[i] = q.x;
    v[i + 1] = q.y;
    v[i + 2] = q.z;
    v[i + 3] = q.w;
  }
}

// Pixel-row tiling of the per-pixel BN passes: block = 256 threads = lanes (16-byte channel chunks,
// at most 256) x R pixel rows; blockIdx.y = channel group.  A thread keeps one channel chunk, so its
// per-channel terms are loaded once, and walks K = pix / R pixels in batches of 4 with every load
// of a batch issued before any use.
struct BnTile {
  int lanes, R, cgroups, pix, blocks;
};
static inline BnTile bn_tile(long P, int C, int N, long min_blocks = 2048) {  // k_bn_bwd_apply
  BnTile t;
  const int CV = C / N;
  t.lanes = CV < 256 ? CV : 256;
  t.R = 256 / t.lanes;
  t.cgroups = CV > 256 ? CV / 256 : 1;
  int K = 16;  // pixels per thread: fewer (down to 4) while that leaves fewer than min_blocks blocks
  while (K > 4 && ((P + (long)t.R * K - 1) / ((long)t.R * K)) * t.cgroups < min_blocks) K >>= 1;
  t.pix = t.R * K;
  t.blocks = (int)((P + t.pix - 1) / t.pix);
  return t;
}

template <typename T>
__global__ void k_bn_apply(const T* __restrict__ x, long P, int C, const float* __restrict__ scale,
                           const float* __restrict__ shift, const T* __restrict__ res, int ldr, int cr0, int relu,
                           T* __restrict__ y, int ldy, int cy0) {
  // grid-stride over 16-byte chunks (measured faster here than bn_tile's pixel-row tiling)
  constexpr int N = V16<T>::N;
  const int CV = C / N;
  const long total = P * CV;
  int cur = -1;  // channel chunk whose scale / shift are in registers (16-byte loads)
  float sc[N], sh[N];
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    long p = e / CV;
    int c = (int)(e - p * CV) * N;
    float v[N], r[N];
    V16<T>::load(x + p * C + c, v);
    if (res) V16<T>::load(res + p * ldr + cr0 + c, r);
    if (c != cur) {
      cur = c;
      load_chan<N>(scale + c, sc);
      load_chan<N>(shift + c, sh);
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
      float o = __builtin_fmaf(v[i], sc[i], sh[i]);  // the backward's mask (relu mode 2) repeats this
      if (res) o += r[i];
      if (relu) o = fmaxf(o, 0.f);
      v[i] = o;
    }
    V16<T>::store(y + p * ldy + cy0 + c, v);
  }
}

// (round 5) the same pass with U chunks per thread in flight and 32-bit shift indexing, for C/N a
// power of two dividing 256: a block's chunk runs start at multiples of 256, so a thread's channel
// chunk is fixed (tid mod C/N) and its scale / shift are loaded once
template <typename T, int U>
__global__ void __launch_bounds__(256) k_bn_apply_u(const T* __restrict__ x, unsigned total, int cvs, int C,
                                                    const float* __restrict__ scale, const float* __restrict__ shift,
                                                    const T* __restrict__ res, int ldr, int cr0, int relu,
                                                    T* __restrict__ y, int ldy, int cy0) {
  constexpr int N = V16<T>::N;
  const unsigned tid = threadIdx.x;
  const int c = (int)(tid & ((1u << cvs) - 1u)) * N;
  float sc[N], sh[N];
  load_chan<N>(scale + c, sc);
  load_chan<N>(shift + c, sh);
  for (unsigned base = blockIdx.x * 256u * U; base < total; base += gridDim.x * 256u * U) {
    float v[U][N], r[U][N];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const unsigned e = base + k * 256u + tid;
      if (e < total) {
        const unsigned p = e >> cvs;
        V16<T>::load(x + (size_t)p * C + c, v[k]);
        if (res) V16<T>::load(res + (size_t)p * ldr + cr0 + c, r[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const unsigned e = base + k * 256u + tid;
      if (e >= total) break;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        float o = __builtin_fmaf(v[k][i], sc[i], sh[i]);
        if (res) o += r[k][i];
        if (relu) o = fmaxf(o, 0.f);
        v[k][i] = o;
      }
      V16<T>::store(y + (size_t)(e >> cvs) * ldy + cy0 + c, v[k]);
    }
  }
}

// Pixels per partial slot of the backward reduction: 16 pixel rows per thread row, fewer (down to
// 4) while that leaves fewer than 512 slots -- 32x32 layers at 256-512 channels would otherwise
// run on 64 workgroups (more slots make the totals pass, which reads every slot, the slower one).  Rows per block assume 16-byte bf16 lanes (C/8 lanes, at most 256); any
// multiple of the kernel's row count works, the fp32 kernel included.
static inline int bn_bwd_pix(int P, int C) {
  const int lanes = C / 8 < 256 ? (C / 8 > 0 ? C / 8 : 1) : 256;
  const int R = 256 / lanes > 0 ? 256 / lanes : 1;
  int rows = 16;
  // large layers (up2 at bs 32: 4096 slots at 16 rows): up to 64 rows while >= 1024 slots remain --
  // fewer partials for the totals pass to read
  while (rows < 64 && (P + R * rows * 2 - 1) / (R * rows * 2) >= 1024) rows <<= 1;
  while (rows > 4 && (P + R * rows - 1) / (R * rows) < 512) rows >>= 1;
  return R * rows;
}

// block: 256 threads = (C/N) chunk lanes x R rows.  MODE: ReLU mask source (0 none, 1 the stored
// activation y, 2 recomputed from the raw x); HX: x given (sum g*xhat as well).  Templated so each
// instance holds only the registers its streams need (the runtime-mode kernel spilled at 128 VGPRs).
template <typename T, int MODE, bool HX>
__global__ void __launch_bounds__(256) k_bn_bwd_reduce(const T* __restrict__ dy, int lddy, int cdy0,
                                                       const T* __restrict__ y, int ldy, int cy0,
                                                       const T* __restrict__ x, long P, int C,
                                                       const float* __restrict__ save, float* __restrict__ part,
                                                       int parts, int pix) {
  constexpr int N = V16<T>::N;
  static_assert(MODE != 2 || HX, "mask from raw needs x");
  __shared__ float red[2][256][N];
  const int CV = C / N;
  const int lanes = CV < 256 ? CV : 256;  // chunk lanes per row
  const int R = 256 / lanes;
  const int cgi = blockIdx.y;
  const int cl = threadIdx.x % lanes, row = threadIdx.x / lanes;
  const int c = (cgi * lanes + cl) * N;
  const long p0 = (long)blockIdx.x * pix;
  const long p1 = min(P, p0 + pix);
  float sg[N], sgx[N], mean[N], inv[N], msc[N], msh[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    sg[i] = sgx[i] = 0.f;
    mean[i] = (HX && c < C) ? save[c + i] : 0.f;
    inv[i] = (HX && c < C) ? save[C + c + i] : 0.f;
    msc[i] = (MODE == 2 && c < C) ? save[2 * C + c + i] : 0.f;
    msh[i] = (MODE == 2 && c < C) ? save[3 * C + c + i] : 0.f;
  }
  if (row < R && c < C) {
    // U pixels per iteration with all loads issued before any use: the loop is otherwise
    // latency-bound (one dependent HBM round trip per pixel row)
    constexpr int U = 4;  // pixels in flight per thread (the pixel count per thread, pix / R, is 4, 8 or 16)
    auto body = [&](const uint4& gd, const uint4& yd, const uint4& xd, bool ok) {
      float g[N], yy[N], xx[N];
      V16<T>::load((const T*)&gd, g);
#pragma unroll
      for (int i = 0; i < N; ++i) g[i] = ok ? g[i] : 0.f;
      if (MODE == 1) {
        V16<T>::load((const T*)&yd, yy);
#pragma unroll
        for (int i = 0; i < N; ++i) g[i] = yy[i] > 0.f ? g[i] : 0.f;
      }
      if (HX) {
        V16<T>::load((const T*)&xd, xx);
        if (MODE == 2)
#pragma unroll
          for (int i = 0; i < N; ++i) g[i] = __builtin_fmaf(xx[i], msc[i], msh[i]) > 0.f ? g[i] : 0.f;
#pragma unroll
        for (int i = 0; i < N; ++i) sgx[i] += g[i] * (xx[i] - mean[i]) * inv[i];
      }
#pragma unroll
      for (int i = 0; i < N; ++i) sg[i] += g[i];
    };
    // batches of U rows with every load issued before any use; rows past the end load the last
    // row again (clamped address) and contribute zero
    const uint4 z = make_uint4(0, 0, 0, 0);
    for (long pb = p0 + row; pb < p1; pb += U * R) {
      uint4 gd[U], yd[U], xd[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long pp = min(pb + u * R, p1 - 1);
        gd[u] = *(const uint4*)(dy + pp * lddy + cdy0 + c);
        yd[u] = MODE == 1 ? *(const uint4*)(y + pp * ldy + cy0 + c) : z;
        xd[u] = HX ? *(const uint4*)(x + pp * C + c) : z;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) body(gd[u], yd[u], xd[u], pb + u * R < p1);
    }
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    red[0][threadIdx.x][i] = sg[i];
    red[1][threadIdx.x][i] = sgx[i];
  }
  __syncthreads();
  if (row == 0 && c < C) {
    for (int r = 1; r < R; ++r)
#pragma unroll
      for (int i = 0; i < N; ++i) {
        sg[i] += red[0][r * lanes + cl][i];
        sgx[i] += red[1][r * lanes + cl][i];
      }
#pragma unroll
    for (int i = 0; i < N; ++i) {
      part[(size_t)blockIdx.x * C + c + i] = sg[i];
      part[((size_t)(parts + 1) + blockIdx.x) * C + c + i] = sgx[i];
    }
  }
}

// totals over parts -> part[0][parts][c], part[1][parts][c]; dgamma / dbeta
// block = 8 channels x 128 part lanes (1024 threads; C / 8 blocks: 8 for a 64-channel BN, where the
// former 32 x 32 layout ran 2 blocks for the whole GPU); each lane sums its parts (4 loads per
// stream in flight), then a fixed pairwise tree over the 128 lanes (deterministic)
// oparts: the totals go to rows oparts of both halves (the [2][oparts + 1][C] layout zp_bn_bwd_apply
// reads; oparts != parts after a zp_conv2d launch with bnr_part) -- only this block touches channel c,
// and it writes after every read of its parts
__global__ void __launch_bounds__(1024) k_bn_bwd_totals(float* __restrict__ part, int parts, int C, float* dgamma,
                                                        float* dbeta, int accumulate, int oparts) {
  __shared__ double sh[2][128][9];
  const int cl = threadIdx.x & 7, pl = threadIdx.x >> 3;
  const int c = blockIdx.x * 8 + cl;
  double s = 0, q = 0;
  if (c < C)
    for (int k0 = pl; k0 < parts; k0 += 128 * 4) {
      // clamped, unconditional loads: no branch between them
      float a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = min(k0 + 128 * u, parts - 1);
        a[u] = part[(size_t)k * C + c];
        b[u] = part[((size_t)parts + 1 + k) * C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool in = k0 + 128 * u < parts;
        s += in ? (double)a[u] : 0.0;
        q += in ? (double)b[u] : 0.0;
      }
    }
  sh[0][pl][cl] = s;
  sh[1][pl][cl] = q;
  __syncthreads();
  for (int w = 64; w > 0; w >>= 1) {
    if (pl < w) {
      sh[0][pl][cl] += sh[0][pl + w][cl];
      sh[1][pl][cl] += sh[1][pl + w][cl];
    }
    __syncthreads();
  }
  if (pl != 0 || c >= C) return;
  s = sh[0][0][cl];
  q = sh[1][0][cl];
  part[(size_t)oparts * C + c] = (float)s;
  part[((size_t)oparts + 1 + oparts) * C + c] = (float)q;
  if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)q : (float)q;
  if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)s : (float)s;
}

template <typename T, int relu>
__global__ void __launch_bounds__(256) k_bn_bwd_apply(const T* __restrict__ dy, int lddy, int cdy0,
                                                      const T* __restrict__ y, int ldy, int cy0,
                                                      const T* __restrict__ x, long P, int C,
                                                      const float* __restrict__ save, const float* __restrict__ part,
                                                      int parts, const float* __restrict__ gamma, T* __restrict__ dx,
                                                      T* __restrict__ dres, int lddres, int cdres0, int racc, int pix) {
  // pixel-row tiling (bn_tile)
  constexpr int N = V16<T>::N;
  constexpr int U = 4;
  const int CV = C / N;
  const int lanes = CV < 256 ? CV : 256;
  const int R = 256 / lanes;
  const int cl = threadIdx.x % lanes, row = threadIdx.x / lanes;
  const int c = (blockIdx.y * lanes + cl) * N;
  if (row >= R || c >= C) return;
  const long p0 = (long)blockIdx.x * pix;
  const long p1 = min(P, p0 + pix);
  const float invP = 1.f / (float)P;
  float mean[N], inv[N], sg[N], sgx[N], gm[N], msc[N], msh[N];
  if (dx) {
    load_chan<N>(save + c, mean);
    load_chan<N>(save + C + c, inv);
    if (relu == 2) {
      load_chan<N>(save + 2 * C + c, msc);
      load_chan<N>(save + 3 * C + c, msh);
    }
    load_chan<N>(part + (size_t)parts * C + c, sg);
    load_chan<N>(part + ((size_t)parts + 1 + parts) * C + c, sgx);
    load_chan<N>(gamma + c, gm);
#pragma unroll
    for (int i = 0; i < N; ++i) {
      sg[i] *= invP;
      sgx[i] *= invP;
    }
  }
  // optional streams loaded under their (uniform) condition and read only under it -- a select
  // between the stream and a zero constant made the compiler load through a pointer select of
  // global and private memory (flat loads, a 32-byte private segment)
  const bool hx = dx != nullptr, hr = dres != nullptr && racc;
  for (long pb = p0 + row; pb < p1; pb += U * R) {
    uint4 gd[U], yd[U], xd[U], rd[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long pp = min(pb + u * R, p1 - 1);
      gd[u] = *(const uint4*)(dy + pp * lddy + cdy0 + c);
      if constexpr (relu == 1) yd[u] = *(const uint4*)(y + pp * ldy + cy0 + c);
      if (hx) xd[u] = *(const uint4*)(x + pp * C + c);
      if (hr) rd[u] = *(const uint4*)(dres + pp * lddres + cdres0 + c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long p = pb + u * R;
      if (p >= p1) break;
      float g[N], yy[N], xx[N], o[N];
      V16<T>::load((const T*)&gd[u], g);
      if (relu == 1) {
        V16<T>::load((const T*)&yd[u], yy);
#pragma unroll
        for (int i = 0; i < N; ++i) g[i] = yy[i] > 0.f ? g[i] : 0.f;
      }
      if (dx) {
        V16<T>::load((const T*)&xd[u], xx);
        if (relu == 2)
#pragma unroll
          for (int i = 0; i < N; ++i) g[i] = __builtin_fmaf(xx[i], msc[i], msh[i]) > 0.f ? g[i] : 0.f;
#pragma unroll
        for (int i = 0; i < N; ++i) {
          float xh = (xx[i] - mean[i]) * inv[i];
          o[i] = gm[i] * inv[i] * (g[i] - sg[i] - xh * sgx[i]);
        }
        V16<T>::store(dx + p * C + c, o);
      }
      if (dres) {
        T* d = dres + p * lddres + cdres0 + c;
        if (racc) {
          float r[N];
          V16<T>::load((const T*)&rd[u], r);
#pragma unroll
          for (int i = 0; i < N; ++i) r[i] += g[i];
          V16<T>::store(d, r);
        } else {
          V16<T>::store(d, g);
        }
      }
    }
  }
}

// ------------------------------------------------------------------ mask resampling (v3 net)
// F.interpolate(mask [B,1,H,W] f32, (OH, OW), mode="bilinear", align_corners=False) written into
// an NHWC channel of the concat buffer (aspp_v3.py:89, 96-97; torch.cat at :90, :98, :101).  Same
// arithmetic as PyTorch's CPU kernel: scale = (float)in / out, src = max(scale * (d + 0.5) - 0.5, 0),
// i0 = (int)src, i1 = i0 + (i0 < in - 1), l1 = src - i0, out = l0 (w0 v00 + w1 v01) + l1 (w0 v10 + w1 v11).
struct LinIdx {
  int i0, i1;
  float l0, l1;
};
__device__ __forceinline__ LinIdx lin_idx(int d, int n_in, int n_out) {
  const float sc = (float)n_in / (float)n_out;
  float src = sc * ((float)d + 0.5f) - 0.5f;
  src = src < 0.f ? 0.f : src;
  LinIdx r;
  r.i0 = (int)src;
  r.i1 = r.i0 + (r.i0 < n_in - 1 ? 1 : 0);
  r.l1 = src - (float)r.i0;
  r.l0 = 1.f - r.l1;
  return r;
}

template <typename T>
__global__ void k_mask_interp(const float* __restrict__ x, int B, int H, int W, int OH, int OW, T* __restrict__ y,
                              int ldy, int cy0) {
  const long total = (long)B * OH * OW;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int ox = (int)(e % OW);
    const long t = e / OW;
    const int oy = (int)(t % OH), b = (int)(t / OH);
    const LinIdx ly = lin_idx(oy, H, OH), lx = lin_idx(ox, W, OW);
    const float* s = x + (size_t)b * H * W;
    const float v = ly.l0 * (lx.l0 * s[ly.i0 * W + lx.i0] + lx.l1 * s[ly.i0 * W + lx.i1]) +
                    ly.l1 * (lx.l0 * s[ly.i1 * W + lx.i0] + lx.l1 * s[ly.i1 * W + lx.i1]);
    y[e * ldy + cy0] = Elem<T>::cvt(v);
  }
}

// weight of input index i in output d (both taps may hit i when i1 == i0)
__device__ __forceinline__ float lin_w(const LinIdx& l, int i) {
  return (l.i0 == i ? l.l0 : 0.f) + (l.i1 == i ? l.l1 : 0.f);
}

// backward, gather form (deterministic): dx[b, h, w] (+)= sum over the outputs whose taps include (h, w)
template <typename T>
__global__ void k_mask_interp_bwd(const T* __restrict__ dy, int lddy, int cdy0, int B, int OH, int OW, int H, int W,
                                  float* __restrict__ dx, int accumulate) {
  const long total = (long)B * H * W;
  const float sh = (float)H / (float)OH, sw = (float)W / (float)OW;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int w = (int)(e % W);
    const long t = e / W;
    const int h = (int)(t % H), b = (int)(t / H);
    // outputs d with i0(d) in {i - 1, i}: d ~ (i + 0.5) / scale - 0.5, +-2 of slack
    const int oy0 = max(0, (int)floorf((h - 0.5f) / sh - 0.5f) - 2), oy1 = min(OH - 1, (int)((h + 1.5f) / sh) + 2);
    const int ox0 = max(0, (int)floorf((w - 0.5f) / sw - 0.5f) - 2), ox1 = min(OW - 1, (int)((w + 1.5f) / sw) + 2);
    float acc = 0.f;
    for (int oy = oy0; oy <= oy1; ++oy) {
      const float wy = lin_w(lin_idx(oy, H, OH), h);
      if (wy == 0.f) continue;
      for (int ox = ox0; ox <= ox1; ++ox) {
        const float wx = lin_w(lin_idx(ox, W, OW), w);
        if (wx == 0.f) continue;
        acc += wy * wx * Elem<T>::ld(dy + (((size_t)b * OH + oy) * OW + ox) * lddy + cdy0);
      }
    }
    dx[e] = accumulate ? dx[e] + acc : acc;
  }
}

// ------------------------------------------------------------------ layout / pooling
template <typename T>
__global__ void k_nchw_to_nhwc(const float* __restrict__ x, int B, int C, int H, int W, int cpad, T* __restrict__ y) {
  constexpr int N = V16<T>::N;
  const long HW = (long)H * W, total = (long)B * HW;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    long b = e / HW, s = e - b * HW;
    T* o = y + e * cpad;
    if (cpad % N == 0) {  // one 16 B store per N channels (the network's input: 3 -> 8 bf16 = one store)
      for (int c0 = 0; c0 < cpad; c0 += N) {
        float v[N];
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] = c0 + i < C ? x[(b * C + c0 + i) * HW + s] : 0.f;
        V16<T>::store(o + c0, v);
      }
    } else {
      for (int c = 0; c < cpad; ++c) o[c] = Elem<T>::cvt(c < C ? x[(b * C + c) * HW + s] : 0.f);
    }
  }
}

template <typename T>
__global__ void k_maxpool(const T* __restrict__ x, int B, int IH, int IW, int ldx, int cx0, int C, T* __restrict__ y,
                          int OH, int OW, int ldy, int cy0) {
  constexpr int N = V16<T>::N;
  const int CV = C / N;
  const long total = (long)B * OH * OW * CV;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    long pix = e / CV;
    int c = (int)(e - pix * CV) * N;
    int ox = (int)(pix % OW);
    long t = pix / OW;
    int oy = (int)(t % OH), b = (int)(t / OH);
    float m[N];
#pragma unroll
    for (int i = 0; i < N; ++i) m[i] = -INFINITY;
    for (int ky = 0; ky < 3; ++ky) {
      int iy = oy * 2 - 1 + ky;
      if ((unsigned)iy >= (unsigned)IH) continue;
      for (int kx = 0; kx < 3; ++kx) {
        int ix = ox * 2 - 1 + kx;
        if ((unsigned)ix >= (unsigned)IW) continue;
        float v[N];
        V16<T>::load(x + (((size_t)b * IH + iy) * IW + ix) * ldx + cx0 + c, v);
#pragma unroll
        for (int i = 0; i < N; ++i)
          if (v[i] > m[i] || isnan(v[i])) m[i] = v[i];  // PyTorch CPU max_pool2d rule
      }
    }
    V16<T>::store(y + pix * ldy + cy0 + c, m);
  }
}

// Split-fp32 stem im2col (zp_im2col_split): thread per (output pixel, 8-element chunk of the
// kpad-long patch row); taps gathered from the f32 NHWC image (L2-resident: each input pixel is
// read by <= 16 overlapping 7x7 / s2 windows), each element split into the NPL planes
template <int NPL>
__global__ void k_im2col_split(const float* __restrict__ x, int B, int H, int W, int ldx, int C, int k, int s, int p,
                               int OH, int OW, int kpad, unsigned short* __restrict__ y, unsigned* rflag) {
  const int KC = kpad / 8, KK = k * k * C;
  bool bad = false;
  const long total = (long)B * OH * OW * KC;
  const long plane = (long)B * OH * OW * kpad;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long pix = e / KC;
    const int kc = (int)(e - pix * KC);
    const int ox = (int)(pix % OW);
    const long t = pix / OW;
    const int oy = (int)(t % OH), b = (int)(t / OH);
    uint32_t w[NPL][4];
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      unsigned short q[2][NPL];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int kk = kc * 8 + i + h;
        float v = 0.f;
        if (kk < KK) {
          const int tap = kk / C, c = kk - tap * C;
          const int ky = tap / k, kx = tap - ky * k;
          const int iy = oy * s - p + ky, ix = ox * s - p + kx;
          if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) v = x[(((long)b * H + iy) * W + ix) * ldx + c];
        }
        SplitF32<NPL>::split(v, q[h]);
        if constexpr (NPL == 2) bad |= h2_overflow(v);
      }
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) w[pl][i >> 1] = (uint32_t)q[0][pl] | ((uint32_t)q[1][pl] << 16);
    }
    unsigned short* yo = y + pix * kpad + kc * 8;
#pragma unroll
    for (int pl = 0; pl < NPL; ++pl) *(uint4*)(yo + pl * plane) = make_uint4(w[pl][0], w[pl][1], w[pl][2], w[pl][3]);
  }
  if constexpr (NPL == 2) raise_range_flag(rflag, bad);
}

// Split-fp32 max pool (NPL planes, SplitF32<NPL>): the 3x3 window max of the joined f32 values
// (PyTorch CPU rule), stored split again (joining is exact, so the winner's value is reproduced
// exactly).  Planes: x + p * psx, y + p * psy.
template <int NPL>
__global__ void k_maxpool_split(const unsigned short* __restrict__ x, long psx, int B, int IH, int IW, int ldx, int cx0,
                                int C, unsigned short* __restrict__ y, long psy, int OH, int OW, int ldy, int cy0) {
  const int CV = C / 8;
  const long total = (long)B * OH * OW * CV;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    long pix = e / CV;
    int c = (int)(e - pix * CV) * 8;
    int ox = (int)(pix % OW);
    long t = pix / OW;
    int oy = (int)(t % OH), b = (int)(t / OH);
    float m[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) m[i] = -INFINITY;
    for (int ky = 0; ky < 3; ++ky) {
      int iy = oy * 2 - 1 + ky;
      if ((unsigned)iy >= (unsigned)IH) continue;
      for (int kx = 0; kx < 3; ++kx) {
        int ix = ox * 2 - 1 + kx;
        if ((unsigned)ix >= (unsigned)IW) continue;
        const size_t o = (((size_t)b * IH + iy) * IW + ix) * ldx + cx0 + c;
        uint32_t w[NPL][4];
#pragma unroll
        for (int p = 0; p < NPL; ++p) {
          const uint4 q = *(const uint4*)(x + o + p * psx);
          w[p][0] = q.x;
          w[p][1] = q.y;
          w[p][2] = q.z;
          w[p][3] = q.w;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int s = (i & 1) * 16;
          unsigned short q[NPL];
#pragma unroll
          for (int p = 0; p < NPL; ++p) q[p] = (unsigned short)(w[p][i >> 1] >> s);
          const float v = SplitF32<NPL>::join(q);
          if (v > m[i] || isnan(v)) m[i] = v;
        }
      }
    }
    uint32_t o[NPL][4];
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      unsigned short q0[NPL], q1[NPL];
      SplitF32<NPL>::split(m[i], q0);
      SplitF32<NPL>::split(m[i + 1], q1);
#pragma unroll
      for (int p = 0; p < NPL; ++p) o[p][i >> 1] = (uint32_t)q0[p] | ((uint32_t)q1[p] << 16);
    }
    unsigned short* yo = y + pix * ldy + cy0 + c;
#pragma unroll
    for (int p = 0; p < NPL; ++p) *(uint4*)(yo + p * psy) = make_uint4(o[p][0], o[p][1], o[p][2], o[p][3]);
  }
}

// Split-fp32 global average pool: block = (64 channels, image b); the joined values summed in
// double (CPU adaptive_avg_pool2d's accumulator) over 4 pixel lanes, combined in a fixed order; the
// f32 mean stored split into y [NPL][B][C]
template <int NPL>
__global__ void __launch_bounds__(256) k_avgpool_split(const unsigned short* __restrict__ x, long psx, int H, int W,
                                                       int ldx, int cx0, int C, unsigned short* __restrict__ y,
                                                       long psy) {
  __shared__ double red[4][64];
  const int b = blockIdx.y;
  const long HW = (long)H * W;
  const int cl = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double s = 0.0;
  if (c < C)
    for (long p = sl; p < HW; p += 4) {
      const size_t o = ((size_t)b * HW + p) * ldx + cx0 + c;
      unsigned short q[NPL];
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) q[pl] = x[o + pl * psx];
      s += (double)SplitF32<NPL>::join(q);
    }
  red[sl][cl] = s;
  __syncthreads();
  if (threadIdx.x < 64 && c < C) {
    const double t = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
    unsigned short q[NPL];
    SplitF32<NPL>::split((float)(t / (double)HW), q);
    const size_t o = (size_t)b * C + c;
#pragma unroll
    for (int pl = 0; pl < NPL; ++pl) y[o + pl * psy] = q[pl];
  }
}

// Split-fp32 global average pool, vectorised: block = (64 channels, image b), 256 threads = 8
// channel vectors (8 channels, 16 B per plane) x 32 pixel lanes; each thread sums every 32nd pixel
// in double (four pixels' loads in flight), the 32 lane sums meet in LDS in a fixed order.  Same
// sums as k_avgpool_split up to the (double) association; 16 B loads instead of 2 B
// (r03: k_avgpool_split read 67 MB in 71 us, 0.94 TB/s).
template <int NPL>
__global__ void __launch_bounds__(256) k_avgpool_split8(const unsigned short* __restrict__ x, long psx, int H, int W,
                                                        int ldx, int cx0, int C, unsigned short* __restrict__ y,
                                                        long psy) {
  __shared__ double red[32][65];
  const int b = blockIdx.y;
  const int HW = H * W;
  const int cv = threadIdx.x & 7, pl0 = threadIdx.x >> 3;
  const int c = blockIdx.x * 64 + cv * 8;
  double s[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) s[r] = 0.0;
  if (c < C) {
    const unsigned short* xb = x + (size_t)b * HW * ldx + cx0 + c;
    int p = pl0;
    for (; p + 96 < HW; p += 128) {
      uint4 q[4][NPL];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) q[u][pl] = *(const uint4*)(xb + (size_t)(p + 32 * u) * ldx + pl * psx);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          unsigned short h[NPL];
#pragma unroll
          for (int pl = 0; pl < NPL; ++pl) {
            const uint32_t w4[4] = {q[u][pl].x, q[u][pl].y, q[u][pl].z, q[u][pl].w};
            h[pl] = (unsigned short)(w4[r >> 1] >> ((r & 1) * 16));
          }
          s[r] += (double)SplitF32<NPL>::join(h);
        }
      }
    }
    for (; p < HW; p += 32) {
      uint4 q[NPL];
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) q[pl] = *(const uint4*)(xb + (size_t)p * ldx + pl * psx);
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        unsigned short h[NPL];
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) {
          const uint32_t w4[4] = {q[pl].x, q[pl].y, q[pl].z, q[pl].w};
          h[pl] = (unsigned short)(w4[r >> 1] >> ((r & 1) * 16));
        }
        s[r] += (double)SplitF32<NPL>::join(h);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 8; ++r) red[pl0][cv * 8 + r] = s[r];
  __syncthreads();
  if (threadIdx.x < 64 && blockIdx.x * 64 + (int)threadIdx.x < C) {
    double t = 0.0;
    for (int k = 0; k < 32; ++k) t += red[k][threadIdx.x];
    unsigned short q[NPL];
    SplitF32<NPL>::split((float)(t / (double)HW), q);
    const size_t o = (size_t)b * C + blockIdx.x * 64 + threadIdx.x;
#pragma unroll
    for (int pl = 0; pl < NPL; ++pl) y[o + pl * psy] = q[pl];
  }
}

// Window (oy, ox) of the 3x3 / stride-2 / pad-1 pool: per channel, the tap (ky*3+kx, -1 when the
// window lies outside the output) of its first maximum in (ky, kx) scan order (PyTorch CPU rule:
// `>` or NaN) and the window's dy.
template <typename T>
__device__ __forceinline__ void mp_window(const T* __restrict__ x, int ldx, int cx0, const T* __restrict__ dy,
                                          int lddy, int cdy0, int b, int c, int IH, int IW, int OH, int OW, int oy,
                                          int ox, int* pos, float* g) {
  constexpr int N = V16<T>::N;
#pragma unroll
  for (int i = 0; i < N; ++i) pos[i] = -1;
  if (oy >= OH || ox >= OW) return;
  float m[N];
#pragma unroll
  for (int i = 0; i < N; ++i) m[i] = -INFINITY;
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int yy = oy * 2 - 1 + ky;
    if ((unsigned)yy >= (unsigned)IH) continue;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int xx = ox * 2 - 1 + kx;
      if ((unsigned)xx >= (unsigned)IW) continue;
      float v[N];
      V16<T>::load(x + (((size_t)b * IH + yy) * IW + xx) * ldx + cx0 + c, v);
#pragma unroll
      for (int i = 0; i < N; ++i)
        if (v[i] > m[i] || isnan(v[i])) {
          m[i] = v[i];
          pos[i] = ky * 3 + kx;
        }
    }
  }
  V16<T>::load(dy + (((size_t)b * OH + oy) * OW + ox) * lddy + cdy0 + c, g);
}

// Backward of the 3x3 / stride-2 / pad-1 max pool, gather form without atomics.  A thread owns the
// 2x2 input block (rows 2k, 2k+1; cols 2j, 2j+1) for one 16-byte channel vector, over a chunk of
// MP_ROWS consecutive k.  Row 2k lies only in window row k, row 2k+1 in window rows k and k+1 (same
// for columns), so the block needs windows (k|k+1, j|j+1); the k+1 pair is carried to the next k,
// i.e. two windows (18 loads) per block instead of a window walk per input pixel.  Contributions are
// added in (oy, ox) order, then the existing dx when accumulating.
constexpr int MP_ROWS = 4;
template <typename T>
__global__ void __launch_bounds__(256) k_maxpool_bwd(const T* __restrict__ x, int ldx, int cx0,
                                                     const T* __restrict__ dy, int lddy, int cdy0, int B, int IH,
                                                     int IW, int C, int OH, int OW, T* __restrict__ dx, int lddx,
                                                     int cdx0, int accumulate) {
  constexpr int N = V16<T>::N;
  const int CV = C / N, JP = (IW + 1) / 2, KP = (IH + 1) / 2, KC = (KP + MP_ROWS - 1) / MP_ROWS;
  const long total = (long)B * KC * JP * CV;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int c = (int)(e % CV) * N;
    long t = e / CV;
    const int j = (int)(t % JP);
    t /= JP;
    const int kc = (int)(t % KC), b = (int)(t / KC);
    const int k0 = kc * MP_ROWS, k1 = min(k0 + MP_ROWS, KP);
    int p00[N], p01[N], p10[N], p11[N];
    float g00[N], g01[N], g10[N], g11[N];
    mp_window(x, ldx, cx0, dy, lddy, cdy0, b, c, IH, IW, OH, OW, k0, j, p00, g00);
    mp_window(x, ldx, cx0, dy, lddy, cdy0, b, c, IH, IW, OH, OW, k0, j + 1, p01, g01);
    for (int k = k0; k < k1; ++k) {
      mp_window(x, ldx, cx0, dy, lddy, cdy0, b, c, IH, IW, OH, OW, k + 1, j, p10, g10);
      mp_window(x, ldx, cx0, dy, lddy, cdy0, b, c, IH, IW, OH, OW, k + 1, j + 1, p11, g11);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int iy = 2 * k + (q >> 1), ix = 2 * j + (q & 1);
        if (iy >= IH || ix >= IW) continue;
        float acc[N];
#pragma unroll
        for (int i = 0; i < N; ++i) {
          float a = 0.f;
          // taps of (iy, ix) in windows (k, j), (k, j+1), (k+1, j), (k+1, j+1)
          if (q == 0) {
            if (p00[i] == 4) a += g00[i];
          } else if (q == 1) {
            if (p00[i] == 5) a += g00[i];
            if (p01[i] == 3) a += g01[i];
          } else if (q == 2) {
            if (p00[i] == 7) a += g00[i];
            if (p10[i] == 1) a += g10[i];
          } else {
            if (p00[i] == 8) a += g00[i];
            if (p01[i] == 6) a += g01[i];
            if (p10[i] == 2) a += g10[i];
            if (p11[i] == 0) a += g11[i];
          }
          acc[i] = a;
        }
        T* o = dx + (((size_t)b * IH + iy) * IW + ix) * lddx + cdx0 + c;
        if (accumulate) {
          float r[N];
          V16<T>::load(o, r);
#pragma unroll
          for (int i = 0; i < N; ++i) acc[i] += r[i];
        }
        V16<T>::store(o, acc);
      }
#pragma unroll
      for (int i = 0; i < N; ++i) {
        p00[i] = p10[i];
        g00[i] = g10[i];
        p01[i] = p11[i];
        g01[i] = g11[i];
      }
    }
  }
}

// Per-channel sums over H*W: block = (image b, 64 channels), 256 threads = 64 channels x 4 pixel
// slices (coalesced 64-channel rows), slices combined through LDS in a fixed order.
template <typename T, typename ACC>
__device__ __forceinline__ ACC sum_hw_block(const T* __restrict__ x, long HW, int ld, int c0, int C, int b) {
  __shared__ ACC red[4][64];
  const int cl = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  ACC s = 0;
  if (c < C)
    for (long p = sl; p < HW; p += 4) s += (ACC)Elem<T>::ld(x + ((size_t)b * HW + p) * ld + c0 + c);
  red[sl][cl] = s;
  __syncthreads();
  return red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
}

// Vectorised form (C, c0, ld multiples of the 16 B vector width N): block = (image b, 64
// channels), 256 threads = (64 / N) chunk lanes x (256 N / 64) pixel lanes, 16 B loads; the pixel
// lanes are combined through LDS in a fixed order (deterministic).  MODE 0: mean over H*W in
// double, converted to T (CPU adaptive_avg_pool2d accumulates in double); MODE 1: float sum -> T.
template <typename T, int MODE>
__global__ void __launch_bounds__(256) k_hw_reduce_vec(const T* __restrict__ x, int H, int W, int ld, int c0, int C,
                                                       T* __restrict__ y) {
  constexpr int N = V16<T>::N;
  constexpr int CL = 64 / N, PL = 256 / CL;
  using ACC = typename std::conditional<MODE == 0, double, float>::type;
  __shared__ ACC red[PL][64];
  const int b = blockIdx.y;
  const long HW = (long)H * W;
  const int cl = threadIdx.x % CL, pl = threadIdx.x / CL;
  const int c = blockIdx.x * 64 + cl * N;
  ACC s[N];
#pragma unroll
  for (int i = 0; i < N; ++i) s[i] = 0;
  if (c < C) {
    const T* base = x + (size_t)b * HW * ld + c0 + c;
    long p = pl;
    for (; p + 3 * PL < HW; p += 4 * PL) {
      uint4 u[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) u[k] = *(const uint4*)(base + (p + k * PL) * ld);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float v[N];
        V16<T>::load((const T*)&u[k], v);
#pragma unroll
        for (int i = 0; i < N; ++i) s[i] += (ACC)v[i];
      }
    }
    for (; p < HW; p += PL) {
      float v[N];
      V16<T>::load(base + p * ld, v);
#pragma unroll
      for (int i = 0; i < N; ++i) s[i] += (ACC)v[i];
    }
  }
#pragma unroll
  for (int i = 0; i < N; ++i) red[pl][cl * N + i] = s[i];
  __syncthreads();
  if (threadIdx.x < 64) {
    const int cc = blockIdx.x * 64 + threadIdx.x;
    ACC t = 0;
    for (int k = 0; k < PL; ++k) t += red[k][threadIdx.x];
    if (cc < C) {
      if (MODE == 0) y[(size_t)b * C + cc] = Elem<T>::cvt((float)((double)t / (double)HW));
      else y[(size_t)b * C + cc] = Elem<T>::cvt((float)t);
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) k_avgpool(const T* __restrict__ x, int H, int W, int ldx, int cx0, int C,
                                                 T* __restrict__ y) {
  const int b = blockIdx.y;
  const long HW = (long)H * W;
  // CPU adaptive_avg_pool2d accumulates in acc_type<float> = double
  double s = sum_hw_block<T, double>(x, HW, ldx, cx0, C, b);
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  if (threadIdx.x < 64 && c < C) y[(size_t)b * C + c] = Elem<T>::cvt((float)(s / (double)HW));
}

template <typename T>
__global__ void __launch_bounds__(256) k_sum_hw(const T* __restrict__ dy, int H, int W, int lddy, int cdy0, int C,
                                                T* __restrict__ out) {
  const int b = blockIdx.y;
  float s = sum_hw_block<T, float>(dy, (long)H * W, lddy, cdy0, C, b);
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  if (threadIdx.x < 64 && c < C) out[(size_t)b * C + c] = Elem<T>::cvt(s);
}

// y[b, p, cy0 + c] = src[b, c] for every pixel, one 16 B store per N channels (C, ldy, cy0
// multiples of N)
template <typename T>
__global__ void k_broadcast_vec(const T* __restrict__ src, int B, int C, T* __restrict__ y, int H, int W, int ldy,
                                int cy0) {
  constexpr int N = V16<T>::N;
  const int CV = C / N;
  const long HW = (long)H * W, total = (long)B * HW * CV;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long pix = e / CV;
    const int c = (int)(e - pix * CV) * N;
    const long b = pix / HW;
    *(uint4*)(y + pix * ldy + cy0 + c) = *(const uint4*)(src + b * C + c);
  }
}

template <typename T>
__global__ void k_broadcast(const T* __restrict__ src, int B, int C, float mul, T* __restrict__ y, int H, int W, int ldy,
                            int cy0, int accumulate, int convert) {
  const long HW = (long)H * W, total = (long)B * HW * C;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    long pix = e / C;
    int c = (int)(e - pix * C);
    long b = pix / HW;
    T* o = y + pix * ldy + cy0 + c;
    if (!convert) {
      *o = src[b * C + c];
    } else {
      float v = Elem<T>::ld(src + b * C + c) * mul;
      if (accumulate) v += Elem<T>::ld(o);
      *o = Elem<T>::cvt(v);
    }
  }
}

template <typename TX, typename TY>
__global__ void k_copy_slice(const TX* __restrict__ x, int ldx, int cx0, TY* __restrict__ y, int ldy, int cy0, long P,
                             int C, int accumulate) {
  const long total = P * C;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    long p = e / C;
    int c = (int)(e - p * C);
    float v = Elem<TX>::ld(x + p * ldx + cx0 + c);
    TY* o = y + p * ldy + cy0 + c;
    if (accumulate) v += Elem<TY>::ld(o);
    *o = Elem<TY>::cvt(v);
  }
}

template <typename T>
__global__ void k_head_grad(const float* __restrict__ dmask, const float* __restrict__ dcode, int B, int L, int H, int W,
                            int ldy, T* __restrict__ y) {
  const long HW = (long)H * W, total = (long)B * HW;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    long b = e / HW, s = e - b * HW;
    T* o = y + e * ldy;
    if constexpr (sizeof(T) == 2) {
      if (ldy % 8 == 0) {  // (round 5) 16-byte stores of 8 channels: the 2-byte form took 50 us at bs 32
        for (int c0 = 0; c0 < ldy; c0 += 8) {
          uint32_t w[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            uint32_t h[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
              const int c = c0 + 2 * q + k;
              const float v = c == 0 ? dmask[b * HW + s] : (c <= L ? dcode[(b * L + c - 1) * HW + s] : 0.f);
              h[k] = H16<T>::to(v);
            }
            w[q] = h[0] | (h[1] << 16);
          }
          *(uint4*)(o + c0) = make_uint4(w[0], w[1], w[2], w[3]);
        }
        continue;
      }
    }
    o[0] = Elem<T>::cvt(dmask[b * HW + s]);
    for (int c = 0; c < L; ++c) o[1 + c] = Elem<T>::cvt(dcode[(b * L + c) * HW + s]);
    for (int c = L + 1; c < ldy; ++c) o[c] = Elem<T>::cvt(0.f);
  }
}

__global__ void k_threshold(const float* __restrict__ x, long n, int f64, void* out) {
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    bool b = x[e] > 8.940696716308594e-08f;  // NaN -> false
    if (f64) ((double*)out)[e] = b ? 1.0 : 0.0;
    else ((uint8_t*)out)[e] = b ? 1 : 0;
  }
}

__global__ void k_adam(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
                       long n, float lr_bc1, float w1, float b2, float w2, float bc2_sqrt, float eps) {
  // torch.optim.Adam (_single_tensor_adam) op by op, each op rounded separately (no FMA contraction):
  //   exp_avg.lerp_(grad, w1 = 1 - beta1)      (w1 < 0.5: m + w1 * (g - m))
  //   exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=w2 = 1 - beta2)
  //   denom = exp_avg_sq.sqrt() / sqrt(bc2) + eps;  param.addcdiv_(exp_avg, denom, value=-lr/bc1)
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const float gg = g[e];
    float mm = m[e];
    mm = fmaf(w1, __fsub_rn(gg, mm), mm);  // ATen lerp: fmadd(weight, end - self, self)
    float vv = __fmul_rn(v[e], b2);
    vv = __fadd_rn(vv, __fmul_rn(__fmul_rn(w2, gg), gg));
    m[e] = mm;
    v[e] = vv;
    const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(vv), bc2_sqrt), eps);
    p[e] = __fadd_rn(p[e], __fmul_rn(-lr_bc1, __fdiv_rn(mm, denom)));
  }
}

// multi-tensor Adam: one launch updates up to ADAM_MT tensors; the tensor of a block comes from
// the prefix sums of per-tensor block counts (ADAM_CHUNK elements per block)
constexpr int ADAM_MT = 40;
constexpr int ADAM_CHUNK = 4096;
struct AdamTable {
  float* p[ADAM_MT];
  const float* g[ADAM_MT];
  float* m[ADAM_MT];
  float* v[ADAM_MT];
  long long n[ADAM_MT];
  int blk0[ADAM_MT + 1];
  int count;
};

__global__ void __launch_bounds__(256) k_adam_multi(const AdamTable T, float lr_bc1, float w1, float b2, float w2,
                                                    float bc2_sqrt, float eps, const float* __restrict__ step_dev,
                                                    double lr, double beta1, double beta2) {
  if (step_dev) {
    // capturable form (zp_adam_multi_dev): the step count lives on the device, so a captured
    // graph replays with the current count; the host's double-precision bias corrections, per block
    const double st = (double)step_dev[0];
    lr_bc1 = (float)(lr / (1.0 - pow(beta1, st)));
    bc2_sqrt = (float)sqrt(1.0 - pow(beta2, st));
  }
  const int b = blockIdx.x;
  int lo = 0, hi = T.count - 1;  // last t with blk0[t] <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (T.blk0[mid] <= b) lo = mid;
    else hi = mid - 1;
  }
  const int t = lo;
  const long long e0 = (long long)(b - T.blk0[t]) * ADAM_CHUNK;
  const long long e1 = min(T.n[t], e0 + ADAM_CHUNK);
  float* __restrict__ p = T.p[t];
  const float* __restrict__ g = T.g[t];
  float* __restrict__ m = T.m[t];
  float* __restrict__ v = T.v[t];
  for (long long e = e0 + threadIdx.x; e < e1; e += 256) {
    // identical op sequence to k_adam (torch.optim.Adam single-tensor order)
    const float gg = g[e];
    float mm = m[e];
    mm = fmaf(w1, __fsub_rn(gg, mm), mm);
    float vv = __fmul_rn(v[e], b2);
    vv = __fadd_rn(vv, __fmul_rn(__fmul_rn(w2, gg), gg));
    m[e] = mm;
    v[e] = vv;
    const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(vv), bc2_sqrt), eps);
    p[e] = __fadd_rn(p[e], __fmul_rn(-lr_bc1, __fdiv_rn(mm, denom)));
  }
}

}  // namespace zp

using namespace zp;

// ZP_F16 is an inference dtype: accepted by the forward-path entry points, refused by the
// training-only ones (ZP_DTYPE_CHECK_TRAIN)
#define ZP_DTYPE_CHECK(fn, dt) \
  ZP_CHECK_ARG((dt) == ZP_F32 || (dt) == ZP_BF16 || (dt) == ZP_F16, fn ": bad dtype %d", (int)(dt))
#define ZP_DTYPE_CHECK_TRAIN(fn, dt) \
  ZP_CHECK_ARG((dt) == ZP_F32 || (dt) == ZP_BF16, fn ": dtype %d (fp16 is inference-only)", (int)(dt))
#define ZP_BY_DTYPE(dt, KERNEL, grid, block, st, ...)                                   \
  do {                                                                                  \
    if ((dt) == ZP_BF16) hipLaunchKernelGGL(KERNEL<bf16_t>, grid, block, 0, st, __VA_ARGS__); \
    else if ((dt) == ZP_F16) hipLaunchKernelGGL(KERNEL<f16_t>, grid, block, 0, st, __VA_ARGS__); \
    else hipLaunchKernelGGL(KERNEL<float>, grid, block, 0, st, __VA_ARGS__);            \
  } while (0)

// zp_split_range_flag registry: one word per device, set by the caller
static unsigned* g_range_flag[64];

unsigned* zp::range_flag() {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return nullptr;
  return g_range_flag[d];
}

extern "C" int zp_split_range_flag(unsigned int* flag) {
  int d = 0;
  ZP_CHECK_ARG(hipGetDevice(&d) == hipSuccess && d >= 0 && d < 64, "zp_split_range_flag: no current device");
  g_range_flag[d] = flag;
  return ZP_OK;
}

extern "C" int zp_abi_version(void) { return ZP_ABI_VERSION; }
extern "C" long long zp_bn_finalize_floats(int parts, int C) {
  if (parts <= 0 || C <= 0) return 0;
  return 3LL * parts * C + (C + 31) / 32;  // statistics + the one-launch merge's counters (ABI 4)
}
extern "C" const char* zp_last_error(void) { return g_err; }
extern "C" int zp_conv_rows_pad(int Cout) {
  int tc = Cout > 64 ? 128 : (Cout > 32 ? 64 : 32);
  return (Cout + tc - 1) / tc * tc;
}

extern "C" int zp_pack_weight(const float* src, int d0, int d1, int kh, int kw, int transposed, int ntaps, const int* ky,
                              const int* kx, int cstride, int dtype, void* dst, int rows_pad, int k_pad, void* stream) {
  ZP_CHECK_ARG(dtype == ZP_F32 || dtype == ZP_BF16 || dtype == ZP_F16 || dtype == ZP_F32X3 || dtype == ZP_F32H2,
               "zp_pack_weight: bad dtype %d", dtype);
  ZP_CHECK_ARG(src && dst && ky && kx, "zp_pack_weight: null pointer");
  ZP_CHECK_ARG(ntaps >= 1 && ntaps <= ZP_MAX_TAPS, "zp_pack_weight: ntaps %d", ntaps);
  ZP_CHECK_ARG(cstride >= (transposed ? d0 : d1) && (long)ntaps * cstride <= k_pad, "zp_pack_weight: cstride/k_pad");
  ZP_CHECK_ARG(rows_pad >= (transposed ? d1 : d0), "zp_pack_weight: rows_pad");
  PackArgs a;
  a.src = src; a.dst = dst; a.d0 = d0; a.d1 = d1; a.kh = kh; a.kw = kw; a.transposed = transposed;
  a.ntaps = ntaps; a.cstride = cstride; a.rows_pad = rows_pad; a.k_pad = k_pad;
  for (int t = 0; t < ntaps; ++t) {
    ZP_CHECK_ARG(ky[t] >= 0 && ky[t] < kh && kx[t] >= 0 && kx[t] < kw, "zp_pack_weight: tap %d out of range", t);
    a.ky[t] = (signed char)ky[t];
    a.kx[t] = (signed char)kx[t];
  }
  if (dtype == ZP_F32X3)
    hipLaunchKernelGGL(k_pack_split<3>, dim3(grid_for((long)rows_pad * k_pad)), dim3(256), 0, (hipStream_t)stream, a,
                       nullptr);
  else if (dtype == ZP_F32H2)
    hipLaunchKernelGGL(k_pack_split<2>, dim3(grid_for((long)rows_pad * k_pad)), dim3(256), 0, (hipStream_t)stream, a,
                       range_flag());
  else
    ZP_BY_DTYPE(dtype, k_pack, dim3(grid_for((long)rows_pad * k_pad)), dim3(256), (hipStream_t)stream, a);
  ZP_LAUNCH_CHECK("zp_pack_weight");
  return ZP_OK;
}

extern "C" int zp_pack_weight_multi(int n, const zp_pack_job* jobs, const long long* prefix, long long total,
                                    void* stream) {
  ZP_CHECK_ARG(n >= 0 && n <= 65535 && total >= 0 && total < (1ll << 40) && (n == 0 || (jobs && prefix)),
               "zp_pack_weight_multi: bad args");
  if (n == 0 || total == 0) return ZP_OK;
  // blocks per job, each walking the job's 8-row x 64-channel tiles: 64 measured best of 32 / 64 / 128
  // / 256 on the training step's ~100 jobs (256: 170 us, most blocks of the small jobs empty; 64: 134
  // us; a flat tile space over all jobs, blocks scanning the jobs' tile counts, ran 228 us at 172
  // VGPRs); ZP_PACK_GX for A/B
  static const int gx = getenv("ZP_PACK_GX") ? atoi(getenv("ZP_PACK_GX")) : 64;
  static const int forms = getenv("ZP_PACK_FORMS") ? atoi(getenv("ZP_PACK_FORMS")) : 1;
  hipLaunchKernelGGL(k_pack_multi, dim3(gx > 0 ? gx : 64, n), dim3(256), 0, (hipStream_t)stream, jobs, range_flag(),
                     forms);
  ZP_LAUNCH_CHECK("zp_pack_weight_multi");
  return ZP_OK;
}

extern "C" int zp_bn_fold(const float* g, const float* b, const float* m, const float* v, const float* bias, float eps,
                          int C, float* scale, float* shift, void* stream) {
  ZP_CHECK_ARG(g && b && m && v && scale && shift && C > 0, "zp_bn_fold: bad args");
  hipLaunchKernelGGL(k_bn_fold, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, g, b, m, v, bias, eps, C,
                     scale, shift);
  ZP_LAUNCH_CHECK("zp_bn_fold");
  return ZP_OK;
}

extern "C" int zp_bn_train_finalize(float* partials, int parts, int C, long long count, float eps, float momentum,
                                    const float* gamma, const float* beta, const float* conv_bias, float* running_mean,
                                    float* running_var, int64_t* nbt, float* scale, float* shift, float* save,
                                    void* stream) {
  ZP_CHECK_ARG(partials && gamma && beta && running_mean && running_var && scale && shift && save && parts > 0 &&
                   C > 0 && count > 0,
               "zp_bn_train_finalize: bad args");
  (void)count;
  const BnFin f{eps, momentum, gamma, beta, conv_bias, running_mean, running_var, nbt, scale, shift, save};
  hipStream_t st = (hipStream_t)stream;
  // the partials buffer is the caller's scratch (zp_conv2d stats): level 1 merges in place
  int stride = 1;
  if (parts <= BN_MERGE1_MAX) {  // (both key-15 modes: one level, one launch)
    hipLaunchKernelGGL(k_bn_stat_merge1, dim3((C + 7) / 8), dim3(1024), 0, st, partials, parts, C, f);
    ZP_LAUNCH_CHECK("zp_bn_train_finalize (one level)");
    return ZP_OK;
  }
  if (parts > 2 * BN_MERGE_R) {
    const int groups = (C + 31) / 32;
    static const int env = getenv("ZP_BN_FUSED") ? atoi(getenv("ZP_BN_FUSED")) : 1;
    const bool fused_on = (g_bn_fused >= 0 ? g_bn_fused : env) != 0;
    if (fused_on) {
      unsigned* cnt = (unsigned*)(partials + (size_t)3 * parts * C);
      if (hipMemsetAsync(cnt, 0, (size_t)groups * sizeof(unsigned), st) != hipSuccess) {
        set_error("zp_bn_train_finalize: counter reset failed");
        return ZP_ERR_HIP;
      }
      hipLaunchKernelGGL(k_bn_stat_merge_fin, dim3(groups, (parts + BN_MERGE_R - 1) / BN_MERGE_R), dim3(256), 0, st,
                         partials, parts, C, cnt, f);
      ZP_LAUNCH_CHECK("zp_bn_train_finalize (fused merge)");
      return ZP_OK;
    }
    hipLaunchKernelGGL(k_bn_stat_merge, dim3(groups, (parts + BN_MERGE_R - 1) / BN_MERGE_R), dim3(256), 0, st,
                       partials, parts, C);
    ZP_LAUNCH_CHECK("zp_bn_train_finalize merge");
    stride = BN_MERGE_R;
  }
  hipLaunchKernelGGL(k_bn_train_finalize, dim3((C + 31) / 32), dim3(256), 0, st, partials, parts, stride, C, f);
  ZP_LAUNCH_CHECK("zp_bn_train_finalize");
  return ZP_OK;
}

extern "C" int zp_bn_apply(const void* x, int P, int C, const float* scale, const float* shift, const void* res, int ldr,
                           int cr0, int relu, int dtype, void* y, int ldy, int cy0, void* stream) {
  ZP_DTYPE_CHECK("zp_bn_apply", dtype);
  const int N = dtype == ZP_F32 ? 4 : 8;
  ZP_CHECK_ARG(x && y && scale && shift && P > 0 && C % N == 0 && ldy % N == 0 && cy0 % N == 0,
               "zp_bn_apply: bad args");
  if (res) ZP_CHECK_ARG(ldr % N == 0 && cr0 % N == 0, "zp_bn_apply: residual alignment");
  long total = (long)P * (C / N);
  const int CV = C / N;
  const char* ev = getenv("ZP_BN_APPLY_U");  // A/B knob (0: the grid-stride kernel), read per call
  const int use_u = ev ? atoi(ev) : 1;
  if (use_u && (CV & (CV - 1)) == 0 && 256 % CV == 0 && total < (1L << 31) - (1L << 20)) {
    constexpr int U = 4;
    const int cvs = __builtin_ctz((unsigned)CV);
    long g = (total + 256L * U - 1) / (256L * U);
    const dim3 grid((unsigned)(g > 65535 ? 65535 : g));
    hipStream_t st = (hipStream_t)stream;
    if (dtype == ZP_BF16)
      hipLaunchKernelGGL((k_bn_apply_u<bf16_t, U>), grid, dim3(256), 0, st, (const bf16_t*)x, (unsigned)total, cvs, C,
                         scale, shift, (const bf16_t*)res, ldr, cr0, relu, (bf16_t*)y, ldy, cy0);
    else if (dtype == ZP_F16)
      hipLaunchKernelGGL((k_bn_apply_u<f16_t, U>), grid, dim3(256), 0, st, (const f16_t*)x, (unsigned)total, cvs, C,
                         scale, shift, (const f16_t*)res, ldr, cr0, relu, (f16_t*)y, ldy, cy0);
    else
      hipLaunchKernelGGL((k_bn_apply_u<float, U>), grid, dim3(256), 0, st, (const float*)x, (unsigned)total, cvs, C,
                         scale, shift, (const float*)res, ldr, cr0, relu, (float*)y, ldy, cy0);
    ZP_LAUNCH_CHECK("zp_bn_apply");
    return ZP_OK;
  }
  if (dtype == ZP_BF16)
    hipLaunchKernelGGL(k_bn_apply<bf16_t>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                       (long)P, C, scale, shift, (const bf16_t*)res, ldr, cr0, relu, (bf16_t*)y, ldy, cy0);
  else if (dtype == ZP_F16)
    hipLaunchKernelGGL(k_bn_apply<f16_t>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, (const f16_t*)x,
                       (long)P, C, scale, shift, (const f16_t*)res, ldr, cr0, relu, (f16_t*)y, ldy, cy0);
  else
    hipLaunchKernelGGL(k_bn_apply<float>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, (const float*)x,
                       (long)P, C, scale, shift, (const float*)res, ldr, cr0, relu, (float*)y, ldy, cy0);
  ZP_LAUNCH_CHECK("zp_bn_apply");
  return ZP_OK;
}

extern "C" int zp_bn_bwd_parts(int P, int C) {
  const int pix = bn_bwd_pix(P, C);
  return (P + pix - 1) / pix;
}

extern "C" int zp_bn_bwd_reduce(const void* dy, int lddy, int cdy0, const void* y, int ldy, int cy0, const void* x, int P,
                                int C, const float* save, int relu, int dtype, float* partials, float* dgamma,
                                float* dbeta, int accumulate, void* stream) {
  ZP_DTYPE_CHECK_TRAIN("zp_bn_bwd_reduce", dtype);
  const int N = dtype == ZP_F32 ? 4 : 8;
  ZP_CHECK_ARG(dy && partials && P > 0 && C % N == 0 && relu >= 0 && relu <= 2 && (relu != 1 || y) &&
                   (relu != 2 || x) && (!x || save),
               "zp_bn_bwd_reduce: bad args");
  ZP_CHECK_ARG(C / N <= 256 || (C / N) % 256 == 0, "zp_bn_bwd_reduce: C %d", C);
  const int parts = zp_bn_bwd_parts(P, C);
  const int CV = C / N;
  const int cgroups = CV > 256 ? CV / 256 : 1;
  const int pix = bn_bwd_pix(P, C);
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(parts, cgroups);
#define ZP_BNR(T, M, HX)                                                                                           \
  hipLaunchKernelGGL((k_bn_bwd_reduce<T, M, HX>), grid, dim3(256), 0, st, (const T*)dy, lddy, cdy0, (const T*)y, ldy, \
                     cy0, (const T*)x, (long)P, C, save, partials, parts, pix)
#define ZP_BNR_T(T)             \
  do {                          \
    if (relu == 2)              \
      ZP_BNR(T, 2, true);       \
    else if (relu == 1 && x)    \
      ZP_BNR(T, 1, true);       \
    else if (relu == 1)         \
      ZP_BNR(T, 1, false);      \
    else if (x)                 \
      ZP_BNR(T, 0, true);       \
    else                        \
      ZP_BNR(T, 0, false);      \
  } while (0)
  if (dtype == ZP_BF16)
    ZP_BNR_T(bf16_t);
  else
    ZP_BNR_T(float);
#undef ZP_BNR_T
#undef ZP_BNR
  ZP_LAUNCH_CHECK("zp_bn_bwd_reduce");
  hipLaunchKernelGGL(k_bn_bwd_totals, dim3((C + 7) / 8), dim3(1024), 0, st, partials, parts, C, dgamma, dbeta,
                     accumulate, parts);
  ZP_LAUNCH_CHECK("zp_bn_bwd_reduce totals");
  return ZP_OK;
}

extern "C" int zp_bn_bwd_totals(float* partials, int parts, int C, int out_parts, float* dgamma, float* dbeta,
                                int accumulate, void* stream) {
  ZP_CHECK_ARG(partials && parts > 0 && out_parts > 0 && C > 0, "zp_bn_bwd_totals: bad args");
  hipLaunchKernelGGL(k_bn_bwd_totals, dim3((C + 7) / 8), dim3(1024), 0, (hipStream_t)stream, partials, parts, C,
                     dgamma, dbeta, accumulate, out_parts);
  ZP_LAUNCH_CHECK("zp_bn_bwd_totals");
  return ZP_OK;
}

extern "C" int zp_bn_bwd_apply(const void* dy, int lddy, int cdy0, const void* y, int ldy, int cy0, const void* x, int P,
                               int C, const float* save, const float* partials, const float* gamma, int relu, int dtype,
                               void* dx, void* dres, int lddres, int cdres0, int res_accumulate, void* stream) {
  ZP_DTYPE_CHECK_TRAIN("zp_bn_bwd_apply", dtype);
  const int N = dtype == ZP_F32 ? 4 : 8;
  ZP_CHECK_ARG(dy && P > 0 && C % N == 0 && relu >= 0 && relu <= 2 && (relu != 1 || y) && (relu != 2 || dx) &&
                   (!dx || (x && save && partials && gamma)),
               "zp_bn_bwd_apply: bad args");
  ZP_CHECK_ARG(C / N <= 256 || (C / N) % 256 == 0, "zp_bn_bwd_apply: C %d", C);
  const int parts = zp_bn_bwd_parts(P, C);
  const BnTile t = bn_tile(P, C, N);
  const dim3 grid(t.blocks, t.cgroups);
  hipStream_t st = (hipStream_t)stream;
#define ZP_BNA(T, M)                                                                                             \
  hipLaunchKernelGGL((k_bn_bwd_apply<T, M>), grid, dim3(256), 0, st, (const T*)dy, lddy, cdy0, (const T*)y, ldy,  \
                     cy0, (const T*)x, (long)P, C, save, partials, parts, gamma, (T*)dx, (T*)dres, lddres, cdres0, \
                     res_accumulate, t.pix)
#define ZP_BNA_T(T)     \
  do {                  \
    if (relu == 2)      \
      ZP_BNA(T, 2);     \
    else if (relu == 1) \
      ZP_BNA(T, 1);     \
    else                \
      ZP_BNA(T, 0);     \
  } while (0)
  if (dtype == ZP_BF16)
    ZP_BNA_T(bf16_t);
  else
    ZP_BNA_T(float);
#undef ZP_BNA_T
#undef ZP_BNA
  ZP_LAUNCH_CHECK("zp_bn_bwd_apply");
  return ZP_OK;
}

#define ZP_TLAUNCH(dt, KERNEL, grid, st, ...)                                                \
  do {                                                                                      \
    if ((dt) == ZP_BF16) {                                                                  \
      using T = bf16_t;                                                                     \
      hipLaunchKernelGGL(KERNEL<T>, grid, dim3(256), 0, st, __VA_ARGS__);                   \
    } else if ((dt) == ZP_F16) {                                                            \
      using T = f16_t;                                                                      \
      hipLaunchKernelGGL(KERNEL<T>, grid, dim3(256), 0, st, __VA_ARGS__);                   \
    } else {                                                                                \
      using T = float;                                                                      \
      hipLaunchKernelGGL(KERNEL<T>, grid, dim3(256), 0, st, __VA_ARGS__);                   \
    }                                                                                       \
  } while (0)

extern "C" int zp_im2col_split(const float* x, int B, int H, int W, int ldx, int C, int k, int s, int p, int OH,
                               int OW, int kpad, int dtype, void* y, void* stream) {
  ZP_CHECK_ARG(dtype == ZP_F32X3 || dtype == ZP_F32H2, "zp_im2col_split: dtype %d is not a split-fp32 form", dtype);
  ZP_CHECK_ARG(x && y && B > 0 && H > 0 && W > 0 && C > 0 && ldx >= C && k > 0 && s > 0 && p >= 0 && OH > 0 &&
                   OW > 0 && kpad % 8 == 0 && kpad >= k * k * C,
               "zp_im2col_split: bad args");
  const long total = (long)B * OH * OW * (kpad / 8);
  if (dtype == ZP_F32X3)
    hipLaunchKernelGGL(k_im2col_split<3>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, x, B, H, W, ldx,
                       C, k, s, p, OH, OW, kpad, (unsigned short*)y, nullptr);
  else
    hipLaunchKernelGGL(k_im2col_split<2>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, x, B, H, W, ldx,
                       C, k, s, p, OH, OW, kpad, (unsigned short*)y, range_flag());
  ZP_LAUNCH_CHECK("zp_im2col_split");
  return ZP_OK;
}

extern "C" int zp_nchw_to_nhwc(const float* x, int B, int C, int H, int W, int cpad, int dtype, void* y, void* stream) {
  ZP_DTYPE_CHECK("zp_nchw_to_nhwc", dtype);
  ZP_CHECK_ARG(x && y && B > 0 && C > 0 && cpad >= C, "zp_nchw_to_nhwc: bad args");
  ZP_TLAUNCH(dtype, k_nchw_to_nhwc, dim3(grid_for((long)B * H * W)), (hipStream_t)stream, x, B, C, H, W, cpad, (T*)y);
  ZP_LAUNCH_CHECK("zp_nchw_to_nhwc");
  return ZP_OK;
}

extern "C" int zp_maxpool3s2(const void* x, int B, int IH, int IW, int ldx, int cx0, int C, int dtype, void* y, int OH,
                             int OW, int ldy, int cy0, void* stream) {
  if (dtype == ZP_F32X3 || dtype == ZP_F32H2) {
    ZP_CHECK_ARG(x && y && C % 8 == 0 && cx0 % 8 == 0 && ldx % 8 == 0 && cy0 % 8 == 0 && ldy % 8 == 0,
                 "zp_maxpool3s2: bad args / alignment");
    ZP_CHECK_ARG(OH == (IH - 1) / 2 + 1 && OW == (IW - 1) / 2 + 1, "zp_maxpool3s2: OH/OW");
    const long total = (long)B * OH * OW * (C / 8);
    if (dtype == ZP_F32X3)
      hipLaunchKernelGGL(k_maxpool_split<3>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                         (const unsigned short*)x, (long)B * IH * IW * ldx, B, IH, IW, ldx, cx0, C, (unsigned short*)y,
                         (long)B * OH * OW * ldy, OH, OW, ldy, cy0);
    else
      hipLaunchKernelGGL(k_maxpool_split<2>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                         (const unsigned short*)x, (long)B * IH * IW * ldx, B, IH, IW, ldx, cx0, C, (unsigned short*)y,
                         (long)B * OH * OW * ldy, OH, OW, ldy, cy0);
    ZP_LAUNCH_CHECK("zp_maxpool3s2");
    return ZP_OK;
  }
  ZP_DTYPE_CHECK("zp_maxpool3s2", dtype);
  const int N = dtype == ZP_F32 ? 4 : 8;
  ZP_CHECK_ARG(x && y && C % N == 0 && cx0 % N == 0 && ldx % N == 0 && cy0 % N == 0 && ldy % N == 0,
               "zp_maxpool3s2: bad args / alignment");
  ZP_CHECK_ARG(OH == (IH - 1) / 2 + 1 && OW == (IW - 1) / 2 + 1, "zp_maxpool3s2: OH/OW");
  long total = (long)B * OH * OW * (C / N);
  ZP_TLAUNCH(dtype, k_maxpool, dim3(grid_for(total)), (hipStream_t)stream, (const T*)x, B, IH, IW, ldx, cx0, C, (T*)y,
             OH, OW, ldy, cy0);
  ZP_LAUNCH_CHECK("zp_maxpool3s2");
  return ZP_OK;
}

extern "C" int zp_maxpool3s2_bwd(const void* x, int ldx, int cx0, const void* dy, int lddy, int cdy0, int B, int IH,
                                 int IW, int C, int OH, int OW, int dtype, void* dx, int lddx, int cdx0, int accumulate,
                                 void* stream) {
  ZP_DTYPE_CHECK_TRAIN("zp_maxpool3s2_bwd", dtype);
  const int N = dtype == ZP_F32 ? 4 : 8;
  ZP_CHECK_ARG(x && dy && dx && C % N == 0 && cx0 % N == 0 && cdy0 % N == 0 && cdx0 % N == 0,
               "zp_maxpool3s2_bwd: bad args");
  ZP_CHECK_ARG(OH == (IH + 1) / 2 && OW == (IW + 1) / 2, "zp_maxpool3s2_bwd: OH/OW must be the 3x3 s2 p1 output");
  const long total = (long)B * (((IH + 1) / 2 + MP_ROWS - 1) / MP_ROWS) * ((IW + 1) / 2) * (C / N);
  ZP_TLAUNCH(dtype, k_maxpool_bwd, dim3(grid_for(total)), (hipStream_t)stream, (const T*)x, ldx, cx0, (const T*)dy,
             lddy, cdy0, B, IH, IW, C, OH, OW, (T*)dx, lddx, cdx0, accumulate);
  ZP_LAUNCH_CHECK("zp_maxpool3s2_bwd");
  return ZP_OK;
}

extern "C" int zp_global_avgpool(const void* x, int B, int H, int W, int ldx, int cx0, int C, int dtype, void* y,
                                 void* stream) {
  if (dtype == ZP_F32X3 || dtype == ZP_F32H2) {  // y: [NPL][B][C]
    ZP_CHECK_ARG(x && y && B > 0 && H > 0 && W > 0 && C > 0, "zp_global_avgpool: bad args");
    if (C % 8 == 0 && cx0 % 8 == 0 && ldx % 8 == 0) {  // 16-byte vectors
      if (dtype == ZP_F32X3)
        hipLaunchKernelGGL(k_avgpool_split8<3>, dim3((C + 63) / 64, B), dim3(256), 0, (hipStream_t)stream,
                           (const unsigned short*)x, (long)B * H * W * ldx, H, W, ldx, cx0, C, (unsigned short*)y,
                           (long)B * C);
      else
        hipLaunchKernelGGL(k_avgpool_split8<2>, dim3((C + 63) / 64, B), dim3(256), 0, (hipStream_t)stream,
                           (const unsigned short*)x, (long)B * H * W * ldx, H, W, ldx, cx0, C, (unsigned short*)y,
                           (long)B * C);
    } else if (dtype == ZP_F32X3)
      hipLaunchKernelGGL(k_avgpool_split<3>, dim3((C + 63) / 64, B), dim3(256), 0, (hipStream_t)stream,
                         (const unsigned short*)x, (long)B * H * W * ldx, H, W, ldx, cx0, C, (unsigned short*)y,
                         (long)B * C);
    else
      hipLaunchKernelGGL(k_avgpool_split<2>, dim3((C + 63) / 64, B), dim3(256), 0, (hipStream_t)stream,
                         (const unsigned short*)x, (long)B * H * W * ldx, H, W, ldx, cx0, C, (unsigned short*)y,
                         (long)B * C);
    ZP_LAUNCH_CHECK("zp_global_avgpool");
    return ZP_OK;
  }
  ZP_DTYPE_CHECK("zp_global_avgpool", dtype);
  ZP_CHECK_ARG(x && y && B > 0 && H > 0 && W > 0 && C > 0, "zp_global_avgpool: bad args");
  const int N = dtype == ZP_F32 ? 4 : 8;
  if (C % N == 0 && cx0 % N == 0 && ldx % N == 0) {
    if (dtype == ZP_BF16)
      hipLaunchKernelGGL((k_hw_reduce_vec<bf16_t, 0>), dim3((C + 63) / 64, B), dim3(256), 0, (hipStream_t)stream,
                         (const bf16_t*)x, H, W, ldx, cx0, C, (bf16_t*)y);
    else if (dtype == ZP_F16)
      hipLaunchKernelGGL((k_hw_reduce_vec<f16_t, 0>), dim3((C + 63) / 64, B), dim3(256), 0, (hipStream_t)stream,
                         (const f16_t*)x, H, W, ldx, cx0, C, (f16_t*)y);
    else
      hipLaunchKernelGGL((k_hw_reduce_vec<float, 0>), dim3((C + 63) / 64, B), dim3(256), 0, (hipStream_t)stream,
                         (const float*)x, H, W, ldx, cx0, C, (float*)y);
  } else {
    ZP_TLAUNCH(dtype, k_avgpool, dim3((C + 63) / 64, B), (hipStream_t)stream, (const T*)x, H, W, ldx, cx0, C, (T*)y);
  }
  ZP_LAUNCH_CHECK("zp_global_avgpool");
  return ZP_OK;
}

extern "C" int zp_broadcast_hw(const void* src, int B, int C, int dtype, void* y, int H, int W, int ldy, int cy0,
                               void* stream) {
  if (dtype == ZP_F32X3 || dtype == ZP_F32H2) {  // src [NPL][B][C] -> the planes of y [NPL][B, H, W, ldy]
    ZP_CHECK_ARG(src && y && B > 0 && C > 0 && C % 8 == 0 && ldy % 8 == 0 && cy0 % 8 == 0,
                 "zp_broadcast_hw: bad args / alignment");
    const long total = (long)B * H * W * C;
    const int npl = dtype == ZP_F32X3 ? 3 : 2;
    for (int p = 0; p < npl; ++p)
      hipLaunchKernelGGL(k_broadcast_vec<bf16_t>, dim3(grid_for(total / 8)), dim3(256), 0, (hipStream_t)stream,
                         (const bf16_t*)src + (long)p * B * C, B, C, (bf16_t*)y + (long)p * B * H * W * ldy, H, W,
                         ldy, cy0);
    ZP_LAUNCH_CHECK("zp_broadcast_hw");
    return ZP_OK;
  }
  ZP_DTYPE_CHECK("zp_broadcast_hw", dtype);
  ZP_CHECK_ARG(src && y && B > 0 && C > 0, "zp_broadcast_hw: bad args");
  long total = (long)B * H * W * C;
  const int N = dtype == ZP_F32 ? 4 : 8;
  if (C % N == 0 && ldy % N == 0 && cy0 % N == 0) {
    ZP_TLAUNCH(dtype, k_broadcast_vec, dim3(grid_for(total / N)), (hipStream_t)stream, (const T*)src, B, C, (T*)y, H,
               W, ldy, cy0);
  } else {
    ZP_TLAUNCH(dtype, k_broadcast, dim3(grid_for(total)), (hipStream_t)stream, (const T*)src, B, C, 1.f, (T*)y, H, W,
               ldy, cy0, 0, 0);
  }
  ZP_LAUNCH_CHECK("zp_broadcast_hw");
  return ZP_OK;
}

extern "C" int zp_sum_hw(const void* dy, int B, int H, int W, int lddy, int cdy0, int C, int dtype, void* out,
                         void* stream) {
  ZP_DTYPE_CHECK_TRAIN("zp_sum_hw", dtype);
  ZP_CHECK_ARG(dy && out && B > 0 && C > 0, "zp_sum_hw: bad args");
  const int N = dtype == ZP_F32 ? 4 : 8;
  if (C % N == 0 && cdy0 % N == 0 && lddy % N == 0) {
    if (dtype == ZP_BF16)
      hipLaunchKernelGGL((k_hw_reduce_vec<bf16_t, 1>), dim3((C + 63) / 64, B), dim3(256), 0, (hipStream_t)stream,
                         (const bf16_t*)dy, H, W, lddy, cdy0, C, (bf16_t*)out);
    else
      hipLaunchKernelGGL((k_hw_reduce_vec<float, 1>), dim3((C + 63) / 64, B), dim3(256), 0, (hipStream_t)stream,
                         (const float*)dy, H, W, lddy, cdy0, C, (float*)out);
  } else {
    ZP_TLAUNCH(dtype, k_sum_hw, dim3((C + 63) / 64, B), (hipStream_t)stream, (const T*)dy, H, W, lddy, cdy0, C,
               (T*)out);
  }
  ZP_LAUNCH_CHECK("zp_sum_hw");
  return ZP_OK;
}

extern "C" int zp_add_broadcast_hw(const void* src, float mul, int B, int C, int dtype, void* y, int H, int W, int ldy,
                                   int cy0, int accumulate, void* stream) {
  ZP_DTYPE_CHECK_TRAIN("zp_add_broadcast_hw", dtype);
  ZP_CHECK_ARG(src && y && B > 0 && C > 0, "zp_add_broadcast_hw: bad args");
  long total = (long)B * H * W * C;
  ZP_TLAUNCH(dtype, k_broadcast, dim3(grid_for(total)), (hipStream_t)stream, (const T*)src, B, C, mul, (T*)y, H, W,
             ldy, cy0, accumulate, 1);
  ZP_LAUNCH_CHECK("zp_add_broadcast_hw");
  return ZP_OK;
}

extern "C" int zp_copy_slice(const void* x, int ldx, int cx0, int xdtype, void* y, int ldy, int cy0, int ydtype, int P,
                             int C, int accumulate, void* stream) {
  ZP_DTYPE_CHECK_TRAIN("zp_copy_slice", xdtype);
  ZP_DTYPE_CHECK_TRAIN("zp_copy_slice", ydtype);
  ZP_CHECK_ARG(x && y && P > 0 && C > 0, "zp_copy_slice: bad args");
  long total = (long)P * C;
  dim3 g(grid_for(total));
  hipStream_t st = (hipStream_t)stream;
  if (xdtype == ZP_BF16 && ydtype == ZP_BF16)
    hipLaunchKernelGGL((k_copy_slice<bf16_t, bf16_t>), g, dim3(256), 0, st, (const bf16_t*)x, ldx, cx0, (bf16_t*)y, ldy,
                       cy0, (long)P, C, accumulate);
  else if (xdtype == ZP_BF16)
    hipLaunchKernelGGL((k_copy_slice<bf16_t, float>), g, dim3(256), 0, st, (const bf16_t*)x, ldx, cx0, (float*)y, ldy,
                       cy0, (long)P, C, accumulate);
  else if (ydtype == ZP_BF16)
    hipLaunchKernelGGL((k_copy_slice<float, bf16_t>), g, dim3(256), 0, st, (const float*)x, ldx, cx0, (bf16_t*)y, ldy,
                       cy0, (long)P, C, accumulate);
  else
    hipLaunchKernelGGL((k_copy_slice<float, float>), g, dim3(256), 0, st, (const float*)x, ldx, cx0, (float*)y, ldy,
                       cy0, (long)P, C, accumulate);
  ZP_LAUNCH_CHECK("zp_copy_slice");
  return ZP_OK;
}

extern "C" int zp_head_grad_to_nhwc(const float* dmask, const float* dcode, int B, int L, int H, int W, int ldy,
                                    int dtype, void* y, void* stream) {
  ZP_DTYPE_CHECK_TRAIN("zp_head_grad_to_nhwc", dtype);
  ZP_CHECK_ARG(dmask && (dcode || L == 0) && y && ldy >= L + 1, "zp_head_grad_to_nhwc: bad args");
  ZP_TLAUNCH(dtype, k_head_grad, dim3(grid_for((long)B * H * W)), (hipStream_t)stream, dmask, dcode, B, L, H, W, ldy,
             (T*)y);
  ZP_LAUNCH_CHECK("zp_head_grad_to_nhwc");
  return ZP_OK;
}

extern "C" int zp_threshold(const float* logits, long long n, int out_f64, void* bits, void* stream) {
  ZP_CHECK_ARG(logits && bits && n >= 0, "zp_threshold: bad args");
  if (n == 0) return ZP_OK;
  hipLaunchKernelGGL(k_threshold, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, logits, (long)n, out_f64, bits);
  ZP_LAUNCH_CHECK("zp_threshold");
  return ZP_OK;
}

extern "C" int zp_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long long n, double lr,
                       double beta1, double beta2, double eps, long long step, void* stream) {
  ZP_CHECK_ARG(param && grad && exp_avg && exp_avg_sq && n >= 0 && step >= 1, "zp_adam: bad args");
  if (n == 0) return ZP_OK;
  double bc1 = 1.0 - pow(beta1, (double)step);
  double bc2 = 1.0 - pow(beta2, (double)step);
  hipLaunchKernelGGL(k_adam, dim3(grid_for(n, 256, 16384)), dim3(256), 0, (hipStream_t)stream, param, grad, exp_avg,
                     exp_avg_sq, (long)n, (float)(lr / bc1), (float)(1.0 - beta1), (float)beta2,
                     (float)(1.0 - beta2), (float)sqrt(bc2), (float)eps);
  ZP_LAUNCH_CHECK("zp_adam");
  return ZP_OK;
}

static int adam_multi(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                      float* const* exp_avg_sq, const long long* numel, double lr, double beta1, double beta2,
                      double eps, long long step, const float* step_dev, void* stream) {
  ZP_CHECK_ARG(count >= 0 && (count == 0 || (params && grads && exp_avg && exp_avg_sq && numel)) &&
                   (step >= 1 || step_dev),
               "zp_adam_multi: bad args");
  const double bc1 = step_dev ? 1.0 : 1.0 - pow(beta1, (double)step);
  const double bc2 = step_dev ? 1.0 : 1.0 - pow(beta2, (double)step);
  // each launch takes up to ADAM_MT non-empty tensors; the next launch starts where this one's scan
  // stopped (empty tensors are skipped, never counted twice)
  for (int t0 = 0; t0 < count;) {
    AdamTable T{};
    int nb = 0;
    T.count = 0;
    int t = t0;
    for (; t < count && T.count < ADAM_MT; ++t) {
      ZP_CHECK_ARG(numel[t] >= 0 && (numel[t] == 0 || (params[t] && grads[t] && exp_avg[t] && exp_avg_sq[t])),
                   "zp_adam_multi: tensor %d", t);
      if (numel[t] == 0) continue;
      const int k = T.count++;
      T.p[k] = params[t];
      T.g[k] = grads[t];
      T.m[k] = exp_avg[t];
      T.v[k] = exp_avg_sq[t];
      T.n[k] = numel[t];
      T.blk0[k] = nb;
      const long long blocks = (numel[t] + ADAM_CHUNK - 1) / ADAM_CHUNK;
      ZP_CHECK_ARG(nb + blocks < (1ll << 30), "zp_adam_multi: too many elements");
      nb += (int)blocks;
    }
    t0 = t;
    T.blk0[T.count] = nb;
    if (nb == 0) continue;
    hipLaunchKernelGGL(k_adam_multi, dim3(nb), dim3(256), 0, (hipStream_t)stream, T, (float)(lr / bc1),
                       (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)sqrt(bc2), (float)eps,
                       step_dev, lr, beta1, beta2);
    ZP_LAUNCH_CHECK("zp_adam_multi");
  }
  return ZP_OK;
}

extern "C" int zp_adam_multi(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                             float* const* exp_avg_sq, const long long* numel, double lr, double beta1, double beta2,
                             double eps, long long step, void* stream) {
  return adam_multi(count, params, grads, exp_avg, exp_avg_sq, numel, lr, beta1, beta2, eps, step, nullptr, stream);
}

extern "C" int zp_adam_multi_dev(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                                 float* const* exp_avg_sq, const long long* numel, double lr, double beta1,
                                 double beta2, double eps, const float* step_dev, void* stream) {
  ZP_CHECK_ARG(step_dev, "zp_adam_multi_dev: step_dev");
  return adam_multi(count, params, grads, exp_avg, exp_avg_sq, numel, lr, beta1, beta2, eps, 0, step_dev, stream);
}

extern "C" int zp_mask_interp(const float* x, int B, int H, int W, int OH, int OW, int dtype, void* y, int ldy, int cy0,
                              void* stream) {
  ZP_DTYPE_CHECK("zp_mask_interp", dtype);
  ZP_CHECK_ARG(x && y && B > 0 && H > 0 && W > 0 && OH > 0 && OW > 0 && ldy > cy0 && cy0 >= 0,
               "zp_mask_interp: bad args");
  ZP_TLAUNCH(dtype, k_mask_interp, dim3(grid_for((long)B * OH * OW)), (hipStream_t)stream, x, B, H, W, OH, OW, (T*)y,
             ldy, cy0);
  ZP_LAUNCH_CHECK("zp_mask_interp");
  return ZP_OK;
}

extern "C" int zp_mask_interp_bwd(const void* dy, int lddy, int cdy0, int B, int OH, int OW, int H, int W, int dtype,
                                  float* dx, int accumulate, void* stream) {
  ZP_DTYPE_CHECK_TRAIN("zp_mask_interp_bwd", dtype);
  ZP_CHECK_ARG(dy && dx && B > 0 && H > 0 && W > 0 && OH > 0 && OW > 0 && lddy > cdy0 && cdy0 >= 0,
               "zp_mask_interp_bwd: bad args");
  ZP_TLAUNCH(dtype, k_mask_interp_bwd, dim3(grid_for((long)B * H * W)), (hipStream_t)stream, (const T*)dy, lddy, cdy0,
             B, OH, OW, H, W, dx, accumulate);
  ZP_LAUNCH_CHECK("zp_mask_interp_bwd");
  return ZP_OK;
}
