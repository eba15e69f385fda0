// Split-fp32 (ZP_F32X3, include/zp.h) forward convolutions for gfx950: k_conv3 (generic implicit
// GEMM: strided / dilated / 1x1 convs, ConvTranspose phases, the merged ASPP, the NCHW head) and
// k_conv3s (3x3 stride-1 convs with activation-strip reuse), their shared epilogue and the host
// dispatch zp_conv2d calls for dtype ZP_F32X3.
#include <stdlib.h>
#include "zp_conv_kern.h"
#include "zp_conv3.h"

namespace zp {

// s_barrier + a compiler memory fence: the barrier intrinsic does not order memory accesses for
// the compiler, so a plain (C++) LDS load after it -- the fragment reads of the register-pipelined
// schedule and of k_conv3s -- could be hoisted above it and read a buffer another wave's LDS-DMA is
// still filling (seen as wrong 32-pixel groups in ~2% of the head's tiles at bs=32 with the fp16
// split).  The empty asm with a "memory" clobber pins every later memory access below the barrier.
__device__ __forceinline__ void block_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// k_conv3 epilogue: BN scale / shift (+ bias), split residual, ReLU, then split NHWC stores (NPL
// planes, SplitF32<NPL>) or the f32 NCHW head split.  acc[i][j] = 4 consecutive output channels x
// one pixel.
template <int NPL, int WC, int WP>
__device__ __forceinline__ void conv3_epilogue(const zp_conv_args& A, const zp_conv_sub& S, f32x4 (&acc)[WC][WP],
                                               const int p0, const int c0, const int wc, const int wp,
                                               const int lane, const int M, const int GHW, const int flags,
                                               unsigned* rflag) {
  using SP = SplitF32<NPL>;
  const int lr = lane & 15;
  bool bad = false;  // NPL == 2: a finite value beyond fp16's range (zp_split_range_flag)
  int pn[WP], poy[WP], pox[WP];
  bool pok[WP];
#pragma unroll
  for (int j = 0; j < WP; ++j) {
    const int p = p0 + wp * 16 * WP + j * 16 + lr;
    pok[j] = p < M;
    const int pp = pok[j] ? p : 0;
    const int n = pp / GHW, rr = pp - n * GHW;
    const int gy = rr / A.GW, gx = rr - gy * A.GW;
    pn[j] = n;
    poy[j] = gy * S.oys + S.oyo;
    pox[j] = gx * S.oxs + S.oxo;
  }
  const long psy = (long)A.N * S.OH * S.OW * S.ldy;
  const long psr = (long)A.N * S.OH * S.OW * A.ldr;
  // Paired form (k_conv3w's epilogue): v_permlane16_swap pairs the lane groups of cout blocks
  // (i, i + 1) so that a lane holds 8 consecutive channels of one pixel -- 16-byte stores (and
  // residual loads) per lane and plane instead of 8.  NHWC output with 8-aligned channel slices and
  // Cout a multiple of 32 (a block pair is then wholly in or out of range); flag 512: the 8-byte
  // form (A/B).
  if constexpr (WC % 2 == 0) {
    const bool paired = A.out_mode == ZP_OUT_NHWC && S.ldy % 8 == 0 && S.cy0 % 8 == 0 && A.Cout % 32 == 0 &&
                        (!A.res || (A.ldr % 8 == 0 && A.cr0 % 8 == 0)) && !(flags & 512);
    if (paired) {
      const int g = lane >> 4;
#pragma unroll
      for (int i = 0; i < WC; i += 2) {
        const int cs = c0 + wc * 16 * WC + (i + (g & 1)) * 16 + (g >> 1) * 8;  // this lane's 8 channels
        const bool cok = c0 + wc * 16 * WC + i * 16 < A.Cout;                  // (wave-uniform)
        float sc[8], sh[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          sc[r] = 1.f;
          sh[r] = 0.f;
        }
        if (cok && S.scale) {
          const float4 a0 = *(const float4*)(S.scale + cs), a1 = *(const float4*)(S.scale + cs + 4);
          sc[0] = a0.x; sc[1] = a0.y; sc[2] = a0.z; sc[3] = a0.w; sc[4] = a1.x; sc[5] = a1.y; sc[6] = a1.z; sc[7] = a1.w;
        }
        if (cok && S.shift) {
          const float4 a0 = *(const float4*)(S.shift + cs), a1 = *(const float4*)(S.shift + cs + 4);
          sh[0] = a0.x; sh[1] = a0.y; sh[2] = a0.z; sh[3] = a0.w; sh[4] = a1.x; sh[5] = a1.y; sh[6] = a1.z; sh[7] = a1.w;
        }
#pragma unroll
        for (int j = 0; j < WP; ++j) {
          float v[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {  // all lanes active (cross-lane op)
            const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][j][r]), __float_as_uint(acc[i + 1][j][r]),
                                                             false, false);
            v[r] = __uint_as_float(sw[0]);
            v[r + 4] = __uint_as_float(sw[1]);
          }
          if (!pok[j] || !cok) continue;
          const size_t pix = ((size_t)pn[j] * S.OH + poy[j]) * S.OW + pox[j];
#pragma unroll
          for (int r = 0; r < 8; ++r) v[r] = v[r] * sc[r] + sh[r];
          if (A.res) {
            const unsigned short* R = (const unsigned short*)A.res + pix * A.ldr + A.cr0 + cs;
            uint4 rq[NPL];
#pragma unroll
            for (int p = 0; p < NPL; ++p) rq[p] = *(const uint4*)(R + p * psr);
#pragma unroll
            for (int r = 0; r < 8; ++r) {
              unsigned short q[NPL];
#pragma unroll
              for (int p = 0; p < NPL; ++p) {
                const uint32_t w4[4] = {rq[p].x, rq[p].y, rq[p].z, rq[p].w};
                q[p] = (unsigned short)(w4[r >> 1] >> ((r & 1) * 16));
              }
              v[r] += SP::join(q);
            }
          }
          if (A.relu) {
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = fmaxf(v[r], 0.f);
          }
          uint32_t o[NPL][4];
#pragma unroll
          for (int r = 0; r < 8; r += 2) {
            unsigned short q0[NPL], q1[NPL];
            SP::split(v[r], q0);
            SP::split(v[r + 1], q1);
            if constexpr (NPL == 2) bad |= h2_overflow(v[r]) || h2_overflow(v[r + 1]);
#pragma unroll
            for (int p = 0; p < NPL; ++p) o[p][r >> 1] = (uint32_t)q0[p] | ((uint32_t)q1[p] << 16);
          }
          if ((flags & 16384) && v[0] != 1.f) continue;  // diagnostic: no stores (unless a value is exactly 1)
          unsigned short* Y = (unsigned short*)S.y + pix * S.ldy + S.cy0 + cs;
#pragma unroll
          for (int p = 0; p < NPL; ++p) *(uint4*)(Y + p * psy) = make_uint4(o[p][0], o[p][1], o[p][2], o[p][3]);
        }
      }
      if constexpr (NPL == 2) raise_range_flag(rflag, bad);
      return;
    }
  }
  const int cbase = c0 + wc * 16 * WC + (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < WC; ++i) {
    const int cf = cbase + i * 16;
    if (cf >= A.Cout) continue;
    const bool full = cf + 3 < A.Cout;
    float sc[4], sh[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sc[r] = (S.scale && cf + r < A.Cout) ? S.scale[cf + r] : 1.f;
      sh[r] = (S.shift && cf + r < A.Cout) ? S.shift[cf + r] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < WP; ++j) {
      if (!pok[j]) continue;
      const size_t pix = ((size_t)pn[j] * S.OH + poy[j]) * S.OW + pox[j];
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * sc[r] + sh[r];
      if (A.res) {
        const unsigned short* R = (const unsigned short*)A.res + pix * A.ldr + A.cr0 + cf;
        if (full) {
          uint32_t w[NPL][2];
#pragma unroll
          for (int p = 0; p < NPL; ++p) {
            const uint2 q = *(const uint2*)(R + p * psr);
            w[p][0] = q.x;
            w[p][1] = q.y;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            unsigned short q[NPL];
#pragma unroll
            for (int p = 0; p < NPL; ++p) q[p] = (unsigned short)(w[p][r >> 1] >> ((r & 1) * 16));
            v[r] += SP::join(q);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (cf + r < A.Cout) {
              unsigned short q[NPL];
#pragma unroll
              for (int p = 0; p < NPL; ++p) q[p] = R[r + p * psr];
              v[r] += SP::join(q);
            }
        }
      }
      if (A.relu) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      if (A.out_mode == ZP_OUT_HEAD_NCHW) {
        const size_t plane = (size_t)S.OH * S.OW;
        const size_t sp = (size_t)poy[j] * S.OW + pox[j];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = cf + r;
          if (c >= A.Cout) continue;
          if (c == 0) ((float*)S.y)[(size_t)pn[j] * plane + sp] = v[r];
          else ((float*)S.y2)[((size_t)pn[j] * (A.Cout - 1) + (c - 1)) * plane + sp] = v[r];
        }
        continue;
      }
      unsigned short q[4][NPL];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        SP::split(v[r], q[r]);
        if constexpr (NPL == 2) bad |= h2_overflow(v[r]);
      }
      if ((flags & 16384) && v[0] != 1.f) continue;  // diagnostic: no stores (unless a value is exactly 1)
      unsigned short* Y = (unsigned short*)S.y + pix * S.ldy + S.cy0 + cf;
      if (full) {
#pragma unroll
        for (int p = 0; p < NPL; ++p)
          *(uint2*)(Y + p * psy) = make_uint2((uint32_t)q[0][p] | ((uint32_t)q[1][p] << 16),
                                              (uint32_t)q[2][p] | ((uint32_t)q[3][p] << 16));
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (cf + r < A.Cout)
#pragma unroll
            for (int p = 0; p < NPL; ++p) Y[r + p * psy] = q[r][p];
      }
    }
  }
  if constexpr (NPL == 2) raise_range_flag(rflag, bad);
}

// split-K slice: the raw f32 sums of this tile into ws [M][Cout] (acc[i][j] = 4 consecutive output
// channels x one grid point)
template <int WC, int WP>
__device__ __forceinline__ void splitk_store(float* __restrict__ ws, const int Cout, const f32x4 (&acc)[WC][WP],
                                             const int p0, const int c0, const int wc, const int wp, const int lane,
                                             const int M) {
  const int lr = lane & 15;
  const int cbase = c0 + wc * 16 * WC + (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < WP; ++j) {
    const int p = p0 + wp * 16 * WP + j * 16 + lr;
    if (p >= M) continue;
#pragma unroll
    for (int i = 0; i < WC; ++i) {
      const int cf = cbase + i * 16;
      if (cf + 3 < Cout) {
        *(float4*)(ws + (size_t)p * Cout + cf) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (cf + r < Cout) ws[(size_t)p * Cout + cf + r] = acc[i][j][r];
      }
    }
  }
}

// split-K epilogue: thread per (grid point, 4 output channels) of sub-problem blockIdx.y; the
// slices summed in slice order (deterministic), then conv3_epilogue's BN / bias, split residual,
// ReLU and split store (NHWC output)
template <int NPL>
__global__ void k_splitk_epi(const zp_conv_args A, const float* __restrict__ ws, const int nsplit, unsigned* rflag) {
  using SP = SplitF32<NPL>;
  bool bad = false;
  const zp_conv_sub& S = A.sub[blockIdx.y];
  ws += (size_t)blockIdx.y * nsplit * ((size_t)A.N * A.GH * A.GW) * A.Cout;
  const int GHW = A.GH * A.GW, M = A.N * GHW, C4 = (A.Cout + 3) / 4;
  const long psy = (long)A.N * S.OH * S.OW * S.ldy;
  const long psr = (long)A.N * S.OH * S.OW * A.ldr;
  // vector form: a thread per (grid point, 8 channels), 16-byte loads of the slices and of the
  // residual, 16-byte stores per plane (the scalar form below stored 2 bytes per channel and plane)
  if (A.Cout % 8 == 0 && S.ldy % 8 == 0 && S.cy0 % 8 == 0 && (!A.res || (A.ldr % 8 == 0 && A.cr0 % 8 == 0))) {
    const int C8 = A.Cout / 8;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < (long)M * C8; e += (long)gridDim.x * blockDim.x) {
      const int p = (int)(e / C8), cf = (int)(e - (long)p * C8) * 8;
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int z = 0; z < nsplit; ++z) {  // slice order: the scalar form's sums, bit for bit
        const float* w = ws + ((size_t)z * M + p) * A.Cout + cf;
        const float4 a = *(const float4*)w, b = *(const float4*)(w + 4);
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
        v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
      }
      const int n = p / GHW, rr = p - n * GHW;
      const int gy = rr / A.GW, gx = rr - gy * A.GW;
      const size_t pix = ((size_t)n * S.OH + gy * S.oys + S.oyo) * S.OW + gx * S.oxs + S.oxo;
      uint4 rq[NPL];
      if (A.res) {
        const unsigned short* R = (const unsigned short*)A.res + pix * A.ldr + A.cr0 + cf;
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) rq[pl] = *(const uint4*)(R + pl * psr);
      }
      uint32_t o[NPL][4];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        float x = v[r] * (S.scale ? S.scale[cf + r] : 1.f) + (S.shift ? S.shift[cf + r] : 0.f);
        if (A.res) {
          unsigned short q[NPL];
#pragma unroll
          for (int pl = 0; pl < NPL; ++pl) {
            const uint32_t w4[4] = {rq[pl].x, rq[pl].y, rq[pl].z, rq[pl].w};
            q[pl] = (unsigned short)(w4[r >> 1] >> ((r & 1) * 16));
          }
          x += SP::join(q);
        }
        if (A.relu) x = fmaxf(x, 0.f);
        unsigned short q[NPL];
        SP::split(x, q);
        if constexpr (NPL == 2) bad |= h2_overflow(x);
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) {
          if (r & 1) o[pl][r >> 1] |= (uint32_t)q[pl] << 16;
          else o[pl][r >> 1] = q[pl];
        }
      }
      unsigned short* Y = (unsigned short*)S.y + pix * S.ldy + S.cy0 + cf;
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) *(uint4*)(Y + pl * psy) = make_uint4(o[pl][0], o[pl][1], o[pl][2], o[pl][3]);
    }
    if constexpr (NPL == 2) raise_range_flag(rflag, bad);
    return;
  }
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < (long)M * C4; e += (long)gridDim.x * blockDim.x) {
    const int p = (int)(e / C4), cf = (int)(e - (long)p * C4) * 4;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < nsplit; ++z) {
      const float* w = ws + ((size_t)z * M + p) * A.Cout + cf;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (cf + r < A.Cout) v[r] += w[r];
    }
    const int n = p / GHW, rr = p - n * GHW;
    const int gy = rr / A.GW, gx = rr - gy * A.GW;
    const size_t pix = ((size_t)n * S.OH + gy * S.oys + S.oyo) * S.OW + gx * S.oxs + S.oxo;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (cf + r >= A.Cout) continue;
      float o = v[r] * (S.scale ? S.scale[cf + r] : 1.f) + (S.shift ? S.shift[cf + r] : 0.f);
      if (A.res) {
        const unsigned short* R = (const unsigned short*)A.res + pix * A.ldr + A.cr0 + cf + r;
        unsigned short q[NPL];
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) q[pl] = R[pl * psr];
        o += SP::join(q);
      }
      if (A.relu) o = fmaxf(o, 0.f);
      unsigned short q[NPL];
      SP::split(o, q);
      if constexpr (NPL == 2) bad |= h2_overflow(o);
      unsigned short* Y = (unsigned short*)S.y + pix * S.ldy + S.cy0 + cf + r;
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) Y[pl * psy] = q[pl];
    }
  }
  if constexpr (NPL == 2) raise_range_flag(rflag, bad);
}

// The correction terms of a split product (besides hi*hi, plane 0 x plane 0, into the main
// accumulator): plane pairs (A[t], B[t]) of (weight, activation)
template <int NPL> struct Terms;
template <> struct Terms<3> {  // mid*mid, hi*lo, lo*hi, mid*hi, hi*mid
  static constexpr int N = 5;
  static constexpr int A[5] = {1, 0, 2, 1, 0}, B[5] = {1, 2, 0, 0, 1};
};
template <> struct Terms<2> {  // hi*lo', lo'*hi (scaled by 2^-11 at the flush)
  static constexpr int N = 2;
  static constexpr int A[2] = {0, 1}, B[2] = {1, 0};
};
template <int NPL> using SplitMfma = MfmaTraits<std::conditional_t<NPL == 3, bf16_t, f16_t>>;

// acc += c2 * CS (the correction accumulator's flush; CS = 1 for the bf16 split)
template <int NPL>
__device__ __forceinline__ void flush_corr(f32x4& acc, const f32x4& c2) {
  if constexpr (NPL == 3) {
    acc += c2;
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = __builtin_fmaf(c2[r], SplitF32<NPL>::CS, acc[r]);
  }
}

// ------------------------------------------------------------------------------------
// k_conv3: forward convolution on ZP_F32X3 operands (split fp32, zp.h): activations, packed weights
// and the residual are three bf16 planes (hi, mid, lo) whose sum is the f32 value exactly.  Every
// product a * b is formed from its six terms of magnitude >= 2^-16 |a b|:
//   hi*hi + hi*mid + mid*hi + hi*lo + mid*mid + lo*hi
// on v_mfma_f32_16x16x32_bf16 (f32 accumulate); the dropped terms (mid*lo, lo*mid, lo*lo) are below
// 2^-23 |a b|, the order of f32's own product rounding.  That is f32-accurate arithmetic at 6 bf16
// MFMAs per 16x16x32 product block = 6/16 of the v_mfma_f32_16x16x4_f32 cost, and -- since the three
// B planes are staged once and each fragment feeds 3 / 2 / 1 MFMAs -- half the LDS traffic per MFMA
// of the bf16 kernels.
// Two accumulators per tile: hi*hi products in acc, the five correction terms in acc2, added once at
// the end.  Measured (tools/x3_accuracy.py, R34 bs=32): with the correction sums added straight into
// the full-size accumulator every conv carried a systematic NEGATIVE bias of ~-1e-7 relative (the
// bf16 MFMA's internal alignment drops the low bits of addends far below the accumulator), which
// compounded to 3x the exact-f32 engine's end-to-end error; accumulated among themselves the
// correction terms keep their bits.
// Tile: 2 NWP waves = 2 (cout) x NWP (pixel) computing TC = 32 WC output channels x TP = 64 NWP
// pixels.  A K step is one tap x 32 input channels.  Staging: per plane, a 16-row x 32-element tile
// (1 KB) is ONE buffer_load ... lds of 64 lanes, lane l fetching (row l & 15, 8 elements at k (l >>
// 4) * 8): the LDS image is in MFMA fragment order, so every fragment read is a lane-linear
// conflict-free ds_read_b128.  ST-deep ring; the tap walk (scalar), validity masks and out-of-image
// zeros (offset past the buffer end) follow k_conv.
// Schedules:
//   PIPE = false (8 waves, 2 per SIMD): per step [next DMA][fragment reads][MFMAs][wait + barrier];
//     ping-pong (flags & 8): waves 4-7 run one barrier behind, so on each SIMD one wave's MFMAs
//     overlap its partner's reads.
//   PIPE = true (NWP = 2: 4 waves, one per SIMD, 512-register budget): the fragments of step k + 1
//     are read into a second register set while step k's MFMAs run, and the DMA runs ST steps
//     ahead; per step one counted vmcnt wait + one barrier, no LDS read on the MFMA critical path.
// ------------------------------------------------------------------------------------
template <int NPL, int WC, int WP, int NWP, int ST, bool PIPE>
__global__ void __launch_bounds__(128 * NWP) k_conv3(const zp_conv_args A, const conv_taps TG, const int flags,
                                                     float* __restrict__ ws, const int nsplit) {
  constexpr int TC = 32 * WC, TP = 16 * WP * NWP, NW = 2 * NWP;
  constexpr int NTW = TC / 16, NT = (TC + TP) / 16;  // weight tiles / all tiles (16 rows) per plane
  constexpr int UNITS = NPL * NT;                    // (plane, tile) DMA units per stage
  constexpr int TPW = (NT + NW - 1) / NW;            // tiles per wave (some waves idle in the last)
  constexpr int GRP = NPL * TPW;                     // DMA instructions per wave per stage
  using MT = SplitMfma<NPL>;
  using TM = Terms<NPL>;
  static_assert(ST == 2 || ST == 3 || (PIPE && ST == 4), "ring depth");
  static_assert(ST == 2 || NT % NW == 0, "counted vmcnt waits need the same DMA count on every wave");
  static_assert(!PIPE || NW == 4, "the register-pipelined schedule runs one wave per SIMD");
  static_assert(WP == 4 || WP == 8, "pixel fragments per wave");
  __shared__ uint4 lds[ST * UNITS * 64];
  static_assert(ST * UNITS * 1024 <= 160 * 1024, "LDS");
  static_assert(((NPL - 1) * NT + WC + 3) * 1024 < 65536, "ds_read immediate range");
  // split-K (nsplit > 1): blockIdx.z = sub * nsplit + K slice; the slice's raw f32 sums go to ws
  // [nsub][nsplit][M][Cout] and k_splitk_epi finishes them
  int tb = (int)blockIdx.z / nsplit;
  const int kz = (int)blockIdx.z - tb * nsplit;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid / NWP, wp = wid % NWP;
  const int GHW = A.GH * A.GW;
  const int M = A.N * GHW;
  int bx = blockIdx.x, by = blockIdx.y;
  const int total = gridDim.x * gridDim.y;
  if ((flags & 1048576) && nsplit == 1 && A.nsub > 1 && (total & 7) == 0) {
    // several sub-problems over one input (the merged ASPP's four branches, zp_conv_tuning key 16,
    // off by default: see g_subint): the subs of a tile are dispatched next to each other on one
    // XCD (dispatch id % 8 picks the XCD), so the input rows they all read meet in that XCD's L2
    const int gid = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int q = gid >> 3;
    tb = q % A.nsub;
    const int tile = (gid & 7) * (total >> 3) + q / A.nsub;
    bx = tile / gridDim.y;
    by = tile - bx * gridDim.y;
  } else if (flags & 2) {  // XCD-aware order (k_conv): the cout tiles of a pixel tile meet in one L2
    const int bid = blockIdx.x + gridDim.x * blockIdx.y;
    const int lin = (total & 7) ? bid : (bid & 7) * (total >> 3) + (bid >> 3);
    bx = lin / gridDim.y;
    by = lin - bx * gridDim.y;
  }
  tb = __builtin_amdgcn_readfirstlane(tb);
  const zp_conv_sub& S = A.sub[tb];
  const int p0 = bx * TP, c0 = by * TC;
  const int CB = A.Cin / 32;
  const int ny = TG.ny[tb], nx = TG.nx[tb], dty = TG.dty[tb], dtx = TG.dtx[tb];
  const int nK_all = S.ntaps * CB;
  const int ks0 = (int)((long)kz * nK_all / nsplit);
  const int nK = (int)((long)(kz + 1) * nK_all / nsplit) - ks0;  // this slice's K steps
  const int lr = lane & 15, lk = (lane >> 4) * 8;
  // plane strides in bytes (scalar offsets of the DMA: the three planes of a tile share the lane's
  // offset register)
  const unsigned psx_b = (unsigned)((long)A.N * A.IH * A.IW * A.ldx * 2);
  const unsigned psw_b = (unsigned)((long)A.w_rows * A.k_pad * 2);

  // tiles of this wave: T = wid + NW k (all three planes each); wave-uniform kind, per-lane base
  // offset (plane 0, bytes) and tap validity masks
  unsigned ubase[TPW], uym[TPW], uxm[TPW];
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    const int t = wid + NW * k;
    ubase[k] = 0u;
    uym[k] = uxm[k] = 0u;
    if (t >= NT) continue;
    if (t < NTW) {
      ubase[k] = (unsigned)(((long)(c0 + t * 16 + lr) * A.k_pad + lk) * 2);
    } else {
      const int m = p0 + (t - NTW) * 16 + lr;
      const bool ok = m < M;
      const int mm = ok ? m : 0;
      const int n = mm / GHW, rr = mm - n * GHW;
      const int gy = rr / A.GW, gx = rr - gy * A.GW;
      const int y0 = gy * A.sy, x0 = gx * A.sx;
      ubase[k] = (unsigned)(((((long)n * A.IH + y0) * A.IW + x0) * A.ldx + A.cx0 + lk) * 2);
      unsigned ym = 0, xm = 0;
      for (int q = 0; q < ny; ++q) ym |= (unsigned)((unsigned)(y0 + TG.ty0[tb] + q * dty) < (unsigned)A.IH) << q;
      for (int q = 0; q < nx; ++q) xm |= (unsigned)((unsigned)(x0 + TG.tx0[tb] + q * dtx) < (unsigned)A.IW) << q;
      uym[k] = ok ? ym : 0u;
      uxm[k] = xm;
    }
  }
#if defined(__HIP_DEVICE_COMPILE__)
  const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)A.x, (short)0, (int)TG.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)S.w, (short)0, (int)TG.w_bytes[tb], 0x00020000);
#endif
  // scalar walk of the next step to issue.  K order: 32-channel chunk OUTER, taps inner -- the taps
  // of one chunk read nearly the same input rows (shifted by the tap offsets), so all but the
  // first come from L2; with the taps outer (k_conv's order) each tap's sweep over every chunk of
  // a tile evicted the rows before the next tap came back to them, and the staging ran at the
  // Infinity-Cache / HBM rate.  act_off = ((ty * IW + tx) * ldx + cb * 32) * 2; the weight offset
  // of (tap t, chunk cb) in the packed row (k = t * Cin + c) is w_koff = (t * Cin + cb * 32) * 2.
  // the walk starts at step ks0 = (chunk cb, tap t = tyi * nx + txi)
  int w_cb = ks0 / S.ntaps, w_t = ks0 - (ks0 / S.ntaps) * S.ntaps;
  int w_tyi = w_t / nx, w_txi = w_t - (w_t / nx) * nx;
  const int step_x = dtx * A.ldx * 2, step_y = dty * A.IW * A.ldx * 2;
  int act_off = ((TG.ty0[tb] * A.IW + TG.tx0[tb]) * A.ldx) * 2 + w_tyi * step_y + w_txi * step_x + w_cb * 64;
  int w_koff = (w_t * A.Cin + w_cb * 32) * 2;
  const int cin2 = A.Cin * 2;
  // diagnostic ablation flags (timing only, wrong results): 4096 no DMA after the prologue, 8192 no
  // MFMA, 16384 no epilogue stores
  const bool abl_dma = flags & 4096, abl_mfma = flags & 8192;
  auto issue = [&](int ks, int stage) {
    unsigned voff[TPW];
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      const bool w = wid + NW * k < NTW;
      const bool ok = (uym[k] >> w_tyi) & (uxm[k] >> w_txi) & 1u;
      voff[k] = w ? ubase[k] : (ok ? ubase[k] + (unsigned)act_off : 0x80000000u);
    }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      const int t = wid + NW * k;
      if (t >= NT) continue;
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) {
        auto* d = (__attribute__((address_space(3))) void*)&lds[(stage * UNITS + pl * NT + t) * 64];
        if (t < NTW) __builtin_amdgcn_raw_ptr_buffer_load_lds(wrsrc, d, 16, voff[k], pl * psw_b + w_koff, 0, 0);
        else __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, d, 16, voff[k], pl * psx_b, 0, 0);
      }
    }
#endif
    (void)ks;
    ++w_t;
    w_koff += cin2;
    act_off += step_x;
    if (++w_txi == nx) {
      w_txi = 0;
      act_off += step_y - nx * step_x;
      if (++w_tyi == ny) {
        w_tyi = 0;
        w_t = 0;
        ++w_cb;
        act_off += 64 - ny * step_y;
        w_koff = w_cb * 64;
      }
    }
  };

  // PIPE: a full second accumulator for the correction terms (one wave per SIMD has the registers);
  // otherwise each half of the pixel fragments gets a fresh correction accumulator per K step,
  // added into acc by VALU adds (round-to-nearest, unbiased) right after its MFMAs
  constexpr int A2C = PIPE ? WC : 1, A2P = PIPE ? WP : 1;
  f32x4 acc[WC][WP], acc2[A2C][A2P];
#pragma unroll
  for (int i = 0; i < WC; ++i)
#pragma unroll
    for (int j = 0; j < WP; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < A2C; ++i)
#pragma unroll
    for (int j = 0; j < A2P; ++j) acc2[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const unsigned l0 = lds_addr(lds) + (unsigned)lane * 16u;
  unsigned abase[ST], bbase[ST];
#pragma unroll
  for (int s = 0; s < ST; ++s) {
    abase[s] = l0 + (unsigned)(s * UNITS + wc * WC) * 1024u;
    bbase[s] = l0 + (unsigned)(s * UNITS + NTW + wp * WP) * 1024u;
  }
  // fragment reads: inline-asm ds_read_b128 (waited on explicitly) in the single-register-set
  // schedule; plain LDS loads in the register-pipelined one, whose reads stay in flight across the
  // MFMAs -- the compiler then tracks their lgkmcnt itself (an asm read's destination registers
  // are "written" at issue for the compiler, which may copy them before the data lands)
  const int awo = (wc * WC) * 64 + lane, bwo = (NTW + wp * WP) * 64 + lane;
  auto read_a = [&](auto s_c, uint4 (&af)[NPL][WC]) {
    constexpr int s = decltype(s_c)::value;
    static_for<NPL>([&](auto p_c) {
      constexpr int p = decltype(p_c)::value;
      static_for<WC>([&](auto i) {
        if constexpr (PIPE) af[p][i] = lds[(s * UNITS + p * NT + i) * 64 + awo];
        else af[p][i] = ds_read16<(p * NT + i) * 1024>(abase[s]);
      });
    });
  };
  auto read_b = [&](auto s_c, auto j0_c, auto j1_c, uint4 (&bfr)[NPL][WP]) {  // pixel fragments [J0, J1)
    constexpr int s = decltype(s_c)::value, J0 = decltype(j0_c)::value, J1 = decltype(j1_c)::value;
    static_for<NPL>([&](auto p_c) {
      constexpr int p = decltype(p_c)::value;
      static_for<J1 - J0>([&](auto jj) {
        if constexpr (PIPE) bfr[p][J0 + jj] = lds[(s * UNITS + p * NT + J0 + jj) * 64 + bwo];
        else bfr[p][J0 + jj] = ds_read16<(p * NT + J0 + jj) * 1024>(bbase[s]);
      });
    });
  };
  using J0c = std::integral_constant<int, 0>;
  using JHc = std::integral_constant<int, WP / 2>;
  using JWc = std::integral_constant<int, WP>;
  auto read_frags = [&](auto s_c, uint4 (&af)[NPL][WC], uint4 (&bfr)[NPL][WP]) {
    read_a(s_c, af);
    read_b(s_c, J0c{}, JWc{}, bfr);
  };
  auto mfmas_part = [&](auto j0_c, auto j1_c, const uint4 (&af)[NPL][WC], const uint4 (&bfr)[NPL][WP]) {
    constexpr int J0 = decltype(j0_c)::value, J1 = decltype(j1_c)::value;
    // the correction terms (Terms<NPL>) -> acc2 / c2; hi*hi -> acc
    if (!abl_mfma && PIPE) {
      static_for<TM::N + 1>([&](auto t_c) {
        constexpr int t = decltype(t_c)::value;
#pragma unroll
        for (int i = 0; i < WC; ++i)
#pragma unroll
          for (int j = J0; j < J1; ++j) {
            if constexpr (t < TM::N) MT::mma(acc2[PIPE ? i : 0][PIPE ? j : 0], af[TM::A[t]][i], bfr[TM::B[t]][j]);
            else MT::mma(acc[i][j], af[0][i], bfr[0][j]);
          }
      });
    } else if (!abl_mfma) {
      // per half of the pixel fragments: corrections into a fresh c2, hi*hi into acc, then
      // acc += c2 on the VALU
      static_for<2>([&](auto h_c) {
        constexpr int H0 = J0 + decltype(h_c)::value * ((J1 - J0) / 2), HN = (J1 - J0) / 2;
        f32x4 c2[WC][HN];
#pragma unroll
        for (int i = 0; i < WC; ++i)
#pragma unroll
          for (int jj = 0; jj < HN; ++jj) c2[i][jj] = (f32x4){0.f, 0.f, 0.f, 0.f};
        static_for<TM::N>([&](auto t_c) {
          constexpr int t = decltype(t_c)::value;
#pragma unroll
          for (int i = 0; i < WC; ++i)
#pragma unroll
            for (int jj = 0; jj < HN; ++jj) MT::mma(c2[i][jj], af[TM::A[t]][i], bfr[TM::B[t]][H0 + jj]);
        });
#pragma unroll
        for (int i = 0; i < WC; ++i)
#pragma unroll
          for (int jj = 0; jj < HN; ++jj) MT::mma(acc[i][H0 + jj], af[0][i], bfr[0][H0 + jj]);
#pragma unroll
        for (int i = 0; i < WC; ++i)
#pragma unroll
          for (int jj = 0; jj < HN; ++jj) flush_corr<NPL>(acc[i][H0 + jj], c2[i][jj]);
      });
    } else {
#pragma unroll
      for (int p = 0; p < NPL; ++p)
#pragma unroll
        for (int i = 0; i < WC; ++i)
#pragma unroll
          for (int j = J0; j < J1; ++j) acc[i][j][0] += __uint_as_float(af[p][i].x ^ bfr[p][j].y);
    }
  };
  auto mfmas = [&](const uint4 (&af)[NPL][WC], const uint4 (&bfr)[NPL][WP]) { mfmas_part(J0c{}, JWc{}, af, bfr); };

  if constexpr (!PIPE) {
    const bool pingpong = NW == 8 && (flags & 8);
    // step ks reads buffer ks % ST; the DMA of step ks + ST - 1 is issued first into the buffer
    // step ks - 1 read (all waves passed the barrier that ended step ks - 1)
    auto step = [&](auto s_c, int ks) {
      constexpr int s = decltype(s_c)::value;
      const bool more = ks + ST - 1 < nK;
      if (more && !abl_dma) issue(ks + ST - 1, (s + ST - 1) % ST);
      uint4 af[NPL][WC], bfr[NPL][WP];
      // the second half of the pixel fragments is read while the first half's MFMAs run (the
      // buffer is not refilled before the barrier that ends this step)
      read_a(s_c, af);
      read_b(s_c, J0c{}, JHc{}, bfr);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      read_b(s_c, JHc{}, JWc{}, bfr);
      auto wait_next = [&]() {  // step ks + 1's DMA landed (the newest ST - 2 groups may remain)
        if (more && !abl_dma) vm_wait<GRP * (ST - 2)>();
        else vm_wait<0>();
      };
      if (pingpong) {
        wait_next();
        block_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
      if (flags & 4) __builtin_amdgcn_s_setprio(1);
      mfmas_part(J0c{}, JHc{}, af, bfr);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mfmas_part(JHc{}, JWc{}, af, bfr);
      __builtin_amdgcn_sched_barrier(0);
      if (flags & 4) __builtin_amdgcn_s_setprio(0);
      if (!pingpong) wait_next();
      block_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    issue(0, 0);
    if (ST == 3 && nK > 1) {
      issue(1, 1);
      vm_wait<GRP>();
    } else {
      vm_wait<0>();
    }
    block_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (pingpong && wid >= 4) block_barrier();
    if constexpr (ST == 3) {
      for (int ks = 0; ks < nK; ks += 3) {
        step(I0{}, ks);
        if (ks + 1 >= nK) break;
        step(I1{}, ks + 1);
        if (ks + 2 >= nK) break;
        step(I2{}, ks + 2);
      }
    } else {
      for (int ks = 0; ks < nK; ks += 2) {
        step(I0{}, ks);
        if (ks + 1 >= nK) break;
        step(I1{}, ks + 1);
      }
    }
    if (pingpong && wid < 4) block_barrier();
  } else {
    // Prologue: the DMA of steps 0 .. ST - 1 (buffer = step), then step 0's fragments.  Step ks
    // (fragments F[ks & 1] loaded): wait for them; wait for step ks + 1's DMA + barrier (buffer
    // (ks + 1) % ST complete; every wave has read buffer ks % ST); issue the DMA of step ks + ST into
    // buffer ks % ST; issue step ks + 1's fragment reads into F[(ks + 1) & 1]; run step ks's MFMAs.
    // two named fragment sets (a [2][3][WC] array of them was demoted to scratch memory)
    uint4 fa0[NPL][WC], fb0[NPL][WP], fa1[NPL][WC], fb1[NPL][WP];
    int issued = 0;
    for (int q = 0; q < ST; ++q)
      if (q < nK) {
        issue(q, q);
        ++issued;
      }
    // counted only when every wave issues the same DMA count per stage (NT % NW == 0): the head's
    // 10-tile stage (NT = 2 + 8 over 4 waves) gives waves 2 / 3 fewer pieces, and a count of GRP
    // left their first stage's second tile in flight (wrong 32-pixel groups, fp16 split)
    if constexpr (NT % NW == 0) {
      if (issued == ST) vm_wait<GRP * (ST - 1)>();
      else vm_wait<0>();
    } else {
      vm_wait<0>();
    }
    block_barrier();
    __builtin_amdgcn_sched_barrier(0);
    using Z0 = std::integral_constant<int, 0>;
    read_frags(Z0{}, fa0, fb0);
    auto pstep = [&](auto s_c, int ks, uint4 (&ca)[NPL][WC], uint4 (&cb)[NPL][WP], uint4 (&na)[NPL][WC],
                     uint4 (&nb)[NPL][WP]) {
      constexpr int s = decltype(s_c)::value;
      constexpr int sn = (s + 1) % ST;
      // this wave's reads of buffer s (F[ks]) have landed before the barrier below releases the
      // buffer to the next DMA
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      const bool next = ks + 1 < nK;
      if (next) {
        // outstanding DMA groups: steps ks + 1 .. min(ks + ST - 1, nK - 1); the newest
        // ST - 2 of them may stay in flight when they all exist
        if (ks + ST - 1 < nK && !abl_dma) vm_wait<GRP * (ST - 2)>();
        else vm_wait<0>();
        block_barrier();
        __builtin_amdgcn_sched_barrier(0);
        read_frags(std::integral_constant<int, sn>{}, na, nb);
        if (ks + ST < nK && !abl_dma) issue(ks + ST, s);
      }
      if (flags & 4) __builtin_amdgcn_s_setprio(1);
      mfmas(ca, cb);
      if (flags & 4) __builtin_amdgcn_s_setprio(0);
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    using S2 = std::integral_constant<int, 2 % ST>;
    using S3 = std::integral_constant<int, 3 % ST>;
    if constexpr (ST == 2) {
      for (int ks = 0; ks < nK; ks += 2) {
        pstep(S0{}, ks, fa0, fb0, fa1, fb1);
        if (ks + 1 >= nK) break;
        pstep(S1{}, ks + 1, fa1, fb1, fa0, fb0);
      }
    } else if constexpr (ST == 4) {  // buffer period 4, fragment-set period 2: unrolled by 4
      for (int ks = 0; ks < nK; ks += 4) {
        pstep(S0{}, ks, fa0, fb0, fa1, fb1);
        if (ks + 1 >= nK) break;
        pstep(S1{}, ks + 1, fa1, fb1, fa0, fb0);
        if (ks + 2 >= nK) break;
        pstep(S2{}, ks + 2, fa0, fb0, fa1, fb1);
        if (ks + 3 >= nK) break;
        pstep(S3{}, ks + 3, fa1, fb1, fa0, fb0);
      }
    } else {  // buffer period 3, fragment-set period 2: unrolled by 6
      for (int ks = 0; ks < nK; ks += 6) {
        pstep(S0{}, ks, fa0, fb0, fa1, fb1);
        if (ks + 1 >= nK) break;
        pstep(S1{}, ks + 1, fa1, fb1, fa0, fb0);
        if (ks + 2 >= nK) break;
        pstep(S2{}, ks + 2, fa0, fb0, fa1, fb1);
        if (ks + 3 >= nK) break;
        pstep(S0{}, ks + 3, fa1, fb1, fa0, fb0);
        if (ks + 4 >= nK) break;
        pstep(S1{}, ks + 4, fa0, fb0, fa1, fb1);
        if (ks + 5 >= nK) break;
        pstep(S2{}, ks + 5, fa1, fb1, fa0, fb0);
      }
    }
  }
  if constexpr (PIPE) {
#pragma unroll
    for (int i = 0; i < WC; ++i)
#pragma unroll
      for (int j = 0; j < WP; ++j) flush_corr<NPL>(acc[i][j], acc2[PIPE ? i : 0][PIPE ? j : 0]);
  }
  if (nsplit > 1) splitk_store<WC, WP>(ws + ((size_t)tb * nsplit + kz) * M * A.Cout, A.Cout, acc, p0, c0, wc, wp, lane, M);
  else conv3_epilogue<NPL, WC, WP>(A, S, acc, p0, c0, wc, wp, lane, M, GHW, flags, TG.rflag);
}

// ------------------------------------------------------------------------------------
// k_conv3s: the split-fp32 3x3 stride-1 convolution with activation-strip reuse (k_conv_strip2's
// idea on k_conv3's operands).  k_conv3 stages the activation tile of every tap: 9 shifted copies
// of nearly the same rows per 32-channel chunk, and its staging (LDS-DMA, ~7 TB/s aggregate in
// these kernels) -- not the MFMAs -- bounds it (tools/conv3_ab.py: the kernel runs as long without
// MFMAs as with them).  Here a tile is TR = 256 / W full image rows and, per (32-channel chunk, tap
// row) group, ONE strip of TR x (W + 2 pad) input pixels (3 planes) is staged and read by the
// three taps of the row at column offsets 0, d, 2d; weights per tap as k_conv3.  Staged bytes per
// three taps: weights 72 KB + strip <= 54 KB instead of 72 + 144 KB.
// Strip image: 64 B (32 channels) per strip row and plane, its four 16 B chunks stored at
// c ^ ((row >> 1) & 2) -- a ds_read_b128 of ANY 16 consecutive rows (a fragment at any tap column)
// is then conflict-free (exhaustive search over the lane groups of ds_read_b128); the swizzle is
// applied on the per-lane DMA source address (LDS-DMA writes lane-linearly).
// Schedule per step (one tap column): next step's weights (double-buffered slot) and, at the
// group's first step, the next group's strip (double-buffered slot) are issued first; the A tile
// (3 planes x WC) is read whole, the strip fragments stream through a 2-deep ring (3 planes per
// pixel fragment); per pixel fragment a flushed correction accumulator (k_conv3's numerics);
// counted waits: at a group's first step only the weights are waited for (the strip has two more
// steps), later steps wait for all.  244 VGPRs at WC = 4, no spills.
// 8 waves = 2 (cout) x 4 (pixel), TC = 32 WC output channels x 256 pixels.
// ------------------------------------------------------------------------------------
struct strip3_geo {
  int W, TR, SW, SR;            // width, rows per tile, strip width W + 2 pad, strip rows TR * SW
  int ty0, dty, tx0, dtx, pad;  // tap grid (3 x 3) and the halo width
  unsigned x_bytes, w_bytes;
  unsigned* rflag;              // range flag of the two-plane stores (conv_taps::rflag)
};

// Ring depths (WSL weight slots, SSL strip slots): the weights of step s + WSL - 1 and the strip of
// group g + SSL - 1 are issued at step s / group g.  Round 4: layer1's convs ran at 2.1 us per step,
// 6x their MFMA time (profiles/r04_stages.md).  The cause was not the ring depth: the fragment reads
// were plain LDS loads, and the compiler put an s_waitcnt vmcnt(0) in front of the first read after
// each step's DMA issue, so every step waited for the staging of the next.  With inline-asm reads
// (below) layer1 / layer2 ran 64.7 -> 57.1 / 52.0 -> 43.8 us (tools/conv3_ab.py); 4 / 3 rings (3
// steps / 2 groups ahead, 134 KB, flag 1073741824) measured no better than 2 / 2.  Kernel-trace
// ablations of layer1 (57.9 us): without its DMA 52.9, without DMA and MFMAs 37.1, without stores
// too 25.8 -- the fixed per-workgroup and per-step costs of an 18-step K loop dominate.
// Every wave issues the same number of DMA instructions per event
// (WUW per weight step, SUW per strip; past the end or beyond its share: out-of-range no-ops), so
// with in-order vmcnt the wait at the end of a step is a constant: the loads issued after the next
// step's weights are (WSL - 2) weight events and the strips of the group starts among the last
// WSL - 1 steps.
// WP = 2 (round 4): 128-pixel tiles (a wave: 2 pixel blocks) with 144-row strips, 53 KB of LDS
// and ~70 VGPRs, so that three workgroups share a CU: the 64-channel layers' K loops are short
// (18 - 36 steps) and a lone workgroup's per-step latencies and epilogue stood unhidden.
template <int NPL, int WC, int WSL = 2, int SSL = 2, int WP = 4>
__global__ void __launch_bounds__(512) k_conv3s(const zp_conv_args A, const strip3_geo SG, const int flags) {
  constexpr int NW = 8;
  constexpr int TC = 32 * WC, TP = 64 * WP;
  constexpr int NTW = TC / 16;                  // weight tiles per plane
  constexpr int SRP = WP == 2 ? 144 : (WSL > 2 || SSL > 2) ? 272 : 288;  // strip rows per plane slot (>= SR, x16)
  constexpr int SB = SRP / 16;                  // strip row blocks per plane
  constexpr int SU = NPL * SB;                    // strip DMA units per group
  constexpr int SUW = (SU + NW - 1) / NW;       // per wave (padded with no-ops)
  constexpr int WU = NPL * NTW;                   // weight DMA units per step
  constexpr int WUW = (WU + NW - 1) / NW;
  constexpr int WSLOT = NPL * NTW * 1024;         // bytes per weight slot
  constexpr int SSLOT = NPL * SRP * 64;           // bytes per strip slot
  constexpr int DW = WSL - 1, DG = SSL - 1;       // steps / groups of lead
  static_assert(DW >= 1 && DW <= 3 && DG >= 1, "ring depths");
  constexpr bool PAD = WU % NW != 0 || SU % NW != 0;  // a 1 KB scratch block for the padding units
  __shared__ uint4 lds[(WSL * WSLOT + SSL * SSLOT + (PAD ? 1024 : 0)) / 16];
  static_assert(WSL * WSLOT + SSL * SSLOT + (PAD ? 1024 : 0) <= 160 * 1024, "LDS");
  const zp_conv_sub& S = A.sub[0];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid / 4, wp = wid % 4;
  const int GHW = A.GH * A.GW;
  const int M = A.N * GHW;
  int bx = blockIdx.x, by = blockIdx.y;
  if (flags & 2) {  // XCD-aware order (k_conv)
    const int total = gridDim.x * gridDim.y;
    const int bid = blockIdx.x + gridDim.x * blockIdx.y;
    const int lin = (total & 7) ? bid : (bid & 7) * (total >> 3) + (bid >> 3);
    bx = lin / gridDim.y;
    by = lin - bx * gridDim.y;
  }
  const int p0 = bx * TP, c0 = by * TC;
  const int n_img = p0 / GHW, y0 = (p0 - n_img * GHW) / SG.W;
  const int CB = A.Cin / 32;
  const int lr = lane & 15, lk = (lane >> 4) * 8;
  const long psw = (long)A.w_rows * A.k_pad;
#if defined(__HIP_DEVICE_COMPILE__)
  const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)A.x, (short)0, (int)SG.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)S.w, (short)0, (int)SG.w_bytes, 0x00020000);
#endif
  // weight units of this wave: u = wid + NW k -> (plane, tile); per-lane row offset (bytes, plane
  // included; out of range for the padding units); the (tap, chunk) offset is scalar
  unsigned wv[WUW];
#pragma unroll
  for (int k = 0; k < WUW; ++k) {
    const int u = wid + NW * k;
    const int pl = u / NTW, t = u - pl * NTW;
    wv[k] = u < WU ? (unsigned)((pl * psw + (long)(c0 + t * 16 + lr) * A.k_pad + lk) * 2) : 0x80000000u;
  }
  // strip units of this wave: v = wid + NW k -> (plane, row block); lane -> strip row rb * 16 +
  // lane / 4, LDS chunk position lane & 3 holding source chunk (lane & 3) ^ ((row >> 1) & 2).
  // sv: the source offset for tap row 0 / chunk 0 (plane included, 16 B aligned) with a 3-bit
  // "input row inside the image" mask per tap row in the low bits (0 for padding columns / rows)
  const int rowb = A.IW * A.ldx * 2;
  unsigned sv[SUW];
#pragma unroll
  for (int k = 0; k < SUW; ++k) {
    const int v = wid + NW * k;
    const int pl = v / SB, rb = v - pl * SB;
    const int R = rb * 16 + (lane >> 2);
    const int tr = R / SG.SW, col = R - tr * SG.SW;
    const int ix = col + SG.tx0;
    const int c = (lane & 3) ^ ((R >> 1) & 2);
    const bool ok = v < SU && R < SG.SR && (unsigned)ix < (unsigned)A.IW;
    unsigned m = 0;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
      m |= (unsigned)(ok && (unsigned)(y0 + tr + SG.ty0 + ky * SG.dty) < (unsigned)A.IH) << ky;
    const long base = (long)pl * A.N * A.IH * A.IW * A.ldx +
                      (((long)n_img * A.IH + y0 + tr + SG.ty0) * A.IW + ix) * A.ldx + A.cx0 + c * 8;
    sv[k] = ok ? ((unsigned)(base * 2) | m) : 0u;
  }

  // groups (cb outer, ky inner): the three tap rows of one chunk read neighbouring input rows;
  // step s = 3 g + kx
  const int ng = 3 * CB, nsteps = 3 * ng;
  const unsigned l0 = lds_addr(lds);
  auto issue_w = [&](int st) {  // weights of step st into slot st % WSL
    const int g = st / 3, kx = st - 3 * g;
    const int t = (g % 3) * 3 + kx, cb = g / 3;
    const int koff = st < nsteps ? (t * A.Cin + cb * 32) * 2 : 0;
    const int slot = st % WSL;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int k = 0; k < WUW; ++k) {
      const unsigned vo = st < nsteps ? wv[k] : 0x80000000u;
      const bool real = wid + NW * k < WU;  // (wave-uniform) padding units: zeros into the scratch block
      auto* d = (__attribute__((address_space(3))) void*)&lds[(real ? slot * WSLOT + (wid + NW * k) * 1024
                                                                    : WSL * WSLOT + SSL * SSLOT) / 16];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrsrc, d, 16, vo, koff, 0, 0);
    }
#else
    (void)koff; (void)slot;
#endif
  };
  auto issue_s = [&](int g) {  // strip of group g into slot g % SSL
    // the tap-row offset goes into the lane offset (32-bit VALU wrap: the tap-row-0 base may be
    // "negative"), the chunk into the scalar offset
    const int ky = g % 3, cb = g / 3;
    const bool live = g < ng;
    const unsigned rowoff = (unsigned)(ky * SG.dty * rowb);
    const int soff = live ? cb * 64 : 0;
    const int slot = g % SSL;
    unsigned so[SUW];
#pragma unroll
    for (int k = 0; k < SUW; ++k) so[k] = (live && ((sv[k] >> ky) & 1u)) ? (sv[k] & ~15u) + rowoff : 0x80000000u;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int k = 0; k < SUW; ++k) {
      const bool real = wid + NW * k < SU;  // (wave-uniform) padding units: zeros into the scratch block
      auto* d = (__attribute__((address_space(3))) void*)&lds[(real ? WSL * WSLOT + slot * SSLOT + (wid + NW * k) * 1024
                                                                    : WSL * WSLOT + SSL * SSLOT) / 16];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, d, 16, real ? so[k] : 0x80000000u, soff, 0, 0);
    }
#else
    (void)soff; (void)slot; (void)so;
#endif
  };

  f32x4 acc[WC][WP];
#pragma unroll
  for (int i = 0; i < WC; ++i)
#pragma unroll
    for (int j = 0; j < WP; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // fragment addresses: A (weight tile wc * WC + i of plane p, slot w); B (strip, tap column kx,
  // pixel fragment j): per-lane offsets in the strip plane
  // strip row of pixel fragment j at tap column 0 (the fragment at column kx starts kx * dtx rows
  // later; its swizzled address is formed per read: a few VALU beside the MFMAs)
  int brow[WP];
#pragma unroll
  for (int j = 0; j < WP; ++j) {
    const int q = wp * 16 * WP + j * 16 + lr;
    const int r = q / SG.W, x = q - r * SG.W;
    brow[j] = r * SG.SW + x;  // strip column 0 is input column tx0
  }
  const unsigned lch = (unsigned)(lane >> 4);
  // uint4 index of pixel fragment j's chunk at tap column kx in strip slot gs, plane 0
  // (formed per read, a few VALU beside the MFMAs: hoisted out of the loop, the (j, kx, slot)
  // addresses would not fit beside the fragments -- the empty asm keeps them in the loop)
  auto bidx = [&](int j, int kx, int gs) -> int {
    int b = brow[j];
    asm volatile("" : "+v"(b));
    const unsigned R = (unsigned)(b + kx * SG.dtx);
    return (WSL * WSLOT + gs * SSLOT) / 16 + (int)(R * 4u + (lch ^ ((R >> 1) & 2u)));
  };
  using MT = SplitMfma<NPL>;
  using TM = Terms<NPL>;
  // one pixel fragment j: the correction products into a flushed accumulator (WC tiles), then
  // hi x hi into acc and the correction added by VALU (k_conv3's numerics)
  auto frag = [&](auto j_c, const uint4 (&af)[NPL][WC], const uint4 (&bq)[NPL]) {
    constexpr int J = decltype(j_c)::value;
    f32x4 c2[WC];
#pragma unroll
    for (int i = 0; i < WC; ++i) c2[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    static_for<TM::N>([&](auto t_c) {
      constexpr int t = decltype(t_c)::value;
#pragma unroll
      for (int i = 0; i < WC; ++i) MT::mma(c2[i], af[TM::A[t]][i], bq[TM::B[t]]);
    });
#pragma unroll
    for (int i = 0; i < WC; ++i) MT::mma(acc[i][J], af[0][i], bq[0]);
#pragma unroll
    for (int i = 0; i < WC; ++i) {
      flush_corr<NPL>(acc[i][J], c2[i]);
      asm volatile("" : "+v"(acc[i][J]));  // keeps the add here (sunk to the next step's use, all
    }                                      // 4 WP correction accumulators would stay live)
  };

  // one step s = 3 g + KX: issue the weights of step s + DW and, at a group's first step, the strip
  // of group g + DG; read the A tile (NPL planes x WC) whole, stream the strip fragments through a
  // 2-deep ring (plain LDS loads: the compiler counts lgkmcnt for the reads left in flight)
  auto step = [&](auto kx_c, int st) {
    constexpr int KX = decltype(kx_c)::value;
    const int g = st / 3;
    // diagnostic ablations (timing only, wrong results): 4096 no ring DMA (4096 + 2048: issued
    // out of range, no transfers), 8192 no MFMAs
    if (!(flags & 4096)) {
      issue_w(st + DW);
      if (KX == 0) issue_s(g + DG);
    } else if (flags & 2048) {  // (with 4096: out-of-range issues, no transfers)
      issue_w(nsteps + st);
      if (KX == 0) issue_s(ng + g);
    }
    const int ws = st % WSL, gs = g % SSL;
    uint4 af[NPL][WC], bq0[NPL], bq1[NPL];
    // fragment reads: inline-asm ds_read_b128 with explicit lgkmcnt waits -- plain LDS loads after
    // the LDS-DMA issue above made the compiler wait for that DMA (s_waitcnt vmcnt(0)) before the
    // step's first read, i.e. every step waited for the staging of the next one
    const unsigned ab = l0 + (unsigned)(ws * WSLOT + wc * WC * 1024) + (unsigned)lane * 16u;
    static_for<NPL>([&](auto p_c) {
      constexpr int p = decltype(p_c)::value;
      static_for<WC>([&](auto i_c) {
        constexpr int i = decltype(i_c)::value;
        af[p][i] = ds_read16<(p * NTW + i) * 1024>(ab);
      });
    });
    auto rd_b = [&](int j, uint4 (&bq)[NPL]) {
      const unsigned bb = l0 + (unsigned)bidx(j, KX, gs) * 16u;
      static_for<NPL>([&](auto p_c) {
        constexpr int p = decltype(p_c)::value;
        bq[p] = ds_read16<p * SRP * 64>(bb);
      });
    };
    rd_b(0, bq0);
    rd_b(1, bq1);
    if (flags & 4) __builtin_amdgcn_s_setprio(1);
    static_for<WP>([&](auto j_c) {
      constexpr int J = decltype(j_c)::value;
      // fragment J's reads landed: the NPL reads of fragment J + 1 may remain (J + 1 < WP)
      asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(J + 1 < WP ? NPL : 0) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (!(flags & 8192)) {
        if constexpr (J % 2 == 0) frag(j_c, af, bq0);
        else frag(j_c, af, bq1);
      } else {
        asm volatile("" ::"v"(bq0[0].x), "v"(bq1[0].x), "v"(af[0][0].x));
      }
      if constexpr (J + 2 < WP) {
        if constexpr (J % 2 == 0) rd_b(J + 2, bq0);
        else rd_b(J + 2, bq1);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    __builtin_amdgcn_sched_barrier(0);
    if (flags & 4) __builtin_amdgcn_s_setprio(0);
    // the next step's weights (and at a group's last step the next group's strip, issued earlier)
    // must have landed: the loads issued after W(st + 1) are DW - 1 weight events and the strips of
    // the group starts among steps st - DW + 1 .. st
    constexpr int NGS = ((KX % 3) == 0 ? 1 : 0) + (DW > 1 && ((KX + 2) % 3) == 0 ? 1 : 0) +
                        (DW > 2 && ((KX + 1) % 3) == 0 ? 1 : 0);
    vm_wait<(DW - 1) * WUW + NGS * SUW>();
    block_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: the strips of groups 0 .. DG - 1, then the weights of steps 0 .. DW - 1
  for (int g = 0; g < DG; ++g) issue_s(g);
  for (int st = 0; st < DW; ++st) issue_w(st);
  vm_wait<(DW - 1) * WUW>();  // W(0) (and every strip before it)
  block_barrier();
  __builtin_amdgcn_sched_barrier(0);
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;
  using K2 = std::integral_constant<int, 2>;
  for (int st = 0; st < nsteps; st += 3) {
    step(K0{}, st);
    step(K1{}, st + 1);
    step(K2{}, st + 2);
  }
  conv3_epilogue<NPL, WC, WP>(A, S, acc, p0, c0, wc, wp, lane, M, GHW, flags, SG.rflag);
}


static int env_int(const char* name) {
  const char* v = getenv(name);
  return v ? atoi(v) : 0;
}

// zp_conv_tuning key 8.  256 (one workgroup per CU): layer2's 128 -> 128 3x3 at 32 x 32, bs 32
// (128 workgroups of 128 x 256) 107 -> 75 us on 64-channel strip tiles; 512 / 1024 also move
// layer4 / layer5 (256 / 512 workgroups) and slow them, 198 -> 248 / 715 -> 1450 us (g16 logs)
static int g_conv3_min_blocks = 256;

int conv3_min_blocks(int v) {
  const int old = g_conv3_min_blocks;
  g_conv3_min_blocks = v;
  return old;
}

// cout tile: 128 / 64 / 32 by Cout; a launch whose 128 x 256 grid would leave CUs idle (fewer
// workgroups than zp_conv_tuning key 8) takes 64-channel tiles instead (twice the workgroups)
int conv3_tc(const zp_conv_args& a) {
  if (conv3w_ok(a)) return 256;  // k_conv3w
  const int tc = a.Cout > 64 ? 128 : (a.Cout > 32 ? 64 : 32);
  if (tc == 128 && g_conv3_min_blocks > 0) {
    const long blocks = (((long)a.N * a.GH * a.GW + 255) / 256) * ((a.Cout + 127) / 128) * a.nsub;
    if (blocks < g_conv3_min_blocks) return 64;
  }
  return tc;
}

// k_conv3 tiles (4 waves, one per SIMD; tools/conv3_ab.py): 128 x 256 for 128-channel tiles, 64 x 128
// (register-pipelined, 3-deep ring) for 64-channel tiles, 32 x 128 for the head.
int conv3_tp(const zp_conv_args& a, int tc) {
  static const int sched = env_int("ZP_CONV3_SCHED");
  if (tc == 256) return conv3w_tp(a);  // k_conv3w (256, or the 256 x 128 tile)
  if (tc == 128) return sched == 1 ? 128 : 256;  // 8-wave ping-pong 128 x 256, or the pipelined 128 x 128
  return 128;
}

// k_conv3s eligibility: a 3x3 stride-1 same-size conv (one sub, the tap grid rows outer) on W 32 /
// 64 / 128 with whole-row 256-pixel tiles inside one image, 64- or 128-channel cout tiles, and a
// strip of TR x (W + 2 pad) <= 288 rows (layer5's dilation 4 at 32 x 32 needs 320: k_conv3).
// ZP_CONV3_STRIP=0 disables, =2 also takes the 128-channel tiles.
static int g_conv3_strip = -1;  // zp_conv_tuning key 7 (-1: ZP_CONV3_STRIP or the default 1)

int conv3_strip_mode(int v) {
  const int old = g_conv3_strip;
  g_conv3_strip = v;
  return old;
}

static bool conv3_strip(const zp_conv_args& a, int tc, strip3_geo* sg) {
  static const int env = getenv("ZP_CONV3_STRIP") ? env_int("ZP_CONV3_STRIP") : 1;
  const int en = g_conv3_strip >= 0 ? g_conv3_strip : env;
  // 128-channel tiles: k_conv3 (measured 2% faster than k_conv3s<4> on up1/up2, g13 logs) unless
  // ZP_CONV3_STRIP=2; 64-channel tiles: k_conv3s<2> (1.32x on layer1)
  if (!en || a.nsub != 1 || (tc != 128 && tc != 64) || a.Cout % tc != 0 || a.Cin % 32 != 0) return false;
  if (tc == 128 && en != 2) return false;
  if (a.sy != 1 || a.sx != 1 || a.GH != a.IH || a.GW != a.IW) return false;
  const zp_conv_sub& S = a.sub[0];
  if (S.ntaps != 9 || S.oys != 1 || S.oxs != 1 || S.oyo != 0 || S.oxo != 0 || S.OH != a.GH || S.OW != a.GW)
    return false;
  const int ty0 = S.ty[0], tx0 = S.tx[0], dty = S.ty[3] - S.ty[0], dtx = S.tx[1] - S.tx[0];
  for (int t = 0; t < 9; ++t)
    if (S.ty[t] != ty0 + (t / 3) * dty || S.tx[t] != tx0 + (t % 3) * dtx) return false;
  if (tx0 > 0 || tx0 + 2 * dtx < 0 || dtx < 0 || dty < 0) return false;
  const int W = a.GW;
  if (W != 32 && W != 64 && W != 128) return false;
  if (((long)a.GH * a.GW) % 256 != 0) return false;
  const int pad = max(-tx0, tx0 + 2 * dtx);  // left halo = -tx0; the strip spans [tx0, W - 1 + tx0 + 2 dtx]
  const int SW = W + 2 * dtx;
  const int TR = 256 / W, SR = TR * SW;
  if (SR > 288) return false;
  if (sg) {
    sg->W = W;
    sg->TR = TR;
    sg->SW = SW;
    sg->SR = SR;
    sg->ty0 = ty0;
    sg->dty = dty;
    sg->tx0 = tx0;
    sg->dtx = dtx;
    sg->pad = pad;
  }
  return true;
}

static int g_splitk = 1;  // zp_conv_tuning key 9: split-K of small split-fp32 launches (0 off)
// zp_conv_tuning key 16: interleave the subs of a multi-sub k_conv3 launch (-1: ZP_CONV3_SUBINT or 0).
// Measured (merged ASPP, bs 32): 585 -> 734 us with it on.  Each 3 x 3 branch's two-plane weights
// are 4.7 MB, an XCD's whole L2: branch after branch keeps one branch's weights hot, interleaving
// makes every XCD cycle through all four (x_high, 67 MB, is re-read from the Infinity Cache either way)
static int g_subint = -1;
int conv3_subint_mode(int v) {
  const int old = g_subint;
  g_subint = v;
  return old;
}

// zp_conv_tuning key 19: ring depth of the register-pipelined two-plane 64 x 128 k_conv3 tile (one
// wave per SIMD; 2, 3 or 4 stages; -1: ZP_CONV3_PIPE_ST or 2).  The DMA runs ST - 1 steps ahead of
// the step computing; the bs = 1 launches' split-K slices run 5-18 K steps each.  Measured (whole
// fp32 forward, hipGraph, tools/bs1_ab.py, profiles/r06_conv_ablations.md): bs 1 1.540 / 1.580 /
// 1.616 ms and bs 32 9.527 / 9.548 / 9.549 ms for 2 / 3 / 4 stages, bit-identical -- 2 stays
static int g_pipe_st = -1;
int conv3_pipe_st_mode(int v) {
  const int old = g_pipe_st;
  g_pipe_st = v;
  return old;
}
static int conv3_pipe_st() {
  static const int env = getenv("ZP_CONV3_PIPE_ST") ? atoi(getenv("ZP_CONV3_PIPE_ST")) : 2;
  const int v = g_pipe_st >= 0 ? g_pipe_st : env;
  return v == 3 || v == 4 ? v : 2;
}

int conv3_splitk_mode(int v) {
  const int old = g_splitk;
  g_splitk = v;
  return old;
}

// split-K slices of a split-fp32 launch: a one-sub NHWC conv whose grid leaves most CUs idle (under
// 256 workgroups -- bs = 1: layer5's 512 -> 512 runs as 64 workgroups over 144 K steps) is cut
// along K into up to 16 slices of >= 8 steps, for about 512 workgroups
int conv3_nsplit(const zp_conv_args& a) {
  if (!g_splitk || a.out_mode != ZP_OUT_NHWC || a.nsub < 1) return 1;
  const int tc = conv3_tc(a);
  if (tc == 256) return conv3w_splitk(a);
  const long blocks = (long)ceil_div((long)a.N * a.GH * a.GW, conv3_tp(a, tc)) * ceil_div(a.Cout, tc) * a.nsub;
  int nK = 1 << 30;  // the shortest sub-problem's K steps (ConvT phases: 1 .. 4 taps)
  for (int s = 0; s < a.nsub; ++s) nK = min(nK, a.sub[s].ntaps * (a.Cin / 32));
  if (blocks >= 256) return 1;
  int ns = 1;
  while (ns < 16 && blocks * ns * 2 <= 512 && nK / (ns * 2) >= (a.nsub > 1 ? 4 : 8)) ns *= 2;
  return ns;
}

// kernel launches for one split form (NPL planes: 3 = ZP_F32X3, 2 = ZP_F32H2)
template <int NPL>
static void conv3_dispatch(const zp_conv_args& a, const conv_taps& tg, int tc, hipStream_t st, int fl) {
  if (tc == 256) {  // 256 x 256 two-plane tile (zp_conv3w.hip), split-K for small grids
    const int ns = a.stats ? conv3w_splitk(a) : 1;
    conv3w_launch(a, tg, st, fl, (float*)a.stats, ns);
    if (ns > 1) {
      const long total = (long)a.N * a.GH * a.GW * ((a.Cout + 3) / 4);
      const int blocks = (int)(total + 255) / 256 < 8192 ? (int)((total + 255) / 256) : 8192;
      hipLaunchKernelGGL((k_splitk_epi<NPL>), dim3(blocks, a.nsub), dim3(256), 0, st, a, (const float*)a.stats, ns,
                         tg.rflag);
    }
    return;
  }
  const int ns = a.stats ? conv3_nsplit(a) : 1;
  float* ws = (float*)a.stats;
  strip3_geo s3{};
  if (ns == 1 && conv3_strip(a, tc, &s3)) {
    s3.x_bytes = tg.x_bytes;
    s3.w_bytes = tg.w_bytes[0];
    s3.rflag = tg.rflag;
    const dim3 sgrid((unsigned)(((long)a.N * a.GH * a.GW) / 256), (unsigned)(a.Cout / tc), 1);
    // (flags & 1073741824: the 4 / 3 rings on the two-plane 64-channel tile, A/B: measured 59.6 vs
    // 57.1 us on layer1, 45.0 vs 43.8 on layer2 -- the 2 / 2 rings stay the default)
    if (tc == 128) {
      hipLaunchKernelGGL((k_conv3s<NPL, 4>), sgrid, dim3(512), 0, st, a, s3, fl);
    } else if constexpr (NPL == 2) {
      // 128-pixel tiles (three workgroups per CU) unless flag 32 (A/B)
      const int tr2 = 128 / s3.W;
      if (!(fl & 32) && tr2 * s3.SW <= 144 && !(fl & 1073741824)) {
        strip3_geo h = s3;
        h.TR = tr2;
        h.SR = tr2 * s3.SW;
        const dim3 hgrid((unsigned)(((long)a.N * a.GH * a.GW) / 128), (unsigned)(a.Cout / tc), 1);
        hipLaunchKernelGGL((k_conv3s<NPL, 2, 2, 2, 2>), hgrid, dim3(512), 0, st, a, h, fl);
      } else if (s3.SR <= 272 && (fl & 1073741824)) {
        hipLaunchKernelGGL((k_conv3s<NPL, 2, 4, 3>), sgrid, dim3(512), 0, st, a, s3, fl);
      } else {
        hipLaunchKernelGGL((k_conv3s<NPL, 2>), sgrid, dim3(512), 0, st, a, s3, fl);
      }
    } else {
      hipLaunchKernelGGL((k_conv3s<NPL, 2>), sgrid, dim3(512), 0, st, a, s3, fl);
    }
    return;
  }
  const int tp = conv3_tp(a, tc);
  const int gx = ceil_div((long)a.N * a.GH * a.GW, tp), gy = ceil_div(a.Cout, tc);
  const dim3 grid(gx, gy, ns * a.nsub);
  static const int subint_env = getenv("ZP_CONV3_SUBINT") ? atoi(getenv("ZP_CONV3_SUBINT")) : 0;
  if ((g_subint >= 0 ? g_subint : subint_env) && a.nsub > 1) fl |= 1048576;
  // 128-channel layers: 8 waves, 128 x 256, 2-deep ring (two planes: 3-deep, the same LDS);
  // smaller tiles: register-pipelined one wave per SIMD over 128 pixels (ZP_CONV3_SCHED=1: the
  // 128-channel tile that way too)
  // (flags & 32768: the two-plane tile with the 2-deep ring, A/B)
  constexpr int ST8 = NPL == 2 ? 3 : 2;
  if (tc == 128 && tp == 256 && NPL == 2 && (fl & 32768))
    hipLaunchKernelGGL((k_conv3<NPL, 4, 4, 4, 2, false>), grid, dim3(512), 0, st, a, tg, fl, ws, ns);
  else if (tc == 128 && tp == 256)
    hipLaunchKernelGGL((k_conv3<NPL, 4, 4, 4, ST8, false>), grid, dim3(512), 0, st, a, tg, fl, ws, ns);
  else if (tc == 128) hipLaunchKernelGGL((k_conv3<NPL, 4, 4, 2, 2, true>), grid, dim3(256), 0, st, a, tg, fl, ws, ns);
  // (key 19, the deeper rings: the two-plane 64-channel tile only)
  else if (tc == 64 && NPL == 2 && conv3_pipe_st() == 3)
    hipLaunchKernelGGL((k_conv3<NPL, 2, 4, 2, NPL == 2 ? 3 : 2, true>), grid, dim3(256), 0, st, a, tg, fl, ws, ns);
  else if (tc == 64 && NPL == 2 && conv3_pipe_st() == 4)
    hipLaunchKernelGGL((k_conv3<NPL, 2, 4, 2, NPL == 2 ? 4 : 2, true>), grid, dim3(256), 0, st, a, tg, fl, ws, ns);
  else if (tc == 64) hipLaunchKernelGGL((k_conv3<NPL, 2, 4, 2, 2, true>), grid, dim3(256), 0, st, a, tg, fl, ws, ns);
  else hipLaunchKernelGGL((k_conv3<NPL, 1, 4, 2, 2, true>), grid, dim3(256), 0, st, a, tg, fl, ws, ns);
  if (ns > 1) {
    const long total = (long)a.N * a.GH * a.GW * ((a.Cout + 3) / 4);
    const int blocks = (int)(total + 255) / 256 < 8192 ? (int)((total + 255) / 256) : 8192;
    hipLaunchKernelGGL((k_splitk_epi<NPL>), dim3(blocks, a.nsub), dim3(256), 0, st, a, ws, ns, tg.rflag);
  }
}

int conv3_launch(const zp_conv_args& a, hipStream_t st, int fl, const zp_head_args* head) {
  const int npl = a.dtype == ZP_F32H2 ? 2 : 3;
  ZP_CHECK_ARG(a.Cin > 0 && a.Cin % 32 == 0, "zp_conv2d: split fp32 needs Cin %% 32 == 0 (got %d; the stem runs in f32 "
               "with out_mode ZP_OUT_NHWC_X3 / _H2)", a.Cin);
  ZP_CHECK_ARG(a.ldx >= a.cx0 + a.Cin && a.cx0 % 8 == 0 && a.ldx % 8 == 0, "zp_conv2d: bad ldx/cx0");
  ZP_CHECK_ARG(a.k_pad % 32 == 0, "zp_conv2d: k_pad %d not a multiple of 32", a.k_pad);
  // a.stats: for the split forms an optional f32 split-K workspace (zp_conv2d_split_ws bytes)
  ZP_CHECK_ARG(a.out_mode == ZP_OUT_NHWC || a.out_mode == ZP_OUT_HEAD_NCHW,
               "zp_conv2d: split fp32 writes split NHWC (ZP_OUT_NHWC) or the f32 head (ZP_OUT_HEAD_NCHW)");
  const int tc = conv3_tc(a);
  ZP_CHECK_ARG(a.w_rows % tc == 0 && a.w_rows >= a.Cout, "zp_conv2d: w_rows %d", a.w_rows);
  for (int s = 0; s < a.nsub; ++s) {
    const zp_conv_sub& S = a.sub[s];
    ZP_CHECK_ARG(S.w && S.y, "zp_conv2d: sub %d null w/y", s);
    ZP_CHECK_ARG(S.ntaps >= 1 && S.ntaps <= ZP_MAX_TAPS && (long)S.ntaps * a.Cin <= a.k_pad,
                 "zp_conv2d: sub %d ntaps %d / k_pad %d", s, S.ntaps, a.k_pad);
    if (a.out_mode == ZP_OUT_NHWC)
      ZP_CHECK_ARG(S.ldy >= S.cy0 + a.Cout && S.cy0 % 4 == 0 && S.ldy % 4 == 0, "zp_conv2d: bad ldy/cy0");
    else
      ZP_CHECK_ARG(S.y2 || a.Cout == 1, "zp_conv2d: head needs y2");
    // the epilogue's plane strides assume every sub writes the same output tensor shape
    ZP_CHECK_ARG(S.OH == a.sub[0].OH && S.OW == a.sub[0].OW, "zp_conv2d: split-fp32 subs must share the output shape");
  }
  if (a.res) ZP_CHECK_ARG(a.ldr >= a.cr0 + a.Cout && a.cr0 % 4 == 0 && a.ldr % 4 == 0, "zp_conv2d: bad residual ld");
  conv_taps tg{};
  const long long xb = (long long)npl * a.N * a.IH * a.IW * a.ldx * 2;
  const long long wb = (long long)npl * a.w_rows * a.k_pad * 2;
  ZP_CHECK_ARG(xb < (1ll << 31) && wb < (1ll << 31),
               "zp_conv2d: split input (%lld B) / weights (%lld B) must stay below 2 GiB per launch (split the batch)",
               xb, wb);
  tg.x_bytes = (unsigned)xb;
  tg.rflag = npl == 2 ? range_flag() : nullptr;
  for (int s = 0; s < a.nsub; ++s) {
    const zp_conv_sub& S = a.sub[s];
    tg.w_bytes[s] = (unsigned)wb;
    int nx = 1;
    while (nx < S.ntaps && S.ty[nx] == S.ty[0]) ++nx;
    const int ny = S.ntaps / nx;
    tg.ny[s] = ny;
    tg.nx[s] = nx;
    tg.ty0[s] = S.ty[0];
    tg.tx0[s] = S.tx[0];
    tg.dty[s] = ny > 1 ? S.ty[nx] - S.ty[0] : 0;
    tg.dtx[s] = nx > 1 ? S.tx[1] - S.tx[0] : 0;
    bool grid = ny * nx == S.ntaps && ny <= 32 && nx <= 32;
    for (int t = 0; grid && t < S.ntaps; ++t)
      grid = S.ty[t] == tg.ty0[s] + (t / nx) * tg.dty[s] && S.tx[t] == tg.tx0[s] + (t % nx) * tg.dtx[s];
    ZP_CHECK_ARG(grid, "zp_conv2d: sub %d taps must form a (row x column) grid of at most 32 x 32, rows outer", s);
  }
  if (head) {
    const zp_head_args& h = *head;
    ZP_CHECK_ARG(tc == 256 && a.Cout == 256 && a.nsub == 1 && npl == 2,
                 "zp_conv2d_head: not a fused-head geometry (zp_conv2d_head_ok)");
    ZP_CHECK_ARG(h.w && h.mask && (h.code || h.cout == 1) && h.cout >= 1 && h.cout <= 32, "zp_conv2d_head: bad head");
    ZP_CHECK_ARG(h.C2 >= 0 && h.C2 % 32 == 0 && h.k_pad % 8 == 0 && h.k_pad >= a.Cout + h.C2 && h.k_pad <= 504,
                 "zp_conv2d_head: C2 %d / k_pad %d", h.C2, h.k_pad);
    ZP_CHECK_ARG(h.C2 == 0 || (h.x2 && h.ldx2 % 8 == 0 && h.cx20 % 8 == 0 && h.ldx2 >= h.cx20 + h.C2),
                 "zp_conv2d_head: x2 layout");
    conv3w_head_launch(a, tg, h, st, fl);
    ZP_LAUNCH_CHECK("zp_conv2d_head");
    return ZP_OK;
  }
  if (npl == 2) conv3_dispatch<2>(a, tg, tc, st, fl);
  else conv3_dispatch<3>(a, tg, tc, st, fl);
  ZP_LAUNCH_CHECK("zp_conv2d split-f32");
  return ZP_OK;
}


bool conv3_strip_ok(const zp_conv_args& a, int tc) { return conv3_strip(a, tc, nullptr); }

}  // namespace zp
