// Implicit-GEMM convolution for gfx950 (MI355X): forward / data-gradient (k_conv)
// and weight-gradient (k_wgrad).  NHWC activations, packed [rows][tap*Cin] weights.
//
// Replaces the cuDNN convolutions behind nn.Conv2d / nn.ConvTranspose2d at
// model/resnet.py:41-51, model/aspp.py:60-80, 89-112 and the torchvision ResNet
// children reused at resnet.py:191-199 (see include/zp.h).
//
// Forward tile: one workgroup of 2*NWP waves (2 cout x NWP pixel) computes TC (=32*WC)
// output channels x TP (=64*NWP) pixels.  The MFMA A operand is the weight tile (rows =
// output channels), B is the activation tile (cols = pixels), so each lane ends up with 4
// consecutive output channels of one pixel -> 8/16 B NHWC stores.  K steps are 128 bytes per
// row (64 bf16 / 32 f32) of one tap, staged global -> LDS by LDS-DMA through a STAGES-deep
// ring (XOR-swizzled 16 B chunks, one barrier per K step).
#include <type_traits>
#include "zp_common.h"

// Diagnostic ablation builds only (tools/build_ablation.sh -> libzp_abl<N>.so; wrong results):
// ZP_ABL 1 = k_conv / k_conv_strip / k_wgrad_lds issue no LDS-DMA, 2 = they run no MFMA, 3 = k_conv
// / k_conv_strip stage only the weights (no activation DMA), 4 = k_conv_strip stages only the strips,
// 6 = the 16-bit NHWC epilogue stores nothing, 7 = it loads no BN scale / shift.
// The product build is ZP_ABL 0.
#ifndef ZP_ABL
#define ZP_ABL 0
#endif

#include "zp_conv_kern.h"
#include "zp_conv3.h"

namespace zp {

// all-zero source for out-of-image / padding taps of the direct-to-LDS loads
__device__ uint4 g_zero_page[8];

// Conv epilogue shared by k_conv and k_conv_strip: BN scale/shift (+bias), residual, ReLU,
// NHWC (channel slice) / NCHW-head / f32 stores, or train-mode BN partial statistics.
template <typename T, int WC, int WP, int NWP, bool BNR = false>
__device__ __forceinline__ void conv_epilogue(const zp_conv_args& A, const zp_conv_sub& S, f32x4 (&acc)[WC][WP],
                                              const int p0, const int c0, const int wc, const int wp, const int lane,
                                              const int M, const int GHW, const int bx, const int zi,
                                              const int nz, unsigned* rflag = nullptr, float* red = nullptr) {
  // ---------------- epilogue ----------------
  // (zi, nz): this tile's sub-problem and the sub-problem count, for the statistics part index
  // (blockIdx.z / gridDim.z, except in k_conv_quad, whose tiles hold all four sub-pixel phases)
  // output pixel of (lane, j): one division for j = 0, then +16 pixels per j
  int pn[WP], poy[WP], pox[WP];
  bool pok[WP];
  {
    const int pw0 = p0 + wp * 16 * WP + (lane & 15);
    int n = pw0 / GHW, rr = pw0 - n * GHW;
    int gy = rr / A.GW, gx = rr - gy * A.GW;
    const bool fast = A.GW % 16 == 0;
#pragma unroll
    for (int j = 0; j < WP; ++j) {
      const int p = pw0 + j * 16;
      pok[j] = p < M;
      if (j > 0) {
        if (fast) {
          gx += 16;
          if (gx >= A.GW) {
            gx -= A.GW;
            if (++gy == A.GH) {
              gy = 0;
              ++n;
            }
          }
        } else {
          n = p / GHW;
          rr = p - n * GHW;
          gy = rr / A.GW;
          gx = rr - gy * A.GW;
        }
      }
      pn[j] = n;
      poy[j] = gy * S.oys + S.oyo;
      pox[j] = gx * S.oxs + S.oxo;
    }
  }
  // BNR (k_conv_strip2's bnr instance): the fused BN backward sums (zp.h bnr_*) are taken in the
  // paired store loop below, on its 8-channel lanes (16-byte raw loads, issued before the pixel loop)
  constexpr bool BPAIR = BNR && sizeof(T) == 2 && WC % 2 == 0;
  bool bdone = false;  // the paired loop took them
  if constexpr (BPAIR) {
    if (A.bnr_part) __syncthreads();  // red (the kernel's LDS): every wave's main loop has finished reading it
  }
  bool stored = false;
  if constexpr (sizeof(T) == 2 && WC % 2 == 0) {
    // bf16 NHWC fast path: v_permlane16_swap pairs lane groups (g, g + 1) so that each lane
    // holds 8 consecutive output channels of one pixel (tiles i and i + 1 exchange halves):
    // 16 B stores (and residual loads), half the store instructions
    if (A.out_mode == ZP_OUT_NHWC && A.Cout % 8 == 0 && S.ldy % 8 == 0 && S.cy0 % 8 == 0 &&
        (!A.res || (A.ldr % 8 == 0 && A.cr0 % 8 == 0))) {
      stored = true;
      const int g = lane >> 4;
#pragma unroll
      for (int i = 0; i < WC; i += 2) {
        const int cs = c0 + wc * 16 * WC + (i + (g & 1)) * 16 + (g >> 1) * 8;
        const bool cok = cs < A.Cout;
        float sc[8], sh[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          sc[r] = 1.f;
          sh[r] = 0.f;
        }
        const float* psc = S.scale + cs;
        const float* psh = S.shift + cs;
        if (ZP_ABL != 7 && cok && S.scale) {
          const float4 s0 = *(const float4*)psc, s1 = *(const float4*)(psc + 4);
          sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w;
          sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
        }
        if (ZP_ABL != 7 && cok && S.shift) {
          const float4 s0 = *(const float4*)psh, s1 = *(const float4*)(psh + 4);
          sh[0] = s0.x; sh[1] = s0.y; sh[2] = s0.z; sh[3] = s0.w;
          sh[4] = s1.x; sh[5] = s1.y; sh[6] = s1.z; sh[7] = s1.w;
        }
        // BPAIR: this lane's 8 channels' BN terms and the raw x of its WP pixels, loaded up front
        uint4 bx8[BPAIR ? WP : 1];
        float bm[8], bi[8], bsc[8], bsh[8], bs0[8], bs1[8];
        if constexpr (BPAIR) {
          if (A.bnr_part) {
#pragma unroll
            for (int j = 0; j < WP; ++j) {
              const size_t pix = ((size_t)pn[j] * S.OH + poy[j]) * S.OW + pox[j];
              bx8[j] = (pok[j] && cok) ? *(const uint4*)((const unsigned short*)A.bnr_x + pix * A.Cout + cs)
                                       : make_uint4(0u, 0u, 0u, 0u);
            }
            float4 q[8];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              q[2 * t] = cok ? *(const float4*)(A.bnr_save + t * A.Cout + cs) : make_float4(0.f, 0.f, 0.f, 0.f);
              q[2 * t + 1] = cok ? *(const float4*)(A.bnr_save + t * A.Cout + cs + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
            float* dst[4] = {bm, bi, bsc, bsh};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              dst[t][0] = q[2 * t].x; dst[t][1] = q[2 * t].y; dst[t][2] = q[2 * t].z; dst[t][3] = q[2 * t].w;
              dst[t][4] = q[2 * t + 1].x; dst[t][5] = q[2 * t + 1].y; dst[t][6] = q[2 * t + 1].z; dst[t][7] = q[2 * t + 1].w;
            }
#pragma unroll
            for (int r = 0; r < 8; ++r) bs0[r] = bs1[r] = 0.f;
          }
        }
#pragma unroll
        for (int j = 0; j < WP; ++j) {
          float v[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {  // all lanes active here (cross-lane op)
            const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][j][r]),
                                                             __float_as_uint(acc[i + 1][j][r]), false, false);
            v[r] = __uint_as_float(sw[0]);
            v[r + 4] = __uint_as_float(sw[1]);
          }
          if (!pok[j] || !cok) continue;
          const size_t pix = ((size_t)pn[j] * S.OH + poy[j]) * S.OW + pox[j];
#pragma unroll
          for (int r = 0; r < 8; ++r) v[r] = v[r] * sc[r] + sh[r];
          if (A.res) {
            const uint4 rv = *(const uint4*)((const unsigned short*)A.res + pix * A.ldr + A.cr0 + cs);
            const uint32_t rw[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[2 * r] += H16<T>::from(rw[r] & 0xffffu);
              v[2 * r + 1] += H16<T>::from(rw[r] >> 16);
            }
          }
          if (A.relu) {
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = fmaxf(v[r], 0.f);
          }
          uint32_t o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = H16<T>::to(v[2 * r]) | (H16<T>::to(v[2 * r + 1]) << 16);
          if constexpr (BPAIR) {
            if (A.bnr_part) {  // g = the stored gradient; mask and xhat from the raw x (relu mode 2)
              const uint32_t xw[4] = {bx8[j].x, bx8[j].y, bx8[j].z, bx8[j].w};
#pragma unroll
              for (int r = 0; r < 8; ++r) {
                const float xx = H16<T>::from((r & 1) ? (xw[r >> 1] >> 16) : (xw[r >> 1] & 0xffffu));
                float g = H16<T>::from((r & 1) ? (o[r >> 1] >> 16) : (o[r >> 1] & 0xffffu));
                g = __builtin_fmaf(xx, bsc[r], bsh[r]) > 0.f ? g : 0.f;
                bs0[r] += g;
                bs1[r] += g * (xx - bm[r]) * bi[r];
              }
            }
          }
          if (ZP_ABL == 6 && o[0] != 0x3f803f80u) continue;  // diagnostic: no stores (unless a value pair is exactly 1, 1)
          if constexpr (ZP_ABL == 8) {  // diagnostic: non-temporal stores
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            u32x4* yp = (u32x4*)((unsigned short*)S.y + pix * S.ldy + S.cy0 + cs);
            __builtin_nontemporal_store((u32x4){o[0], o[1], o[2], o[3]}, yp);
          } else {
            *(uint4*)((unsigned short*)S.y + pix * S.ldy + S.cy0 + cs) = make_uint4(o[0], o[1], o[2], o[3]);
          }
        }
        if constexpr (BPAIR) {
          if (A.bnr_part) {
            bdone = true;
#pragma unroll
            for (int r = 0; r < 8; ++r) {  // over the 16 pixel lanes of this lane row (all lanes active)
              bs0[r] = row16_sum(bs0[r]);
              bs1[r] = row16_sum(bs1[r]);
            }
            if ((lane & 15) == 0) {  // red: [wp][sum][channel of the tile] (k_conv_strip2 passes it)
              const int ct = cs - c0;
              constexpr int TCB = 32 * WC;
              float* r0 = red + (wp * 2 + 0) * TCB + ct;
              float* r1 = red + (wp * 2 + 1) * TCB + ct;
              *(float4*)r0 = make_float4(bs0[0], bs0[1], bs0[2], bs0[3]);
              *(float4*)(r0 + 4) = make_float4(bs0[4], bs0[5], bs0[6], bs0[7]);
              *(float4*)r1 = make_float4(bs1[0], bs1[1], bs1[2], bs1[3]);
              *(float4*)(r1 + 4) = make_float4(bs1[4], bs1[5], bs1[6], bs1[7]);
            }
          }
        }
      }
    }
  }
  const int cbase = c0 + wc * 16 * WC + (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < WP && !stored; ++j) {
    if (!pok[j]) continue;
    const int n = pn[j], oy = poy[j], ox = pox[j];
    size_t pix = ((size_t)n * S.OH + oy) * S.OW + ox;
#pragma unroll
    for (int i = 0; i < WC; ++i) {
      const int cf = cbase + i * 16;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int c = cf + r;
        float sc = (S.scale && c < A.Cout) ? S.scale[c] : 1.f;
        float sh = (S.shift && c < A.Cout) ? S.shift[c] : 0.f;
        v[r] = acc[i][j][r] * sc + sh;
      }
      if (A.res) {
        const T* R = (const T*)A.res + pix * A.ldr + A.cr0 + cf;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (cf + r < A.Cout) v[r] += Elem<T>::ld(R + r);
      }
      if (A.relu) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      if (A.out_mode == ZP_OUT_HEAD_NCHW) {
        const size_t plane = (size_t)S.OH * S.OW;
        const size_t sp = (size_t)oy * S.OW + ox;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int c = cf + r;
          if (c >= A.Cout) continue;
          if (c == 0)
            ((float*)S.y)[(size_t)n * plane + sp] = v[r];
          else
            ((float*)S.y2)[((size_t)n * (A.Cout - 1) + (c - 1)) * plane + sp] = v[r];
        }
        continue;
      }
      if constexpr (sizeof(T) == 4) {
        if (A.out_mode == ZP_OUT_NHWC_X3 || A.out_mode == ZP_OUT_NHWC_H2) {
          // f32 call writing a split-fp32 tensor (the split-mode stem)
          const long psy = (long)A.N * S.OH * S.OW * S.ldy;
          unsigned short* Y = (unsigned short*)S.y + pix * S.ldy + S.cy0 + cf;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (cf + r >= A.Cout) continue;
            if (A.out_mode == ZP_OUT_NHWC_X3) {
              unsigned short q[3];
              SplitF32<3>::split(v[r], q);
              Y[r] = q[0];
              Y[r + psy] = q[1];
              Y[r + 2 * psy] = q[2];
            } else {
              unsigned short q[2];
              SplitF32<2>::split(v[r], q);
              Y[r] = q[0];
              Y[r + psy] = q[1];
              raise_range_flag(rflag, h2_overflow(v[r]));
            }
          }
          continue;
        }
      }
      if (A.out_mode == ZP_OUT_NHWC_F32 || sizeof(T) == 4) {
        float* Y = (float*)S.y + pix * S.ldy + S.cy0 + cf;
        if (cf + 3 < A.Cout) {
          *(float4*)Y = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (cf + r < A.Cout) Y[r] = v[r];
        }
      } else {
        unsigned short b[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          b[r] = (unsigned short)H16<T>::to(v[r]);
          v[r] = H16<T>::from(b[r]);  // statistics of the stored value
        }
        unsigned short* Y = (unsigned short*)S.y + pix * S.ldy + S.cy0 + cf;
        if (cf + 3 < A.Cout) {
          *(uint2*)Y = make_uint2((uint32_t)b[0] | ((uint32_t)b[1] << 16), (uint32_t)b[2] | ((uint32_t)b[3] << 16));
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (cf + r < A.Cout) Y[r] = b[r];
        }
      }
    }
  }
  if (A.stats) {
    // Train-mode BatchNorm statistics of the raw (stored) conv output, per wave half:
    // (count, mean, M2) with M2 centred on the local mean (two passes over the registers, no
    // E[x^2] - E[x]^2 cancellation); zp_bn_train_finalize merges the parts (Chan et al.).
    // red (k_conv_strip2, round 5): the NWP wave halves of a cout block are merged in LDS first, in
    // wave order (Chan's pairwise update in f32), and the tile writes one part
    // (zp_conv2d_stat_parts): a quarter of the partials for the merge to read -- at 128 x 128,
    // bs 32, 2048 parts instead of 8192 (that merge took 43 us)
    const int parts = red ? gridDim.x * nz : gridDim.x * nz * NWP;
    const int part = red ? zi * gridDim.x + bx : (zi * gridDim.x + bx) * NWP + wp;
    constexpr int TCS = 32 * WC;  // channels of the tile's cout block
    if (red) __syncthreads();  // every wave's last main-loop LDS read precedes the writes below
    float cnt = 0.f;
#pragma unroll
    for (int j = 0; j < WP; ++j) cnt += (p0 + wp * 16 * WP + j * 16 + (lane & 15) < M) ? 1.f : 0.f;
    if constexpr (sizeof(T) == 2) {
          cnt = row16_sum(cnt);
        } else {  // f32 parity mode: DPP temporaries pushed this 128-accumulator tile past 256 VGPRs
#pragma unroll
          for (int off = 1; off < 16; off <<= 1) cnt += __shfl_xor(cnt, off);
        }
#pragma unroll
    for (int i = 0; i < WC; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float vv[WP];
        float sm = 0.f;
#pragma unroll
        for (int j = 0; j < WP; ++j) {
          const bool ok = p0 + wp * 16 * WP + j * 16 + (lane & 15) < M;
          float v = acc[i][j][r];
          if (sizeof(T) == 2 && A.out_mode != ZP_OUT_NHWC_F32) v = H16<T>::from(H16<T>::to(v));  // stored value
          vv[j] = ok ? v : 0.f;
          sm += vv[j];
        }
        if constexpr (sizeof(T) == 2) {
          sm = row16_sum(sm);
        } else {  // f32 parity mode: DPP temporaries pushed this 128-accumulator tile past 256 VGPRs
#pragma unroll
          for (int off = 1; off < 16; off <<= 1) sm += __shfl_xor(sm, off);
        }
        const float mean = cnt > 0.f ? sm / cnt : 0.f;
        float m2 = 0.f;
#pragma unroll
        for (int j = 0; j < WP; ++j) {
          const bool ok = p0 + wp * 16 * WP + j * 16 + (lane & 15) < M;
          const float dlt = vv[j] - mean;
          m2 += ok ? dlt * dlt : 0.f;
        }
        if constexpr (sizeof(T) == 2) {
          m2 = row16_sum(m2);
        } else {  // f32 parity mode: DPP temporaries pushed this 128-accumulator tile past 256 VGPRs
#pragma unroll
          for (int off = 1; off < 16; off <<= 1) m2 += __shfl_xor(m2, off);
        }
        const int c = cbase + i * 16 + r;
        if (red) {
          if ((lane & 15) == 0) {  // [wp][cnt, mean, m2][channel of the tile]
            red[(wp * 3 + 0) * TCS + c - c0] = cnt;
            red[(wp * 3 + 1) * TCS + c - c0] = mean;
            red[(wp * 3 + 2) * TCS + c - c0] = m2;
          }
        } else if ((lane & 15) == 0 && c < A.Cout) {
          A.stats[(size_t)part * A.Cout + c] = cnt;
          A.stats[((size_t)parts + part) * A.Cout + c] = mean;
          A.stats[((size_t)2 * parts + part) * A.Cout + c] = m2;
        }
      }
    if (red) {
      __syncthreads();
      const int t = wc * NWP * 64 + wp * 64 + lane;  // flat thread id: thread t merges channel c0 + t
      if (t < TCS && c0 + t < A.Cout) {
        float n = red[t], mu = red[TCS + t], q = red[2 * TCS + t];
#pragma unroll
        for (int w = 1; w < NWP; ++w) {
          const float nw = red[(w * 3 + 0) * TCS + t];
          if (nw > 0.f) {
            const float mw = red[(w * 3 + 1) * TCS + t], qw = red[(w * 3 + 2) * TCS + t];
            const float nn = n + nw, d = mw - mu;
            mu += d * (nw / nn);
            q += qw + d * d * (n * nw / nn);
            n = nn;
          }
        }
        A.stats[(size_t)part * A.Cout + c0 + t] = n;
        A.stats[((size_t)parts + part) * A.Cout + c0 + t] = mu;
        A.stats[((size_t)2 * parts + part) * A.Cout + c0 + t] = q;
      }
    }
  }
  if (A.bnr_part) {
    // Data gradient feeding a train-mode BN + ReLU backward (zp.h bnr_*): per wave half, the sums
    // zp_bn_bwd_reduce (relu mode 2) takes over the stored gradient g -- masked where the forward's
    // fma(x, scale, shift) was <= 0 -- and g * xhat, xhat = (x - mean) * invstd of the BN's raw
    // input x at the same pixel.  The zp_conv2d checks leave no scale / shift / residual / ReLU here:
    // the stored value is the accumulator (rounded to T).  BPAIR (bdone): the paired store loop
    // took them into red already; otherwise (k_conv / k_conv_quad dgrads, the f32 parity mode) this
    // pass, 4 channels per lane, loads issued per channel block before their use.
    // red (k_conv_strip2: its LDS, free after the main loop): the NWP wave halves of a cout block meet
    // there and the tile writes one part (zp_conv2d_bnr_parts) -- a quarter of the partials for the
    // totals pass to read
    const int parts = red ? gridDim.x * nz : gridDim.x * nz * NWP;
    const int part = red ? zi * gridDim.x + bx : (zi * gridDim.x + bx) * NWP + wp;
    constexpr int TCB = 32 * WC;  // channels of the tile's cout block (2 wave rows of 16 * WC)
    if (!bdone) {
      if (red) __syncthreads();  // every wave's last main-loop LDS read precedes the writes below
      const float* sv = A.bnr_save;
      using XV = typename std::conditional<sizeof(T) == 2, uint2, float4>::type;
#pragma unroll
      for (int i = 0; i < WC; ++i) {
        const int cf = cbase + i * 16;
        const bool cok = cf < A.Cout;  // (Cout % 4 == 0: all four channels or none)
        XV xr[WP];
#pragma unroll
        for (int j = 0; j < WP; ++j) {
          const size_t pix = ((size_t)pn[j] * S.OH + poy[j]) * S.OW + pox[j];
          xr[j] = (pok[j] && cok) ? *(const XV*)((const T*)A.bnr_x + pix * A.Cout + cf) : XV{};
        }
        float4 pm[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) pm[q] = cok ? *(const float4*)(sv + q * A.Cout + cf) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float mean[4] = {pm[0].x, pm[0].y, pm[0].z, pm[0].w}, inv[4] = {pm[1].x, pm[1].y, pm[1].z, pm[1].w};
        const float msc[4] = {pm[2].x, pm[2].y, pm[2].z, pm[2].w}, msh[4] = {pm[3].x, pm[3].y, pm[3].z, pm[3].w};
        float sg[4] = {0.f, 0.f, 0.f, 0.f}, sgx[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < WP; ++j) {
          float xx[4];
          if constexpr (sizeof(T) == 2) {
            xx[0] = H16<T>::from(xr[j].x & 0xffffu);
            xx[1] = H16<T>::from(xr[j].x >> 16);
            xx[2] = H16<T>::from(xr[j].y & 0xffffu);
            xx[3] = H16<T>::from(xr[j].y >> 16);
          } else {
            xx[0] = xr[j].x; xx[1] = xr[j].y; xx[2] = xr[j].z; xx[3] = xr[j].w;
          }
          const bool ok = pok[j] && cok;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float g = acc[i][j][r];
            if (sizeof(T) == 2 && A.out_mode != ZP_OUT_NHWC_F32) g = H16<T>::from(H16<T>::to(g));  // stored value
            g = (ok && __builtin_fmaf(xx[r], msc[r], msh[r]) > 0.f) ? g : 0.f;
            sg[r] += g;
            sgx[r] += g * (xx[r] - mean[r]) * inv[r];
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if constexpr (sizeof(T) == 2) {
            sg[r] = row16_sum(sg[r]);
            sgx[r] = row16_sum(sgx[r]);
          } else {
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) {
              sg[r] += __shfl_xor(sg[r], off);
              sgx[r] += __shfl_xor(sgx[r], off);
            }
          }
        }
        if (red) {
          if ((lane & 15) == 0) {  // [wp][sum][channel of the tile]
            const int ct = cf - c0;
            *(float4*)(red + (wp * 2 + 0) * TCB + ct) = make_float4(sg[0], sg[1], sg[2], sg[3]);
            *(float4*)(red + (wp * 2 + 1) * TCB + ct) = make_float4(sgx[0], sgx[1], sgx[2], sgx[3]);
          }
        } else if ((lane & 15) == 0 && cok) {
          *(float4*)(A.bnr_part + (size_t)part * A.Cout + cf) = make_float4(sg[0], sg[1], sg[2], sg[3]);
          *(float4*)(A.bnr_part + ((size_t)parts + 1 + part) * A.Cout + cf) = make_float4(sgx[0], sgx[1], sgx[2], sgx[3]);
        }
      }
    }
    if (red) {
      __syncthreads();
      // the tile's sums over its NWP wave halves, in wave order: thread t < TCB sums channel t
      const int t = wc * NWP * 64 + wp * 64 + lane;  // flat thread id (wave = wc * NWP + wp)
      if (t < TCB && c0 + t < A.Cout) {
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int w = 0; w < NWP; ++w) {
          s0 += red[(w * 2 + 0) * TCB + t];
          s1 += red[(w * 2 + 1) * TCB + t];
        }
        A.bnr_part[(size_t)part * A.Cout + c0 + t] = s0;
        A.bnr_part[((size_t)parts + 1 + part) * A.Cout + c0 + t] = s1;
      }
    }
  }
}

// Staging: every K step moves TC weight rows + TP activation rows of 128 B each straight
// from global memory into LDS with global_load_lds_dwordx4 (one wave-instruction = 8 rows x
// 128 B, lane-linear in LDS).  The 16 B chunk swizzle (chunk ^ (row & 7), conflict-free
// ds_read_b128 of the MFMA fragments) is applied on the per-lane SOURCE address.  Out-of-
// image taps read g_zero_page.  STAGES LDS buffers: the loads of steps k+1..k+STAGES-1 are
// in flight while step k's MFMAs run; each step ends with a counted vmcnt wait (only the
// oldest step's loads) and a raw s_barrier.
template <typename T, int WC, int WP, int NWP, int STAGES, bool SMALLC>
__global__ void __launch_bounds__(128 * NWP) k_conv(const zp_conv_args A, const conv_taps TG, const int flags) {
  static_assert(STAGES == 2 || STAGES == 3, "2- or 3-deep LDS ring");
  constexpr int E = MfmaTraits<T>::E;
  constexpr int KE = 8 * E;  // elements per K step (128 B)
  constexpr int TC = 32 * WC, TP = 16 * WP * NWP;
  constexpr int NW = 2 * NWP;                 // waves
  constexpr int G = (TC + TP) / 8;            // 8-row groups per K step
  static_assert(G % NW == 0, "row groups must split evenly over the waves");
  constexpr int GPW = G / NW;                 // groups per wave
  // the first WPW groups of every wave are weight rows, the rest activation rows (group g = wid + NW*i
  // is a weight group iff i < WPW): compile-time, so per-pixel state exists only for pixel groups
  static_assert((TC / 8) % NW == 0, "weight groups must split evenly over the waves");
  constexpr int WPW = TC / 8 / NW;
  constexpr int LPS = ZP_ABL == 3 ? WPW : GPW;  // LDS-DMA instructions per wave per stage
  __shared__ uint4 lds0[(TC + TP) * 8];
  __shared__ uint4 lds1[(TC + TP) * 8];
  __shared__ uint4 lds2[STAGES == 3 ? (TC + TP) * 8 : 1];
  auto bufp = [&](auto i_c) -> uint4* {
    constexpr int i = decltype(i_c)::value;
    if constexpr (i == 0) return lds0;
    else if constexpr (i == 1) return lds1;
    else return lds2;
  };

  const zp_conv_sub& S = A.sub[blockIdx.z];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (scalar branches)
  const int wc = wid / NWP, wp = wid % NWP;
  const int GHW = A.GH * A.GW;
  const int M = A.N * GHW;
  // XCD-aware tile order (flags & 2): workgroups are dispatched round-robin over the
  // 8 XCDs, so consecutive linear ids land on different L2s.  Remap so that each XCD walks a
  // contiguous run of (pixel tile, cout tile) pairs, cout tiles fastest: the cout tiles of one
  // pixel tile (same activations) and neighbouring pixel tiles (shared halo rows) then meet in
  // the same L2.
  int bx = blockIdx.x, by = blockIdx.y;
  if (flags & 2) {
    const int total = gridDim.x * gridDim.y;
    const int bid = blockIdx.x + gridDim.x * blockIdx.y;
    const int lin = (total & 7) ? bid : (bid & 7) * (total >> 3) + (bid >> 3);
    bx = lin / gridDim.y;
    by = lin - bx * gridDim.y;
  }
  const int p0 = bx * TP, c0 = by * TC;
  const int lrow = lane >> 3;                  // row within the 8-row group
  const int csrc = (lane & 7) ^ lrow;          // source chunk (swizzle on the source side)

  // per group: weight row or activation row (pixel) of this lane
  int gpix_n[GPW], gpix_y[GPW], gpix_x[GPW];
  bool gvalid[GPW];
#pragma unroll
  for (int i = 0; i < GPW; ++i) {
    if (i < WPW) continue;
    const int r = (wid + NW * i) * 8 + lrow;
    int m = p0 + (r - TC);
    gvalid[i] = r >= TC && m < M;
    int mm = gvalid[i] ? m : 0;
    int n = mm / GHW, rr = mm - n * GHW;
    int gy = rr / A.GW, gx = rr - gy * A.GW;
    gpix_n[i] = n;
    gpix_y[i] = gy * A.sy;
    gpix_x[i] = gx * A.sx;
  }
  const T* __restrict__ X = (const T*)A.x;
  const T* __restrict__ Wt = (const T*)S.w;
  const int CB = SMALLC ? 1 : A.Cin / KE;
  int nK = SMALLC ? A.k_pad / KE : S.ntaps * CB;

  // ---- staging addresses (Cin >= 64 B-chunk path): buffer loads with per-lane 32-bit byte
  // offsets.  The tap walk (ty, tx, channel chunk) is scalar state advanced by one K step per
  // issue; per lane only the pixel's base offset and two validity bit masks (input row / column
  // in range, one bit per tap row / column) are kept.  Invalid taps use an offset past the
  // buffer's end, which the buffer unit returns as zeros: no address clamp, no select of a
  // zero page, no multiplies in the loop.
  const int tb = blockIdx.z;
  const int ny = TG.ny[tb], nx = TG.nx[tb], dty = TG.dty[tb], dtx = TG.dtx[tb];
  unsigned abase[GPW], ymask[GPW], xmask[GPW];
#pragma unroll
  for (int i = 0; i < GPW; ++i) {
    if (i < WPW) continue;
    const int y0 = gpix_y[i], x0 = gpix_x[i];
    abase[i] = (unsigned)(((((long)gpix_n[i] * A.IH + y0) * A.IW + x0) * A.ldx + A.cx0 + csrc * E) * sizeof(T));
    unsigned ym = 0, xm = 0;
    for (int q = 0; q < ny; ++q) ym |= (unsigned)((unsigned)(y0 + TG.ty0[tb] + q * dty) < (unsigned)A.IH) << q;
    for (int q = 0; q < nx; ++q) xm |= (unsigned)((unsigned)(x0 + TG.tx0[tb] + q * dtx) < (unsigned)A.IW) << q;
    ymask[i] = gvalid[i] ? ym : 0u;
    xmask[i] = xm;
  }
  // Tap-row trimming (flags & 16): a tap row whose input rows lie outside the image for every
  // output row of this tile only ever stages zeros.  A tile inside one image runs just the K
  // steps of tap rows [qlo, qhi] (the valid rows are contiguous: the row offset is monotonic in
  // q).  ASPP's dilation-12 / -18 convs at 32 x 32 run 6 of 9 taps on most 8-row tiles.  The
  // test is scalar (wave-uniform) and conservative: it never drops a row holding a valid tap.
  int qlo = 0, qhi = ny - 1;
  if (!SMALLC && (flags & 16) && ny > 1) {
    const int mlast = min(p0 + TP, M) - 1;
    const int n0 = p0 / GHW, n1 = mlast / GHW;
    if (n0 == n1) {
      const int ya = (p0 - n0 * GHW) / A.GW * A.sy, yb = (mlast - n1 * GHW) / A.GW * A.sy;
      int lo = ny, hi = -1;
      for (int q = 0; q < ny; ++q) {
        const int off = TG.ty0[tb] + q * dty;
        if (yb + off >= 0 && ya + off <= A.IH - 1) {
          lo = min(lo, q);
          hi = q;
        }
      }
      if (hi >= lo) {
        qlo = lo;
        qhi = hi;
        nK = (qhi - qlo + 1) * nx * CB;
      }
    }
  }
  const int kb0 = qlo * nx * CB;  // first K step (weights are tap-major: K = (q nx + r) CB + cb)
  const unsigned wbase = (unsigned)(((size_t)(c0 + wid * 8 + lrow) * A.k_pad + csrc * E) * sizeof(T));
  // scalar tap walk: the next K step to issue is (tap row tyi, tap column txi, chunk cb) with
  // act_off = ((ty * IW + tx) * ldx + cb * KE) * sizeof(T)
  int w_tyi = qlo, w_txi = 0, w_cb = 0;
  int act_off = (((TG.ty0[tb] + qlo * dty) * A.IW + TG.tx0[tb]) * A.ldx) * (int)sizeof(T);
  const int step_x = dtx * A.ldx * (int)sizeof(T), step_y = dty * A.IW * A.ldx * (int)sizeof(T);
  const int chunk_b = KE * (int)sizeof(T);
#if defined(__HIP_DEVICE_COMPILE__)
  const __amdgpu_buffer_rsrc_t xrsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)TG.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)Wt, (short)0, (int)TG.w_bytes[tb], 0x00020000);
#endif

  auto issue = [&](int ks, uint4* dst) {
    if constexpr (SMALLC) {
      // small Cin (stem): one K step mixes taps, per-lane tap decode
      const int kw_off = ks * KE;
      int k = ks * KE + csrc * E;
      int t = k / A.Cin;
      const int cc = k - t * A.Cin;
      const bool tok = t < S.ntaps;
      int kyy = t / S.kw;
      const int ty = kyy * S.dil - S.pad;
      const int tx = (t - kyy * S.kw) * S.dil - S.pad;
      const void* srcs[GPW];
#pragma unroll
      for (int i = 0; i < GPW; ++i) {
        const int g = wid + NW * i;
        const int r = g * 8 + lrow;
        const void* src;
        if (i < WPW) {
          src = Wt + (size_t)(c0 + r) * A.k_pad + kw_off + csrc * E;
        } else {
          int iy = gpix_y[i] + ty, ix = gpix_x[i] + tx;
          bool ok = tok && gvalid[i] && (unsigned)iy < (unsigned)A.IH && (unsigned)ix < (unsigned)A.IW;
          int iyc = min(max(iy, 0), A.IH - 1), ixc = min(max(ix, 0), A.IW - 1);
          const T* pv = X + (((size_t)gpix_n[i] * A.IH + iyc) * A.IW + ixc) * A.ldx + A.cx0 + cc;
          src = ok ? (const void*)pv : (const void*)&g_zero_page[lane & 7];
        }
        srcs[i] = src;
      }
#if defined(__HIP_DEVICE_COMPILE__)  // device-only builtin: the host pass would silently drop the kernel stubs
#pragma unroll
      for (int i = 0; i < GPW; ++i) {
        const int g = wid + NW * i;
        __builtin_amdgcn_global_load_lds(srcs[i], (__attribute__((address_space(3))) void*)&dst[g * 64], 16, 0, 0);
      }
#endif
    } else {
      // all offsets first (distinct registers), then the DMA issues back to back: hipcc waits
      // vmcnt(0) before it rewrites the address VGPRs of an in-flight LDS-DMA
      unsigned voff[GPW];
#pragma unroll
      for (int i = 0; i < GPW; ++i) {
        const int g = wid + NW * i;
        if (i < WPW) {  // weight group (compile-time)
          voff[i] = wbase + (unsigned)(NW * i * 8) * (unsigned)(A.k_pad * sizeof(T));
        } else {
          const bool ok = (ymask[i] >> w_tyi) & (xmask[i] >> w_txi) & 1u;
          voff[i] = ok ? abase[i] + (unsigned)act_off : 0x80000000u;
        }
      }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
      for (int i = 0; i < GPW; ++i) {
        const int g = wid + NW * i;
        auto* d = (__attribute__((address_space(3))) void*)&dst[g * 64];
        if (i < WPW)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(wrsrc, d, 16, voff[i], (kb0 + ks) * chunk_b, 0, 0);
        else if (ZP_ABL != 3)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, d, 16, voff[i], 0, 0, 0);
      }
#endif
      // advance the scalar tap walk to step ks + 1 (tap-major: chunks fastest)
      act_off += chunk_b;
      if (++w_cb == CB) {
        w_cb = 0;
        act_off += step_x - CB * chunk_b;
        if (++w_txi == nx) {
          w_txi = 0;
          act_off += step_y - nx * step_x;
          ++w_tyi;
        }
      }
    }
  };

  f32x4 acc[WC][WP];
#pragma unroll
  for (int i = 0; i < WC; ++i)
#pragma unroll
    for (int j = 0; j < WP; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // Three-stage ring: while step k computes from buffer k%3, the DMA of steps k+1 (issued one
  // step earlier) and k+2 (issued now) are in flight.  End of step k: counted vmcnt(GPW) (only
  // step k+2's loads may remain outstanding) + raw s_barrier -- never __syncthreads(), whose
  // vmcnt(0) would drain the ring.  Buffer indices are compile-time (loop unrolled by 3) and the
  // three buffers are distinct LDS objects, so hipcc can prove a ds_read never aliases an
  // in-flight global_load_lds and inserts no vmcnt wait in front of it.
  const bool pingpong = NW == 8 && !SMALLC && (flags & 8);
  // per-lane byte offsets of the MFMA fragments inside a stage buffer: row (lane & 15) of the
  // wave's first 16-row tile, 16 B chunk (s * 4 + lane / 16) swizzled by (row & 7) = (lane & 7);
  // tile i / j adds i * 16 rows = i * 2048 B (an immediate of the ds_read)
  unsigned aoff[2], boff[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const unsigned chunk = (unsigned)(((s2 * 4 + (lane >> 4)) ^ (lane & 7)) * 16);
    aoff[s2] = (unsigned)(wc * 16 * WC + (lane & 15)) * 128u + chunk;
    boff[s2] = (unsigned)(TC + wp * 16 * WP + (lane & 15)) * 128u + chunk;
  }
  auto step = [&](auto cur_c, auto nxt_c, int ks) {
    const bool more = ks + (STAGES - 1) < nK;
    // next stage's DMA first (its tap offsets come from scalar loads, whose lgkmcnt wait must
    // not also wait for this step's fragment reads)
    if constexpr (ZP_ABL != 1) {
      if (more) issue(ks + (STAGES - 1), bufp(nxt_c));
    }
    // fragment reads as inline asm: hipcc's waitcnt pass cannot prove across the loop back-edge
    // that they miss the in-flight LDS-DMA buffers and would put a vmcnt(0) in front of them
    const unsigned cb = lds_addr(bufp(cur_c));
    uint4 af[2][WC], bfr[2][WP];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const unsigned pa = cb + aoff[s2], pb = cb + boff[s2];
      static_for<WC>([&](auto i) { af[s2][i] = ds_read16<i * 2048>(pa); });
      static_for<WP>([&](auto j) { bfr[s2][j] = ds_read16<j * 2048>(pb); });
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (pingpong) {
      // end of the read section: fragments in registers (the other group may refill this
      // buffer after the barrier) and every load but the newest step's retired, so the next
      // step's buffer is complete once all waves have passed the barrier
      if (more) vm_wait<LPS * (STAGES - 2)>();
      else vm_wait<0>();
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    if (flags & 4) __builtin_amdgcn_s_setprio(1);
    if constexpr (ZP_ABL != 2) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < WC; ++i)
#pragma unroll
          for (int j = 0; j < WP; ++j) MfmaTraits<T>::mma(acc[i][j], af[s2][i], bfr[s2][j]);
    } else {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < WC; ++i) acc[i][0][0] += __uint_as_float(af[s2][i].x ^ bfr[s2][0].y);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the MFMAs in front of the wait + barrier
    if (flags & 4) __builtin_amdgcn_s_setprio(0);
    if (!pingpong) {
      if (more) vm_wait<LPS * (STAGES - 2)>();
      else vm_wait<0>();
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  issue(0, lds0);
  if (STAGES == 3 && nK > 1) {
    issue(1, lds1);
    vm_wait<LPS * (STAGES - 2)>();
  } else {
    vm_wait<0>();
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  // Ping-pong (flags & 8, 8-wave tiles): every step is a read section (fragments + next DMA)
  // and an MFMA section, each closed by a barrier; waves 4-7 start one barrier late, so on
  // every SIMD (waves w and w+4 share one) one wave's MFMAs overlap the other's LDS reads.
  if (pingpong && wid >= 4) __builtin_amdgcn_s_barrier();
  if constexpr (STAGES == 3) {
    for (int ks = 0; ks < nK; ks += 3) {
      step(I0{}, I2{}, ks);
      if (ks + 1 >= nK) break;
      step(I1{}, I0{}, ks + 1);
      if (ks + 2 >= nK) break;
      step(I2{}, I1{}, ks + 2);
    }
  } else {
    for (int ks = 0; ks < nK; ks += 2) {
      step(I0{}, I1{}, ks);
      if (ks + 1 >= nK) break;
      step(I1{}, I0{}, ks + 1);
    }
  }

  if (pingpong && wid < 4) __builtin_amdgcn_s_barrier();  // same barrier count for both groups

  // (lds0 as the epilogue's LDS scratch: the BN partials of the tile's wave halves meet there)
  conv_epilogue<T, WC, WP, NWP>(A, S, acc, p0, c0, wc, wp, lane, M, GHW, bx, blockIdx.z, gridDim.z, TG.rflag,
                                (float*)lds0);
}

// ------------------------------------------------------------------------------------
// 3x3 stride-1 convolution with activation-strip reuse (bf16).  k_conv stages the activation
// rows of every tap separately: 9 shifted copies of nearly the same rows per channel chunk, and
// the L2 -> LDS stream (not the MFMA) bounds it (profiles/r01_conv_sweep.md ablations).  Here a
// tile is TR full image rows (TP = TR * W = 256 pixels) and, per (tap row, 64-channel chunk), ONE
// strip of TR x (W + 2d) input pixels is staged and read by the three taps of that row at column
// offsets 0, d, 2d: 3 strips + 9 weight tiles per chunk instead of 9 + 9 tiles.
// K steps run (tap row, chunk, tap column), tap column fastest.  Weights: STAGES-deep ring as
// k_conv; strips: 2-deep ring, each strip issued two steps ahead of its first use.  Every wave
// issues the same number of LDS-DMA instructions per step (padding rows load zeros), so the
// counted vmcnt waits stay exact.  Epilogue shared with k_conv.
// ------------------------------------------------------------------------------------
struct strip_geo {
  int W, TR, SW, SR, SPW;       // width, rows per tile, strip width W + 2d, strip rows, DMA instrs / wave
  int ty0, dty, tx0, dtx, pad;  // tap grid (3 x 3) and the halo width pad = max |offset|
  unsigned x_bytes, w_bytes;
};

template <typename T, int WC, int STAGES, int SPW>
__global__ void __launch_bounds__(512) k_conv_strip(const zp_conv_args A, const strip_geo SG, const int flags) {
  constexpr int WP = 4, NWP = 4, NW = 8;
  constexpr int TC = 32 * WC, TP = 256;
  constexpr int WPW = TC / 8 / NW;  // weight DMA instrs per wave per step
  constexpr int SRP = 64 * SPW;     // strip rows incl. padding (8 waves x SPW instrs x 8 rows)
  static_assert(STAGES == 2 || STAGES == 3, "weight ring");
  // weight ring and strip ring; slots are runtime indices (ks % STAGES, group & 1): the loop is
  // unrolled only over the 3 tap columns of a group (compile-time wait counts), which keeps the
  // 256-channel variant inside the register file
  __shared__ uint4 wring[STAGES * TC * 8];
  __shared__ uint4 sring[2 * SRP * 8];
  auto wbuf = [&](int slot) -> uint4* { return wring + slot * (TC * 8); };
  auto sbuf = [&](int slot) -> uint4* { return sring + slot * (SRP * 8); };
  const zp_conv_sub& S = A.sub[0];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid / NWP, wp = wid % NWP;
  const int GHW = A.GH * A.GW;
  const int M = A.N * GHW;
  int bx = blockIdx.x, by = blockIdx.y;
  if (flags & 2) {
    // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs (bid % 8 share one L2).
    // Give each XCD a contiguous run of (pixel tile, cout tile) pairs, cout tiles fastest, so the
    // cout tiles of one pixel tile (same strip) and neighbouring pixel tiles (shared halo rows)
    // are served by the same L2 instead of each fetching its strip from beyond it.  Bijective for
    // any total (cdna_hip_programming.md T1).
    const int total = gridDim.x * gridDim.y;
    const int bid = blockIdx.x + gridDim.x * blockIdx.y;
    const int xcd = bid & 7, pos = bid >> 3, q = total >> 3, r = total & 7;
    const int lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
    bx = lin / gridDim.y;
    by = lin - bx * gridDim.y;
  }
  const int p0 = bx * TP, c0 = by * TC;
  const int n_img = p0 / GHW, y0 = (p0 - n_img * GHW) / SG.W;
  const int CB = A.Cin / 64;
  const int nK = 9 * CB;
  const int lrow = lane >> 3;
  const int csrc = (lane & 7) ^ lrow;  // weight rows: swizzle by (row & 7) = lrow

#if defined(__HIP_DEVICE_COMPILE__)
  const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)A.x, (short)0, (int)SG.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)S.w, (short)0, (int)SG.w_bytes, 0x00020000);
#endif
  // weight rows of this lane: row c0 + (wid + NW*i)*8 + lrow
  const unsigned wbase = (unsigned)(((size_t)(c0 + wid * 8 + lrow) * A.k_pad + csrc * 8) * 2);
  // strip rows of this lane: s = (wid + 8 i) * 8 + lrow -> (tr, c); input (n, y0 + ty + tr, c - pad)
  // per strip instruction: the byte offset of the row's (tr, column) with tr packed into the low
  // 4 bits (offsets are 16-byte multiples; tr < 16), or -1 for padding rows / columns
  int sbase[SPW];
  const int rowb = A.IW * A.ldx * 2;  // bytes per input row
#pragma unroll
  for (int i = 0; i < SPW; ++i) {
    const int srow = (wid + 8 * i) * 8 + lrow;
    const int tr = srow / SG.SW, c = srow - tr * SG.SW;
    const int ix = c - SG.pad;
    const bool ok = srow < SG.SR && (unsigned)ix < (unsigned)A.IW;
    const int sw = (lane & 7) ^ (srow & 7);  // source-side chunk swizzle by the strip row
    sbase[i] = ok ? ((((n_img * A.IH + y0 + tr) * A.IW + ix) * A.ldx + A.cx0 + sw * 8) * 2) | tr : -1;
  }
  auto issue_w = [&](int ks, uint4* dst) {
    const int g = ks / 3, kx = ks - 3 * g, ky = g / CB, cb = g - ky * CB;
    const int koff = ((ky * 3 + kx) * A.Cin + cb * 64) * 2;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int i = 0; i < WPW; ++i) {
      auto* d = (__attribute__((address_space(3))) void*)&dst[(wid + NW * i) * 64];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrsrc, d, 16, wbase + (unsigned)(NW * i * 8) * (unsigned)(A.k_pad * 2),
                                               koff, 0, 0);
    }
#endif
  };
  // strip pieces [I0, I1) of group g (all SPW pieces by default)
  auto issue_s = [&](int g, uint4* dst, auto i0_c, auto i1_c) {
    constexpr int I0 = decltype(i0_c)::value, I1 = decltype(i1_c)::value;
    const int ky = g / CB, cb = g - ky * CB;
    const int ty = SG.ty0 + ky * SG.dty;
    unsigned voff[SPW];
#pragma unroll
    for (int i = I0; i < I1; ++i) {
      const int tr = sbase[i] & 15;
      const bool ok = sbase[i] >= 0 && (unsigned)(y0 + ty + tr) < (unsigned)A.IH;
      voff[i] = ok ? (unsigned)((sbase[i] & ~15) + ty * rowb + cb * 128) : 0x80000000u;
    }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int i = I0; i < I1; ++i) {
      auto* d = (__attribute__((address_space(3))) void*)&dst[(wid + 8 * i) * 64];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, d, 16, voff[i], 0, 0, 0);
    }
#endif
  };
  using C0 = std::integral_constant<int, 0>;
  using CS = std::integral_constant<int, SPW>;

  f32x4 acc[WC][WP];
#pragma unroll
  for (int i = 0; i < WC; ++i)
#pragma unroll
    for (int j = 0; j < WP; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // fragment offsets: A (weights) as in k_conv; B from the strip: pixel q = wp*64 + j*16 + (lane&15)
  // -> strip row tr*SW + x + (tx + pad), chunk swizzled by that row
  unsigned aoff[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
    aoff[s2] = (unsigned)(wc * 16 * WC + (lane & 15)) * 128u + (unsigned)(((s2 * 4 + (lane >> 4)) ^ (lane & 7)) * 16);
  // strip row of fragment j = bsrow0 + jdelta(j): the wave's 64 pixels are one image row when
  // W >= 64, two rows of 32 when W == 32
  int bsrow0;
  {
    const int q0 = wp * 16 * WP;
    const int tr = q0 / SG.W, x0 = q0 - tr * SG.W;
    bsrow0 = tr * SG.SW + x0 + (lane & 15) + SG.pad;
  }
  const int jrow = SG.W == 32 ? SG.SW - 32 : 0;  // extra offset for fragments 2, 3 when W == 32
  const bool pingpong = (flags & 8) != 0;
  // flags & 32 (3-stage ring only): the next group's strip DMA is spread over the three steps of the
  // current group (pieces [0,N0) | [N0,N0+N1) | [N0+N1,SPW)) instead of all SPW pieces in one step,
  // so no read section carries SPW + WPW LDS-DMA issues (~60-180 cycles each) at once
  const bool spread = STAGES == 3 && (flags & 32) != 0;
  constexpr int N0 = (SPW + 2) / 3, N1 = (SPW + 1) / 3;

  // step phase PH = ks % 3 = tap column (compile-time); weight slot ks % STAGES, strip slot g & 1
  auto step = [&](auto ph_c, int ks) {
    constexpr int PH = decltype(ph_c)::value;
    const bool more_w = ks + (STAGES - 1) < nK;
    const bool strip_next = ((PH + 2) % 3 == 0) && ks + 2 < nK;
    const int gnext = ks / 3 + 1;
    const bool has_next = gnext * 3 < nK;  // the next group exists (its strip is staged by this group)
    if (!spread) {
      // (diagnostic builds: ZP_ABL 1 = no DMA in the loop, 3 = weights only, 4 = strips only)
      if (ZP_ABL != 1 && ZP_ABL != 4 && more_w) issue_w(ks + (STAGES - 1), wbuf((ks + STAGES - 1) % STAGES));
      if (ZP_ABL != 1 && ZP_ABL != 3 && strip_next) issue_s((ks + 2) / 3, sbuf(((ks + 2) / 3) & 1), C0{}, CS{});
    } else if constexpr (PH == 0) {
      if (more_w) issue_w(ks + 2, wbuf((ks + 2) % 3));
      if (has_next) issue_s(gnext, sbuf(gnext & 1), C0{}, std::integral_constant<int, N0>{});
    } else if constexpr (PH == 1) {
      if (more_w) issue_w(ks + 2, wbuf((ks + 2) % 3));
      if (has_next) issue_s(gnext, sbuf(gnext & 1), std::integral_constant<int, N0>{},
                            std::integral_constant<int, N0 + N1>{});
    } else {
      if (has_next) issue_s(gnext, sbuf(gnext & 1), std::integral_constant<int, N0 + N1>{}, CS{});
      if (more_w) issue_w(ks + 2, wbuf((ks + 2) % 3));
    }
    const int g = ks / 3;
    const int txo = SG.tx0 + PH * SG.dtx;
    const unsigned cw = lds_addr(wbuf(ks % STAGES));
    const unsigned csb = lds_addr(sbuf(g & 1));
    // loads allowed to stay in flight at the end of this step: the ones issued for later steps
    constexpr int OUT_S2 = ((PH + 2) % 3 == 0) ? SPW : 0;  // strip issued this step (needed at ks + 2)
    constexpr int OUT = (STAGES == 3 ? WPW : 0) + OUT_S2;
    // (a step whose strip slot would have been refilled past the end issued no strip)
    auto wait_out = [&]() {
      if (spread) {
        // loads allowed in flight: this step's weights (for ks + 2) and the pieces of the next
        // strip issued after the weights of step ks + 1, except in the group's last step
        if constexpr (PH == 0) {
          if (more_w && has_next) vm_wait<WPW + N0>();
          else if (more_w) vm_wait<WPW>();
          else if (has_next) vm_wait<N0>();
          else vm_wait<0>();
        } else if constexpr (PH == 1) {
          if (more_w && has_next) vm_wait<WPW + N0 + N1>();
          else if (more_w) vm_wait<WPW>();
          else if (has_next) vm_wait<N0 + N1>();
          else vm_wait<0>();
        } else {
          if (more_w) vm_wait<WPW>();
          else vm_wait<0>();
        }
        return;
      }
      if (strip_next) vm_wait<OUT>();
      else if (more_w) vm_wait<OUT - OUT_S2>();
      else vm_wait<0>();
    };
    uint4 af[2][WC], bfr[2][WP];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const unsigned pa = cw + aoff[s2];
      static_for<WC>([&](auto i) { af[s2][i] = ds_read16<i * 2048>(pa); });
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        const int sr = bsrow0 + txo + 16 * j + (j >= 2 ? jrow : 0);
        const unsigned pb = csb + (unsigned)sr * 128u + (unsigned)((((s2 * 4 + (lane >> 4)) ^ (sr & 7))) * 16);
        bfr[s2][j] = ds_read16<0>(pb);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (pingpong) {
      wait_out();
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_setprio(1);
    if constexpr (ZP_ABL != 2) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < WC; ++i)
#pragma unroll
          for (int j = 0; j < WP; ++j) MfmaTraits<T>::mma(acc[i][j], af[s2][i], bfr[s2][j]);
    } else {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < WC; ++i)
#pragma unroll
          for (int j = 0; j < WP; ++j) acc[i][j][0] += __uint_as_float(af[s2][i].x ^ bfr[s2][j].y);
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
    if (!pingpong) wait_out();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // prologue: strip of group 0, weights of steps 0 .. STAGES-2; the strip of group 1 is issued
  // at step 1 (two steps ahead of step 3)
  issue_s(0, sbuf(0), C0{}, CS{});
  issue_w(0, wbuf(0));
  if (STAGES == 3) issue_w(1, wbuf(1));
  if (STAGES == 3) vm_wait<WPW>();  // strip(0) and weights(0) landed; weights(1) may be in flight
  else vm_wait<0>();
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if (pingpong && wid >= 4) __builtin_amdgcn_s_barrier();
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  using P2 = std::integral_constant<int, 2>;
  for (int ks = 0; ks < nK; ks += 3) {  // nK = 9 CB: whole groups
    step(P0{}, ks);
    step(P1{}, ks + 1);
    step(P2{}, ks + 2);
  }
  if (pingpong && wid < 4) __builtin_amdgcn_s_barrier();
  conv_epilogue<T, WC, WP, NWP>(A, S, acc, p0, c0, wc, wp, lane, M, GHW, bx, blockIdx.z, gridDim.z);
}

// ------------------------------------------------------------------------------------
// k_conv_strip2: k_conv_strip's algorithm (same staging, same K order, bit-identical results)
// with a lean main loop.  Profiling k_conv_strip (256 -> 256 at 128 x 128, bs 32) showed the
// read section of every step -- not the MFMAs, not L2 / HBM -- as the critical path: the MFMA-free
// ablation ran exactly as long as the full kernel, and each step issued ~65 SALU (runtime
// divisions for the tap / chunk / slot of every DMA, a branch tree of counted waits) and ~70 VALU
// (per-step fragment and DMA address arithmetic, an SGPR-spilled buffer descriptor rebuilt with
// v_readlane) besides its 16 ds_reads and 2-7 LDS-DMAs.  Here:
//   * the loop is unrolled by group parity x tap column, so every LDS address is a per-lane base
//     register + an immediate (weight slot = tap column, strip slot = group parity) and every wait
//     count is a constant; the steady-state groups (all of whose steps prefetch) are separated
//     from the last group, so the loop body has no prefetch conditions;
//   * DMA offsets are per-lane registers computed once (weights: row offsets; strips: one per tap
//     row and piece) plus a scalar offset advanced by additions (no divisions);
//   * one __shared__ array (weights ring, then strip ring).
// ------------------------------------------------------------------------------------
template <typename T, int WC, int WP, int NWP>
__device__ __forceinline__ void head_epilogue16(const zp_conv_args& A, const zp_conv_sub& S, const zp_head_args& H,
                                                f32x4 (&acc)[WC][WP], int p0, int c0, int by, int wc, int wp,
                                                int lane, int M, uint4* lds);

// HEAD (zp_conv2d_head, 16-bit eval): the conv output is not stored; it feeds the fused 1x1 head's
// partial sums over this tile's channels (head_epilogue16)
template <typename T, int WC, int SPW, int DM, bool HEAD = false, bool BNR = false>
__global__ void __launch_bounds__(512) k_conv_strip2(const zp_conv_args A, const strip_geo SG, const int flags,
                                                     const zp_head_args H) {
  // DM: where the next group's strip DMA is issued.  0: the read section of tap column 1; 1: spread
  // over the read sections of the group's three steps; 2: between the MFMAs of tap column 0 (the
  // read sections then carry only the weight pieces: the LDS-DMA issue cost, ~60 cycles per piece
  // among bare MFMAs but 100-185 inside a read section already holding 16 ds_read_b128, leaves the
  // critical path of the ping-pong schedule, and the strip is issued one phase earlier)
  constexpr bool SPREAD = DM == 1, MSEC = DM == 2;
  constexpr int WP = 4, NWP = 4, NW = 8;
  constexpr int TC = 32 * WC, TP = 256;
  constexpr int WPW = TC / 8 / NW;  // weight DMA instrs per wave per step
  constexpr int SRP = 64 * SPW;     // strip rows incl. padding
  constexpr int WSLOT = TC * 128;   // bytes per weight slot (3 slots)
  constexpr int SSLOT = SRP * 128;  // bytes per strip slot (2 slots)
  static_assert(SSLOT < 65536 && 2 * WSLOT + 2048 * (WC - 1) < 65536, "ds_read immediate range");
  __shared__ uint4 lds[(3 * TC + 2 * SRP) * 8];
  const zp_conv_sub& S = A.sub[0];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid / NWP, wp = wid % NWP;
  const int GHW = A.GH * A.GW;
  const int M = A.N * GHW;
  int bx = blockIdx.x, by = blockIdx.y;
  if (flags & 2) {  // XCD-aware order, as k_conv_strip
    const int total = gridDim.x * gridDim.y;
    const int bid = blockIdx.x + gridDim.x * blockIdx.y;
    const int xcd = bid & 7, pos = bid >> 3, q = total >> 3, r = total & 7;
    const int lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
    bx = lin / gridDim.y;
    by = lin - bx * gridDim.y;
  }
  const int p0 = bx * TP, c0 = by * TC;
  const int n_img = p0 / GHW, y0 = (p0 - n_img * GHW) / SG.W;
  const int CB = A.Cin / 64;
  const int lrow = lane >> 3;
  const int csrc = (lane & 7) ^ lrow;

#if defined(__HIP_DEVICE_COMPILE__)
  const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)A.x, (short)0, (int)SG.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)S.w, (short)0, (int)SG.w_bytes, 0x00020000);
#endif
  // weight DMA: per-lane row offsets (piece i = rows (wid + NW i) * 8 + lrow); the K offset of a
  // step is scalar: koff = (ky * 3 + kx) * Cin * 2 + cb * 128
  unsigned wv[WPW];
#pragma unroll
  for (int i = 0; i < WPW; ++i)
    wv[i] = (unsigned)(((size_t)(c0 + (wid + NW * i) * 8 + lrow) * A.k_pad + csrc * 8) * 2);
  const int cin2 = A.Cin * 2;
  // strip DMA: per piece and tap row ky, the lane's source byte offset (chunk 0) or an offset past
  // the buffer end (zeros) for padding rows / columns; the chunk's cb * 128 goes in the scalar offset
  const int rowb = A.IW * A.ldx * 2;
  // pk[i]: the piece's 16-byte-aligned source offset for tap row 0 with a 3-bit "row inside the
  // image" mask per tap row in the low bits; svn[i]: the offsets for the next strip's tap row,
  // recomputed (a few VALU per piece) only when that tap row changes, i.e. 3 times per workgroup
  unsigned pk[SPW], svn[SPW];
#pragma unroll
  for (int i = 0; i < SPW; ++i) {
    const int srow = (wid + 8 * i) * 8 + lrow;
    const int tr = srow / SG.SW, c = srow - tr * SG.SW;
    const int ix = c - SG.pad;
    const bool ok = srow < SG.SR && (unsigned)ix < (unsigned)A.IW;
    const int sw = (lane & 7) ^ (srow & 7);
    const int base = (((n_img * A.IH + y0 + tr) * A.IW + ix) * A.ldx + A.cx0 + sw * 8) * 2 + SG.ty0 * rowb;
    unsigned m = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k)
      m |= (unsigned)(ok && (unsigned)(y0 + SG.ty0 + k * SG.dty + tr) < (unsigned)A.IH) << k;
    pk[i] = (unsigned)base | m;
  }
  const int dtyb = SG.dty * rowb;
  auto set_svn = [&](int k) {
#pragma unroll
    for (int i = 0; i < SPW; ++i)
      svn[i] = (pk[i] >> k) & 1u ? (pk[i] & ~15u) + (unsigned)(k * dtyb) : 0x80000000u;
  };
  const unsigned lds0 = lds_addr(lds);
  // fragment bases: A (weights) row wc*16*WC + (lane & 15), swizzled chunk; + slot * WSLOT + i * 2048
  unsigned aoff[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
    aoff[s2] = lds0 + (unsigned)(wc * 16 * WC + (lane & 15)) * 128u + (unsigned)(((s2 * 4 + (lane >> 4)) ^ (lane & 7)) * 16);
  // B (strip) per tap column PH, half s2, pixel fragment j; + parity * SSLOT
  unsigned bo[3][2][WP];
  {
    const int q0 = wp * 16 * WP;
    const int tr = q0 / SG.W, x0 = q0 - tr * SG.W;
    const int bsrow0 = tr * SG.SW + x0 + (lane & 15) + SG.pad;
    const int jrow = SG.W == 32 ? SG.SW - 32 : 0;
#pragma unroll
    for (int ph = 0; ph < 3; ++ph)
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        const int sr = bsrow0 + SG.tx0 + ph * SG.dtx + 16 * j + (j >= 2 ? jrow : 0);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
          bo[ph][s2][j] = lds0 + 3u * WSLOT + (unsigned)sr * 128u + (unsigned)(((s2 * 4 + (lane >> 4)) ^ (sr & 7)) * 16);
      }
  }
  const bool pingpong = (flags & 8) != 0;

  auto issue_w = [&](int slot, int koff) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int i = 0; i < WPW; ++i) {
      auto* d = (__attribute__((address_space(3))) void*)&lds[(slot * TC + (wid + NW * i) * 8) * 8];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrsrc, d, 16, wv[i], koff, 0, 0);
    }
#endif
  };
  constexpr int N0 = (SPW + 2) / 3, N1 = (SPW + 1) / 3;  // SPREAD: pieces per step (PH 0 / 1 / 2 = rest)
  auto issue_s = [&](int slot, int cb, auto i0_c, auto i1_c) {  // pieces [I0, I1) of the strip svn holds
    constexpr int I0 = decltype(i0_c)::value, I1 = decltype(i1_c)::value;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int i = I0; i < I1; ++i) {
      auto* d = (__attribute__((address_space(3))) void*)&lds[(3 * TC + slot * SRP + (wid + 8 * i) * 8) * 8];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, d, 16, svn[i], cb * 128, 0, 0);
    }
#endif
  };

  f32x4 acc[WC][WP];
#pragma unroll
  for (int i = 0; i < WC; ++i)
#pragma unroll
    for (int j = 0; j < WP; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // one K step: tap column PH of a group with strip parity GP.  Prefetch (issued first): PH 0 the
  // weights of (this group, column 2) -> slot 2; PH 1 the weights of (next group, column 0) -> slot 0
  // and the next group's strip -> slot GP ^ 1; PH 2 the weights of (next group, column 1) -> slot 1.
  // Waits: what the next step reads must have landed.
  auto step = [&](auto gp_c, auto ph_c, auto steady_c, int koff_cur, int koff_next, int ncb) {
    constexpr int GP = decltype(gp_c)::value, PH = decltype(ph_c)::value;
    constexpr bool STEADY = decltype(steady_c)::value;
    using Z = std::integral_constant<int, 0>;
    using K0 = std::integral_constant<int, N0>;
    using K1 = std::integral_constant<int, N0 + N1>;
    using KS = std::integral_constant<int, SPW>;
    if constexpr (ZP_ABL == 1) {  // diagnostic build: no DMA in the loop
    } else if constexpr (!SPREAD) {
      if constexpr (PH == 0) {
        issue_w(2, koff_cur + 2 * cin2);
      } else if constexpr (STEADY && PH == 1) {
        issue_w(0, koff_next);
        if constexpr (!MSEC) issue_s(GP ^ 1, ncb, Z{}, KS{});
      } else if constexpr (STEADY && PH == 2) {
        issue_w(1, koff_next + cin2);
      }
    } else {
      // the next strip in three parts; issue order weights-then-strip (PH 0, 1), strip-then-weights
      // (PH 2) so each counted wait below retires exactly what the next step reads
      if constexpr (PH == 0) {
        issue_w(2, koff_cur + 2 * cin2);
        if constexpr (STEADY) issue_s(GP ^ 1, ncb, Z{}, K0{});
      } else if constexpr (STEADY && PH == 1) {
        issue_w(0, koff_next);
        issue_s(GP ^ 1, ncb, K0{}, K1{});
      } else if constexpr (STEADY && PH == 2) {
        issue_s(GP ^ 1, ncb, K1{}, KS{});
        issue_w(1, koff_next + cin2);
      }
    }
    uint4 af[2][WC], bfr[2][WP];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      static_for<WC>([&](auto i) { af[s2][i] = ds_read16<PH * WSLOT + i * 2048>(aoff[s2]); });
      static_for<WP>([&](auto j) { bfr[s2][j] = ds_read16<GP * SSLOT>(bo[PH][s2][j]); });
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    auto wait_out = [&]() {
      // (MSEC without ping-pong: the wait follows the MFMA section, i.e. this step's strip issue)
      if constexpr (MSEC && PH == 0 && STEADY) {
        if (pingpong) vm_wait<WPW>();
        else vm_wait<WPW + SPW>();
      } else if constexpr (PH == 0) vm_wait<WPW + (SPREAD && STEADY ? N0 : 0)>();
      else if constexpr (STEADY && PH == 1) vm_wait<WPW + (SPREAD ? N0 + N1 : SPW)>();
      else if constexpr (STEADY && PH == 2) vm_wait<WPW>();
      else vm_wait<0>();
    };
    if (pingpong) {
      wait_out();
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_setprio(1);
    if constexpr (ZP_ABL != 2) {
      // MSEC, tap column 0 of a steady group: strip piece k after MFMA SP (k + 1) - 1
      constexpr int NM = 2 * WC * WP, SP = NM / (SPW + 1);
      static_for<NM>([&](auto t_c) {
        constexpr int t = decltype(t_c)::value;
        constexpr int s2 = t / (WC * WP), i = (t / WP) % WC, j = t % WP;
        MfmaTraits<T>::mma(acc[i][j], af[s2][i], bfr[s2][j]);
        if constexpr (MSEC && PH == 0 && STEADY && ZP_ABL != 1 && (t + 1) % SP == 0 && (t + 1) / SP <= SPW) {
          constexpr int k = (t + 1) / SP - 1;
          __builtin_amdgcn_sched_barrier(0);  // pin the piece between MFMAs t and t + 1
          issue_s(GP ^ 1, ncb, std::integral_constant<int, k>{}, std::integral_constant<int, k + 1>{});
          __builtin_amdgcn_sched_barrier(0);
        }
      });
    } else {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < WC; ++i)
#pragma unroll
          for (int j = 0; j < WP; ++j) acc[i][j][0] += __uint_as_float(af[s2][i].x ^ bfr[s2][j].y);
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
    if (!pingpong) wait_out();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  using P2 = std::integral_constant<int, 2>;
  using G0 = std::integral_constant<int, 0>;
  using G1 = std::integral_constant<int, 1>;
  using ST = std::integral_constant<bool, true>;
  using TL = std::integral_constant<bool, false>;
  auto group = [&](auto gp_c, auto steady_c, int koff_cur, int koff_next, int ncb) {
    step(gp_c, P0{}, steady_c, koff_cur, koff_next, ncb);
    step(gp_c, P1{}, steady_c, koff_cur, koff_next, ncb);
    step(gp_c, P2{}, steady_c, koff_cur, koff_next, ncb);
  };

  // groups (ky, cb), cb fastest; koff of (ky, cb, kx = 0) = ky * 3 * Cin * 2 + cb * 128
  int ky = 0, cb = 0;
  auto koff_of = [&](int a, int b) { return a * 3 * cin2 + b * 128; };
  // the next group (its strip is staged during the current one); svn follows its tap row
  int nky = 0, ncb = 0;
  auto advance_next = [&]() {
    if (++ncb == CB) {
      ncb = 0;
      ++nky;
      if (nky < 3) set_svn(nky);
    }
  };
  // prologue: strip of group 0, weights of steps 0 and 1
  set_svn(0);
  issue_s(0, 0, std::integral_constant<int, 0>{}, std::integral_constant<int, SPW>{});
  issue_w(0, 0);
  issue_w(1, cin2);
  vm_wait<WPW>();
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if (pingpong && wid >= 4) __builtin_amdgcn_s_barrier();
  const int ng = 3 * CB;
  advance_next();
  int g = 0;
  for (; g + 2 <= ng - 1; g += 2) {
    group(G0{}, ST{}, koff_of(ky, cb), koff_of(nky, ncb), ncb);
    ky = nky;
    cb = ncb;
    advance_next();
    group(G1{}, ST{}, koff_of(ky, cb), koff_of(nky, ncb), ncb);
    ky = nky;
    cb = ncb;
    advance_next();
  }
  if (g < ng - 1) {
    group(G0{}, ST{}, koff_of(ky, cb), koff_of(nky, ncb), ncb);
    ky = nky;
    cb = ncb;
    ++g;
  }
  if (g & 1) group(G1{}, TL{}, koff_of(ky, cb), 0, 0);
  else group(G0{}, TL{}, koff_of(ky, cb), 0, 0);
  if (pingpong && wid < 4) __builtin_amdgcn_s_barrier();
  if constexpr (ZP_ABL == 5) {  // diagnostic build: no epilogue (one store only if a sum is exactly 1)
    float sm = 0.f;
#pragma unroll
    for (int i = 0; i < WC; ++i)
#pragma unroll
      for (int j = 0; j < WP; ++j) sm += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (sm == 1.f) ((float*)S.y)[tid] = sm;
  } else if constexpr (HEAD) {
    head_epilogue16<T, WC, WP, NWP>(A, S, H, acc, p0, c0, by, wc, wp, lane, M, lds);
  } else {
    conv_epilogue<T, WC, WP, NWP, BNR>(A, S, acc, p0, c0, wc, wp, lane, M, GHW, bx, blockIdx.z, gridDim.z, nullptr,
                                       (float*)lds);
  }
}

// The fused head's epilogue for the 16-bit strip tile (ZP_BF16 / ZP_F16 eval; zp_conv2d_head): the
// tile's TC = 32 WC output channels of 256 pixels, after BN scale / shift, residual and ReLU and
// rounded to the storage type exactly as the unfused path stores them, are the B operand of the head's
// 16 x 16 x 32 MFMAs: the paired lane layout (v_permlane16_swap of cout blocks i, i + 1: a lane holds
// 8 consecutive channels of one pixel) is a B fragment when lane group g is read as k slot g, so the
// head weights are read with the same channel permutation (k slot g <-> channel (g & 1) * 16 +
// (g >> 1) * 8 of the 32-channel slice).  The first cout tile also adds x2 (x_128) at k = Cout + c.
// The two wave rows (wc) of a pixel quarter meet in LDS; the tile's partial sums (rows r < hcout,
// f32) go to H.ws[by][r][p]; k_head_combine16 adds the cout tiles in order, plus the bias.
template <typename T, int WC, int WP, int NWP>
__device__ __forceinline__ void head_epilogue16(const zp_conv_args& A, const zp_conv_sub& S, const zp_head_args& H,
                                                f32x4 (&acc)[WC][WP], int p0, int c0, int by, int wc, int wp,
                                                int lane, int M, uint4* lds) {
  static_assert(WC % 2 == 0, "paired cout blocks");
  using MT = MfmaTraits<T>;
  const int g = lane >> 4, lr = lane & 15;
  const int GHW = S.OH * S.OW;
  f32x4 hacc[2][WP];
#pragma unroll
  for (int hb = 0; hb < 2; ++hb)
#pragma unroll
    for (int j = 0; j < WP; ++j) hacc[hb][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const T* W = (const T*)H.w;
  // head weight fragment: rows hb * 16 + lr, the 8 k of lane group g (k = kbase + perm)
  auto wfrag = [&](int hb, int k) -> uint4 { return *(const uint4*)(W + (size_t)(hb * 16 + lr) * H.k_pad + k); };
#pragma unroll
  for (int i = 0; i < WC; i += 2) {
    const int cs = c0 + wc * 16 * WC + (i + (g & 1)) * 16 + (g >> 1) * 8;  // this lane's 8 channels
    float sc[8], sh[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      sc[r] = S.scale ? S.scale[cs + r] : 1.f;
      sh[r] = S.shift ? S.shift[cs + r] : 0.f;
    }
    const uint4 w0 = wfrag(0, cs), w1 = wfrag(1, cs);
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
      const int p = p0 + wp * 16 * WP + j * 16 + lr;
      const bool ok = p < M;
      const size_t pix = ok ? (size_t)p : 0;
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = v[r] * sc[r] + sh[r];
      if (A.res) {
        const uint4 rv = *(const uint4*)((const unsigned short*)A.res + pix * A.ldr + A.cr0 + cs);
        const uint32_t rw[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[2 * r] += H16<T>::from(rw[r] & 0xffffu);
          v[2 * r + 1] += H16<T>::from(rw[r] >> 16);
        }
      }
      if (A.relu) {
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      uint32_t o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = ok ? (H16<T>::to(v[2 * r]) | (H16<T>::to(v[2 * r + 1]) << 16)) : 0u;
      const uint4 xb = make_uint4(o[0], o[1], o[2], o[3]);
      MT::mma(hacc[0][j], w0, xb);
      MT::mma(hacc[1][j], w1, xb);
    }
  }
  if (by == 0 && wc == 0) {  // x2 (the skip features, NHWC on the output grid), weights at k = Cout + c
    for (int q = 0; q < H.C2 / 32; ++q) {
      const uint4 w0 = wfrag(0, A.Cout + q * 32 + g * 8), w1 = wfrag(1, A.Cout + q * 32 + g * 8);
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        const int p = p0 + wp * 16 * WP + j * 16 + lr;
        const uint4 xq = p < M ? *(const uint4*)((const unsigned short*)H.x2 + (size_t)p * H.ldx2 + H.cx20 + q * 32 + g * 8)
                               : make_uint4(0u, 0u, 0u, 0u);
        MT::mma(hacc[0][j], w0, xq);
        MT::mma(hacc[1][j], w1, xq);
      }
    }
  }
  // the wave rows' sums meet in LDS (free: every wave passed the main loop's last barrier)
  f32x4* red = (f32x4*)lds;  // [wp][hb][j][lane]
  if (wc != 0) {
#pragma unroll
    for (int hb = 0; hb < 2; ++hb)
#pragma unroll
      for (int j = 0; j < WP; ++j) red[((wp * 2 + hb) * WP + j) * 64 + lane] = hacc[hb][j];
  }
  __syncthreads();
  if (wc != 0) return;
#pragma unroll
  for (int hb = 0; hb < 2; ++hb)
#pragma unroll
    for (int j = 0; j < WP; ++j) {
      const f32x4 o = red[((wp * 2 + hb) * WP + j) * 64 + lane];
      const int p = p0 + wp * 16 * WP + j * 16 + lr;
      if (p >= M) continue;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int r = hb * 16 + g * 4 + qq;
        if (r < H.cout) H.ws[((size_t)by * 32 + r) * M + p] = hacc[hb][j][qq] + o[qq];
      }
    }
  (void)GHW;
}

// the fused 16-bit head's second launch: mask / code = ws[0] + ws[1] (the two cout tiles, in that
// order) + bias, f32 NCHW (one thread per output pixel)
__global__ void k_head_combine16(const float* __restrict__ ws, int M, int GHW, int hcout, const float* __restrict__ bias,
                                 float* __restrict__ mask, float* __restrict__ code) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= M) return;
  const int n = p / GHW, sp = p - n * GHW;
  for (int r = 0; r < hcout; ++r) {
    const float v = (ws[(size_t)r * M + p] + ws[((size_t)32 + r) * M + p]) + (bias ? bias[r] : 0.f);
    if (r == 0) mask[(size_t)n * GHW + sp] = v;
    else code[((size_t)n * (hcout - 1) + (r - 1)) * GHW + sp] = v;
  }
}

// ------------------------------------------------------------------------------------
// k_conv_quad: the four sub-pixel phases of a stride-2 transposed structure in ONE tile.
// ConvTranspose2d(3, s2, p1, op1) (model/aspp.py:60-80) -- and the data gradient of a 3x3 stride-2
// conv, which geometry.py plans the same way -- is four stride-1 sub-problems over the same input
// grid, output phase (py, px) at (2 gy + py, 2 gx + px), with 1 / 2 / 2 / 4 taps whose input offsets
// (dy, dx) all lie in {0, 1}^2.  k_conv runs them as four independent tiles (blockIdx.z) that each
// stage their own shifted copies of the input: 9 activation tiles per 64-channel chunk for the 9
// (phase, tap) pairs, and the four phases of one pixel tile land on different XCDs, so the re-staging
// goes to HBM (r01 PMC: 761 MB read per up2 launch against 85 MB algorithmic).
// Here a workgroup owns 256 grid points (TR = 256 / W full rows) x 64 output channels x ALL FOUR
// phases: per chunk it stages ONE strip of (TR + 1) x W input pixels (the +1 row / column of the
// (dy, dx) = 1 taps; column W is outside the image, so the lane that would read it gets zeros by a
// register select instead of a staged padding column) and the 9 weight taps, and every (phase, tap)
// reads its operand from the strip at offset dy * W + dx.
// Per chunk, 5 K steps grouped by input shift (B fragments read once per step):
//   step 0: shift 00, phases 0, 1   step 1: shift 00, phases 2, 3   step 2: shift 01, phases 1, 3
//   step 3: shift 10, phases 2, 3   step 4: shift 11, phase 3
// Weights: one 8 KB LDS slot per (phase, tap) (9 slots, 72 KB); at the start of step s the slots of
// step s - 1 are refilled with the next chunk's taps (4 steps of lead).  Strips: 2-slot ring, the
// next chunk's strip issued at step 0.  8 waves = 2 (32 channels) x 4 (64 grid points), each holding
// 4 phases x 2 x 4 MFMA tiles (128 accumulator registers).  Schedule (ping-pong wave groups, setprio,
// counted vmcnt waits, XCD-aware order) as k_conv_strip2.  Epilogue: k_conv's, once per phase.
// ------------------------------------------------------------------------------------
struct quad_geo {
  unsigned x_bytes, w_bytes;
  int koff[9];  // byte offset of the slot's tap in a packed weight row: local tap index * Cin * 2
};
// slot -> phase (sub-problem) and input shift (host table: quad_plan)
__host__ __device__ constexpr int quad_phase(int slot) { return slot == 0 ? 0 : slot == 1 || slot == 4 ? 1 : slot == 2 || slot == 6 ? 2 : 3; }

template <typename T, int W, bool MS>
__global__ void __launch_bounds__(512) k_conv_quad(const zp_conv_args A, const quad_geo QG, const int flags) {
  // MS (flags & 256, as k_conv_strip2's DM 2): the next chunk's strip DMA is issued between the MFMAs
  // of step 0 instead of in its read section
  constexpr int WC = 2, WP = 4, NWP = 4;
  constexpr int TC = 64, TP = 256, TR = TP / W;
  constexpr int SROWS = (TR + 1) * W;    // strip rows: TR + 1 image rows of W pixels
  constexpr int SPW = (SROWS + 63) / 64;  // strip DMA instructions per wave (8 waves x 8 rows each)
  constexpr int SRP = 64 * SPW;
  constexpr int WSLOT = TC * 128;         // bytes per weight slot (one tap)
  constexpr int SBASE = 9 * WSLOT;        // strip ring after the 9 weight slots
  constexpr int SSLOT = SRP * 128;
  static_assert(SPW == 5, "strip of 5 DMA instructions per wave (W 32 / 64)");
  static_assert(7 * WSLOT + 2048 < 65536 && SSLOT + W * 128 < 65536, "ds_read immediate range");
  __shared__ uint4 lds[(9 * TC + 2 * SRP) * 8];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid / NWP, wp = wid % NWP;
  const int GHW = A.GH * A.GW;
  const int M = A.N * GHW;
  int bx = blockIdx.x, by = blockIdx.y;
  if (flags & 2) {  // XCD-aware order: the cout tiles of one pixel tile (same strip) on one L2
    const int total = gridDim.x * gridDim.y;
    const int bid = blockIdx.x + gridDim.x * blockIdx.y;
    const int xcd = bid & 7, pos = bid >> 3, q = total >> 3, r = total & 7;
    const int lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
    bx = lin / gridDim.y;
    by = lin - bx * gridDim.y;
  }
  const int p0 = bx * TP, c0 = by * TC;
  const int n_img = p0 / GHW, y0 = (p0 - n_img * GHW) / W;
  const int CB = A.Cin / 64;
  const int lrow = lane >> 3;

#if defined(__HIP_DEVICE_COMPILE__)
  const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)A.x, (short)0, (int)QG.x_bytes, 0x00020000);
  __amdgpu_buffer_rsrc_t wrsrc[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
    wrsrc[s] = __builtin_amdgcn_make_buffer_rsrc((void*)A.sub[s].w, (short)0, (int)QG.w_bytes, 0x00020000);
#endif
  // weight DMA: row c0 + wid * 8 + lrow of the slot, source chunk swizzled by the row (lrow)
  const unsigned wv = (unsigned)(((size_t)(c0 + wid * 8 + lrow) * A.k_pad + ((lane & 7) ^ lrow) * 8) * 2);
  // strip DMA: piece i = strip rows (wid + 8 i) * 8 + lrow = (tr, x); rows past the strip or below the
  // image read past the buffer end (zeros)
  unsigned sv[SPW];
#pragma unroll
  for (int i = 0; i < SPW; ++i) {
    const int srow = (wid + 8 * i) * 8 + lrow;
    const int tr = srow / W, x = srow - tr * W;
    const bool ok = srow < SROWS && y0 + tr < A.IH;
    const int sw = (lane & 7) ^ (srow & 7);
    sv[i] = ok ? (unsigned)((((n_img * A.IH + y0 + tr) * A.IW + x) * A.ldx + A.cx0 + sw * 8) * 2) : 0x80000000u;
  }
  const unsigned lds0 = lds_addr(lds);
  unsigned aoff[2], aoff8[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    aoff[s2] = lds0 + (unsigned)(wc * 16 * WC + (lane & 15)) * 128u + (unsigned)(((s2 * 4 + (lane >> 4)) ^ (lane & 7)) * 16);
    aoff8[s2] = aoff[s2] + 8u * WSLOT;
  }
  // B fragment j of the wave: grid point q = wp * 64 + 16 j + (lane & 15) -> strip row tr * W + x + dx
  // (+ dy * W through the immediate offset, which keeps the row's swizzle); the lane at x = W - 1
  // reads garbage for dx = 1 and is zeroed after the read
  unsigned bo[2][2][WP];
#pragma unroll
  for (int dx = 0; dx < 2; ++dx)
#pragma unroll
    for (int j = 0; j < WP; ++j) {
      const int q = wp * 64 + 16 * j + (lane & 15);
      const int sr = (q / W) * W + (q % W) + dx;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        bo[dx][s2][j] = lds0 + (unsigned)SBASE + (unsigned)sr * 128u + (unsigned)((((s2 * 4 + (lane >> 4)) ^ (sr & 7))) * 16);
    }
  const bool edge = (lane & 15) == 15;  // x = W - 1 in fragments j = 3 (W 64) / j odd (W 32)
  // the strip slot of the current chunk alternates: bo moves between the two slots once per chunk
  // (a runtime parity keeps ONE loop body and one tail, so the 128 accumulators stay in place)
  int sdelta = SSLOT;
  auto flip = [&]() {
#pragma unroll
    for (int dx = 0; dx < 2; ++dx)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < WP; ++j) bo[dx][s2][j] += (unsigned)sdelta;
    sdelta = -sdelta;
  };

  auto issue_w = [&](int slot, int cb) {
#if defined(__HIP_DEVICE_COMPILE__)
    auto* d = (__attribute__((address_space(3))) void*)&lds[(slot * TC + wid * 8) * 8];
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wrsrc[quad_phase(slot)], d, 16, wv, QG.koff[slot] + cb * 128, 0, 0);
#endif
  };
  auto issue_s = [&](int gslot, int cb) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int i = 0; i < SPW; ++i) {
      auto* d = (__attribute__((address_space(3))) void*)&lds[(9 * TC + gslot * SRP + (wid + 8 * i) * 8) * 8];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, d, 16, sv[i], cb * 128, 0, 0);
    }
#endif
  };

  f32x4 acc[4][WC][WP];
#pragma unroll
  for (int ph = 0; ph < 4; ++ph)
#pragma unroll
    for (int i = 0; i < WC; ++i)
#pragma unroll
      for (int j = 0; j < WP; ++j) acc[ph][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // one K step S of chunk cb (strip slot gp); STEADY: a next chunk exists (prefetches issued)
  auto step = [&](auto s_c, auto steady_c, int cb, int gp) {
    constexpr int S = decltype(s_c)::value;
    constexpr bool STEADY = decltype(steady_c)::value;
    constexpr int NT = S == 4 ? 1 : 2;
    constexpr int DY = (S == 3 || S == 4) ? 1 : 0, DX = (S == 2 || S == 4) ? 1 : 0;
    if constexpr (ZP_ABL == 1) {  // diagnostic build: no DMA in the loop
    } else if constexpr (S == 0) {
      issue_w(8, cb);
      if constexpr (STEADY && !MS) issue_s(gp ^ 1, cb + 1);
    } else if constexpr (STEADY) {
      issue_w(2 * (S - 1), cb + 1);
      issue_w(2 * (S - 1) + 1, cb + 1);
    }
    uint4 af[NT][2][WC], bfr[2][WP];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      static_for<NT>([&](auto t) {
        constexpr int SL = 2 * S + decltype(t)::value;
        static_for<WC>([&](auto i) {
          if constexpr (SL < 8) af[t][s2][i] = ds_read16<SL * WSLOT + i * 2048>(aoff[s2]);
          else af[t][s2][i] = ds_read16<i * 2048>(aoff8[s2]);
        });
      });
      static_for<WP>([&](auto j) { bfr[s2][j] = ds_read16<DY * W * 128>(bo[DX][s2][j]); });
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (DX == 1) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < WP; ++j)
          if (W == 32 ? (j & 1) : (j == 3)) {
            bfr[s2][j].x = edge ? 0u : bfr[s2][j].x;
            bfr[s2][j].y = edge ? 0u : bfr[s2][j].y;
            bfr[s2][j].z = edge ? 0u : bfr[s2][j].z;
            bfr[s2][j].w = edge ? 0u : bfr[s2][j].w;
          }
    }
    // loads allowed in flight at the end of this step (issued after what the next step reads)
    auto wait_out = [&]() {
      if constexpr (STEADY) {
        if constexpr (S == 0 && MS) vm_wait<5>();  // the strip is issued after this wait
        else if constexpr (S <= 2) vm_wait<5 + SPW>();
        else if constexpr (S == 3) vm_wait<6 + SPW>();
        else vm_wait<6>();
      } else {
        if constexpr (S == 0) vm_wait<5>();
        else if constexpr (S == 1) vm_wait<3>();
        else if constexpr (S == 2) vm_wait<1>();
        else vm_wait<0>();
      }
    };
    // ping-pong: the two wave groups run one barrier apart (the second group's extra prologue
    // barrier), so one group's MFMAs overlap the other's LDS reads
    wait_out();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    static_for<NT>([&](auto t) {
      constexpr int PH = quad_phase(2 * S + decltype(t)::value);
      static_for<2 * WC * WP>([&](auto u_c) {
        constexpr int u = decltype(u_c)::value, s2 = u / (WC * WP), i = (u / WP) % WC, j = u % WP;
        if constexpr (ZP_ABL != 2) MfmaTraits<T>::mma(acc[PH][i][j], af[t][s2][i], bfr[s2][j]);
        else acc[PH][i][j][0] += __uint_as_float(af[t][s2][i].x ^ bfr[s2][j].y);  // diagnostic: no MFMA
        // MS: strip piece k after MFMA 5 (k + 1) - 1 of step 0 (32 MFMAs), pinned between MFMAs
        constexpr int m = decltype(t)::value * 2 * WC * WP + u;
        if constexpr (MS && S == 0 && STEADY && ZP_ABL != 1 && (m + 1) % 5 == 0 && (m + 1) / 5 <= SPW) {
          constexpr int k = (m + 1) / 5 - 1;
          __builtin_amdgcn_sched_barrier(0);
#if defined(__HIP_DEVICE_COMPILE__)
          auto* d = (__attribute__((address_space(3))) void*)&lds[(9 * TC + (gp ^ 1) * SRP + (wid + 8 * k) * 8) * 8];
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, d, 16, sv[k], (cb + 1) * 128, 0, 0);
#endif
          __builtin_amdgcn_sched_barrier(0);
        }
      });
    });
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  using ST = std::integral_constant<bool, true>;
  using TL = std::integral_constant<bool, false>;
  auto chunk = [&](auto steady_c, int cb) {
    const int gp = cb & 1;
    step(std::integral_constant<int, 0>{}, steady_c, cb, gp);
    step(std::integral_constant<int, 1>{}, steady_c, cb, gp);
    step(std::integral_constant<int, 2>{}, steady_c, cb, gp);
    step(std::integral_constant<int, 3>{}, steady_c, cb, gp);
    step(std::integral_constant<int, 4>{}, steady_c, cb, gp);
    flip();
  };
  // prologue: strip of chunk 0, then the weights of slots 0..7 (slot 8 is issued by step 0)
  issue_s(0, 0);
#pragma unroll
  for (int sl = 0; sl < 8; ++sl) issue_w(sl, 0);
  vm_wait<6>();  // strip(0) and slots 0, 1 landed
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if (wid >= 4) __builtin_amdgcn_s_barrier();
  for (int cb = 0; cb < CB - 1; ++cb) chunk(ST{}, cb);
  chunk(TL{}, CB - 1);
  if (wid < 4) __builtin_amdgcn_s_barrier();
  if constexpr (ZP_ABL == 5) {  // diagnostic build: no epilogue (one store only if a sum is exactly 1)
    float sm = 0.f;
    static_for<4>([&](auto ph) {
#pragma unroll
      for (int i = 0; i < WC; ++i)
#pragma unroll
        for (int j = 0; j < WP; ++j) sm += acc[ph][i][j][0] + acc[ph][i][j][1] + acc[ph][i][j][2] + acc[ph][i][j][3];
    });
    if (sm == 1.f) ((float*)A.sub[0].y)[tid] = sm;
  } else {
    static_for<4>([&](auto ph) {
      conv_epilogue<T, WC, WP, NWP>(A, A.sub[ph], acc[ph], p0, c0, wc, wp, lane, M, GHW, bx, ph, 4, nullptr,
                                    (float*)lds);
    });
  }
}

// ------------------------------------------------------------------------------------
// Tiny-M 1x1 convs without statistics or residual (the ASPP image-pool conv, aspp.py:94-96: B
// pixels of a 1x1 image, 512 -> 256 channels).  One wave computes 16 output channels of one pixel:
// lanes split K into 16-byte chunks (coalesced 1 KB weight-row reads), f32 products, a butterfly
// sum over the 64 lanes, and k_conv's epilogue arithmetic (scale / shift, ReLU).  Opt-in (conv flag
// 1024): measured 16.8 vs 17.7 us per eager launch, i.e. both are launch latency, which the
// hipGraph-replayed inference step does not pay; the network tests pass with it enabled.
// ------------------------------------------------------------------------------------
// 1 x 1 conv with a narrow K and a wide output (the head's data gradient in training: 32 -> 320
// channels at 128 x 128, bs 32 -- 34 MB in, 335 MB out).  On k_conv's small-Cin tile it took 177 us
// (2.1 TB/s): one K step per 128 x 256 tile, so every workgroup was prologue + epilogue at one
// workgroup per CU.  Here a block stages the whole packed weight (Cout x Cin, <= 48 KB) in LDS in
// MFMA fragment order once, and each wave walks 16-pixel groups: one 16-byte activation load per lane
// and K step, Cout / 16 MFMAs from LDS fragments, the paired 8-channel epilogue's 16-byte stores.
// Same MFMAs over the same K order as k_conv (its extra K step of zero weights only adds zeros).
constexpr int C1N_MAXCB = 24;  // cout blocks of 16 (384 channels)
template <typename T, int NCB>  // NCB = Cout / 16 (compile-time: the accumulators stay in registers)
__global__ void __launch_bounds__(256) k_conv1x1n(const zp_conv_args A) {
  __shared__ uint4 wl[NCB * 2 * 64];
  const zp_conv_sub& S = A.sub[0];
  constexpr int ncb = NCB;
  const int nks = A.Cin / 32;
  for (int f = threadIdx.x; f < ncb * nks * 64; f += blockDim.x) {  // fragment (i, s), lane l
    const int l = f & 63, fs = f >> 6, i = fs / nks, ks = fs - i * nks;
    wl[f] = *(const uint4*)((const unsigned short*)S.w + (size_t)(i * 16 + (l & 15)) * A.k_pad + ks * 32 + (l >> 4) * 8);
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4;
  const long M = (long)A.N * A.GH * A.GW;
  const long ngroups = (M + 15) / 16;
  for (long grp = (long)blockIdx.x * 4 + wave; grp < ngroups; grp += (long)gridDim.x * 4) {
    const long p = grp * 16 + (lane & 15);
    const bool pok = p < M;
    uint4 b[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      b[ks] = (pok && ks < nks) ? *(const uint4*)((const unsigned short*)A.x + p * A.ldx + A.cx0 + ks * 32 + g * 8)
                                : make_uint4(0u, 0u, 0u, 0u);
    f32x4 acc[NCB];
#pragma unroll
    for (int i = 0; i < NCB; ++i) {
      acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
      MfmaTraits<T>::mma(acc[i], wl[(i * nks) * 64 + lane], b[0]);
      if (nks > 1) MfmaTraits<T>::mma(acc[i], wl[(i * nks + 1) * 64 + lane], b[1]);
    }
    // (stride 1, one sub-problem on the input grid: output pixel = p)
    unsigned short* Y = (unsigned short*)S.y + p * S.ldy + S.cy0;
#pragma unroll
    for (int i = 0; i < NCB; i += 2) {
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // all lanes active (cross-lane op)
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][r]), __float_as_uint(acc[i + 1][r]), false,
                                                         false);
        v[r] = __uint_as_float(sw[0]);
        v[r + 4] = __uint_as_float(sw[1]);
      }
      if (!pok) continue;
      const int cs = (i + (g & 1)) * 16 + (g >> 1) * 8;
      uint32_t o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = H16<T>::to(v[2 * r]) | (H16<T>::to(v[2 * r + 1]) << 16);
      *(uint4*)(Y + cs) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  }
}

template <typename T>
__device__ __forceinline__ void ld16x8(const T* p, float* v) {  // 8 16-bit values, one 16-byte load
  const uint4 u = *(const uint4*)p;
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = H16<T>::from(w[i] & 0xffffu);
    v[2 * i + 1] = H16<T>::from(w[i] >> 16);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) k_conv_smallm(const zp_conv_args A) {
  const zp_conv_sub& S = A.sub[0];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int m = blockIdx.y;  // grid point
  const int GHW = A.GH * A.GW;
  const int n = m / GHW, r = m - n * GHW, gy = r / A.GW, gx = r - gy * A.GW;
  const int iy = gy * A.sy + S.ty[0], ix = gx * A.sx + S.tx[0];
  const bool inb = (unsigned)iy < (unsigned)A.IH && (unsigned)ix < (unsigned)A.IW;
  const T* xr = (const T*)A.x + (((size_t)n * A.IH + (inb ? iy : 0)) * A.IW + (inb ? ix : 0)) * A.ldx + A.cx0;
  const int oy = gy * S.oys + S.oyo, ox = gx * S.oxs + S.oxo;
  const size_t pix = ((size_t)n * S.OH + oy) * S.OW + ox;
  const int co0 = blockIdx.x * 64 + w * 16;
  float acc[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
  for (int k0 = lane * 8; k0 < A.Cin; k0 += 512) {
    float xv[8];
    ld16x8<T>(xr + k0, xv);
#pragma unroll
    for (int i = 0; i < 8; ++i) xv[i] = inb ? xv[i] : 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      float wv[8];
      ld16x8<T>((const T*)S.w + (size_t)(co0 + q) * A.k_pad + k0, wv);  // rows < w_rows (host check)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[q] = fmaf(xv[i], wv[i], acc[q]);
    }
  }
#pragma unroll
  for (int q = 0; q < 16; ++q)
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) acc[q] += __shfl_xor(acc[q], off);
  if (lane < 16) {
    float v = acc[0];
#pragma unroll
    for (int q = 1; q < 16; ++q) v = lane == q ? acc[q] : v;
    const int co = co0 + lane;
    if (co < A.Cout) {
      const float sc = S.scale ? S.scale[co] : 1.f, sh = S.shift ? S.shift[co] : 0.f;
      v = v * sc + sh;
      if (A.relu) v = fmaxf(v, 0.f);
      ((T*)S.y)[pix * S.ldy + S.cy0 + co] = Elem<T>::cvt(v);
    }
  }
}

// ------------------------------------------------------------------------------------
// weight gradient:  ws[split][sub][co][col] = sum over the split's grid points of
//   dy[out pixel][co] * x[in pixel (tap of col)][ci of col],   col = t*Cin + ci
// K (pixels) is the MFMA reduction axis, so both LDS tiles [pixel][channel] are read
// transposed with ds_read_b64_tr_b16 (bf16) / per-lane b32 (f32).
// ------------------------------------------------------------------------------------
template <typename T> struct WgTraits;
template <> struct WgTraits<bf16_t> { static constexpr int KP = 32; };  // pixels per K step
template <> struct WgTraits<float> { static constexpr int KP = 16; };

constexpr int WG_TILE = 128;            // co x col tile
constexpr int WG_ROWB = 256 + 16;       // LDS row bytes (128 ch of bf16 / 64 of f32 -> see below)

template <typename T>
__global__ void __launch_bounds__(256) k_wgrad(const zp_wgrad_args A, float* __restrict__ ws, int pix_per_split,
                                                int col_tiles, int cols_max) {
  constexpr int KP = WgTraits<T>::KP;
  constexpr int CHE = 16 / sizeof(T);            // elements per 16 B chunk
  constexpr int NCH = WG_TILE / CHE;             // chunks per 128-channel row (16 bf16 / 32 f32)
  constexpr int ROWB = WG_TILE * sizeof(T) + 16; // padded LDS row bytes
  constexpr int TILEB = KP * ROWB;
  constexpr int LPT = KP * NCH / 256;            // chunk loads per thread per tile (2)
  __shared__ __attribute__((aligned(16))) unsigned char lds[2][2][TILEB];

  const int sub = blockIdx.z;
  const auto& S = A.sub[sub];
  const int cols = S.ntaps * A.Cin;
  const int ct = blockIdx.y % col_tiles, cot = blockIdx.y / col_tiles;
  const int col0 = ct * WG_TILE, co0 = cot * WG_TILE;
  if (col0 >= cols) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wc = wid >> 1, wk = wid & 1;
  const int GHW = A.GH * A.GW;
  const int M = A.N * GHW;
  const int pbeg = blockIdx.x * pix_per_split;
  const int pend = min(M, pbeg + pix_per_split);

  // thread -> (row, chunk) of both tiles; chunk column fixed for the whole kernel
  const int qc = tid % NCH, qr = tid / NCH;      // rows qr + (256/NCH)*i
  constexpr int RSTEP = 256 / NCH;
  // dy channel of this chunk
  const int dco = co0 + qc * CHE;
  const bool dco_ok = dco < A.Cout;
  // x column of this chunk -> (tap, ci)
  const int xcol = col0 + qc * CHE;
  const bool xcol_ok = xcol < cols;
  const int xt = xcol_ok ? xcol / A.Cin : 0;
  const int xci = xcol - xt * A.Cin;
  const int xty = S.ty[xt], xtx = S.tx[xt];
  const T* __restrict__ X = (const T*)A.x;
  const T* __restrict__ DY = (const T*)S.dy;

  uint4 rd[LPT], rx[LPT];
  auto gload = [&](int pk) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      int p = pk + qr + RSTEP * i;
      uint4 vd = make_uint4(0, 0, 0, 0), vx = make_uint4(0, 0, 0, 0);
      if (p < pend) {
        int n = p / GHW, rr = p - n * GHW;
        int gy = rr / A.GW, gx = rr - gy * A.GW;
        if (dco_ok) {
          int oy = gy * S.oys + S.oyo, ox = gx * S.oxs + S.oxo;
          vd = *(const uint4*)(DY + (((size_t)n * S.OH + oy) * S.OW + ox) * S.lddy + S.cdy0 + dco);
        }
        int iy = gy * A.sy + xty, ix = gx * A.sx + xtx;
        if (xcol_ok && (unsigned)iy < (unsigned)A.IH && (unsigned)ix < (unsigned)A.IW)
          vx = *(const uint4*)(X + (((size_t)n * A.IH + iy) * A.IW + ix) * A.ldx + A.cx0 + xci);
      }
      rd[i] = vd;
      rx[i] = vx;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      int row = qr + RSTEP * i;
      *(uint4*)(&lds[buf][0][row * ROWB + qc * 16]) = rd[i];
      *(uint4*)(&lds[buf][1][row * ROWB + qc * 16]) = rx[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nsteps = pend > pbeg ? (pend - pbeg + KP - 1) / KP : 0;
  if (nsteps > 0) {
    gload(pbeg);
    sstore(0);
  }
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) gload(pbeg + (s + 1) * KP);
    const unsigned char* TD = lds[buf][0];
    const unsigned char* TX = lds[buf][1];
    if constexpr (sizeof(T) == 2) {
      // A[co][k] and B[k][col]: lane l of group g = l>>4 needs k = 8g..8g+7 of column (l & 15)
      typedef __attribute__((ext_vector_type(4))) short s4;
      const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
      bf16x8 af[4], bfm[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int cbase = wc * 64 + i * 16 + 4 * pp;
        const unsigned char* a0 = TD + (8 * g + q) * ROWB + cbase * 2;
        s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(a0));
        s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(a0 + 4 * ROWB));
        typedef __attribute__((ext_vector_type(8))) short s8;
        s8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        af[i] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int cbase = wk * 64 + j * 16 + 4 * pp;
        const unsigned char* b0 = TX + (8 * g + q) * ROWB + cbase * 2;
        s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(b0));
        s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(b0 + 4 * ROWB));
        typedef __attribute__((ext_vector_type(8))) short s8;
        s8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        bfm[j] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfm[j], acc[i][j], 0, 0, 0);
    } else {
      // f32: A[i=l&15][k=l>>4], B[k=l>>4][j=l&15]; 4 MFMAs of K=4 per 16-pixel step
      const int li = lane & 15, g = lane >> 4;
#pragma unroll
      for (int kk = 0; kk < KP; kk += 4) {
        float av[4], bv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          av[i] = *(const float*)(TD + (kk + g) * ROWB + (wc * 64 + i * 16 + li) * 4);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          bv[j] = *(const float*)(TX + (kk + g) * ROWB + (wk * 64 + j * 16 + li) * 4);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
    }
    if (s + 1 < nsteps) sstore(buf ^ 1);
    __syncthreads();
  }
  // write partial tile: ws[((split*nsub + sub)*Cout + co)*cols_max + col]
  float* W = ws + ((size_t)blockIdx.x * A.nsub + sub) * (size_t)A.Cout * cols_max;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int col = col0 + wk * 64 + j * 16 + (lane & 15);
      if (col >= cols) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int co = co0 + wc * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (co < A.Cout) W[(size_t)co * cols_max + col] = acc[i][j][r];
      }
    }
}

// ------------------------------------------------------------------------------------
// bf16 weight gradient, LDS-DMA version.  Same product and workspace layout as k_wgrad.
//
// A workgroup of 8 waves owns a (64*NA output channels) x (64*NB columns) tile; wave
// (a, b) = (w / NB, w % NB) computes a 64 x 64 block with 4 x 4 v_mfma_f32_16x16x32_bf16.
// Every K step covers KP consecutive grid points (pixels).  The stage image is NA + NB
// "panels" of [KP pixel rows][64 channels] (128 B rows): panels 0..NA-1 hold dy channels,
// panels NA.. hold x columns (tap, channel).  They are filled straight from global memory by
// buffer_load ... lds (one wave-instruction = 8 rows), STAGES-deep ring, counted vmcnt + raw
// barrier per step, exactly as k_conv does.
//
// The MFMA reduces over pixels, so both operands are read transposed with
// ds_read_b64_tr_b16: lane 4q+p of 16-lane group g supplies row (8g + q) and columns
// 4p..4p+3 of a 16-column block and receives one column (4 consecutive pixels).  Chunk
// swizzle: the 16 B chunk c of row R sits at chunk c ^ s(R), s(R) = 2 * (bit1(R) | bit3(R) << 1)
// (even, so the chunk pair of a 16-column block stays adjacent): the 8 rows a 32-lane half
// reads (two groups, rows 8g+q, q < 4) then cover all 64 banks once -- conflict-free.  The
// LDS-DMA writes are lane-linear, so the swizzle is applied on the per-lane SOURCE chunk.
//
// The tap walk is per lane: each lane always loads the same pixel row R of the tile (the
// instruction -> row-block map is wave-constant), so the grid point (n, gy, gx) advances
// incrementally by KP per issued step -- no divisions in the loop.
// ------------------------------------------------------------------------------------
struct wg_bounds {
  unsigned x_bytes, dy_bytes[ZP_MAX_SUB];
};

__device__ __forceinline__ int wg_swz(int r) { return (((r >> 1) & 1) | (((r >> 3) & 1) << 1)) << 1; }

template <int OFF>
__device__ __forceinline__ uint2 ds_read_tr8(unsigned addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset range");
  uint2 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF) : "memory");
  return r;
}

template <int KP, int NA, int NB, int STAGES, int WN>
__global__ void __launch_bounds__(512) k_wgrad_lds(const zp_wgrad_args A, float* __restrict__ ws, int pix_per_split,
                                                   int col_tiles, int tiles_per_sub, int cols_max,
                                                   const wg_bounds WB) {
  static_assert(NA * NB == 8 * WN, "8 waves of 64 x (64 WN)");
  constexpr int NBW = NB / WN;           // wave columns
  static_assert(KP == 32 || KP == 64, "K step");
  static_assert(STAGES == 2 || STAGES == 3, "ring depth");
  constexpr int NP = NA + NB;            // panels per stage
  constexpr int PB = KP * 128;           // panel bytes
  constexpr int SB = NP * PB;            // stage bytes
  constexpr int IPP = KP / 8;            // wave-instructions per panel
  constexpr int NI = NP * IPP;           // wave-instructions per stage
  constexpr int JPW = (NI + 7) / 8;      // per wave (the last may be idle)
  static_assert(SB * STAGES <= 160 * 1024, "LDS");
  __shared__ uint4 lds0[SB / 16];
  __shared__ uint4 lds1[SB / 16];
  __shared__ uint4 lds2[STAGES == 3 ? SB / 16 : 1];
  auto bufp = [&](auto i_c) -> uint4* {
    constexpr int i = decltype(i_c)::value;
    if constexpr (i == 0) return lds0;
    else if constexpr (i == 1) return lds1;
    else return lds2;
  };

  // 1-D grid, XCD-aware: workgroups are dispatched round-robin over the 8 XCDs (separate L2s);
  // remap so that each XCD walks a contiguous range of (split, sub, tile) with the tiles
  // fastest -- every tile of one split reads the same dy / x pixel rows, which then meet in one
  // L2 instead of being fetched by all eight.
  const int total = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, pos = bid >> 3, q8 = total >> 3, r8 = total & 7;  // bijective for any total
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + pos;
  const int tiles = tiles_per_sub;
  const int tile = lin % tiles;
  const int rest = lin / tiles;
  const int sub = rest % A.nsub;
  const int split = rest / A.nsub;
  const auto& S = A.sub[sub];
  const int cols = S.ntaps * A.Cin;
  const int ct = tile % col_tiles, cot = tile / col_tiles;
  const int col0 = ct * 64 * NB, co0 = cot * 64 * NA;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wa = wid / NBW, wb = wid % NBW;  // wave (co panel, group of WN column panels)
  const int GHW = A.GH * A.GW;
  const int M = A.N * GHW;
  const int pbeg = split * pix_per_split;
  const int pend = min(M, pbeg + pix_per_split);
  const int nK = pend > pbeg ? (pend - pbeg + KP - 1) / KP : 0;

  // ---- staging state of this lane: pixel row R, source chunk of every panel
  const int rowblk = (KP == 64) ? wid : (wid & 3);
  // panel of this wave's j-th wave-instruction (instruction q = wid + 8 j, IPP per panel)
  auto panel_of = [&](int j) { return KP == 64 ? j : 2 * j + ((wid >> 2) & 1); };
  const int R = rowblk * 8 + (lane >> 3);
  const int lchunk = (lane & 7) ^ wg_swz(R);
  const int cout8 = (A.Cout + 7) & ~7;
  int poff[NP];        // per-panel lane offset (bytes; x panels: relative to the pixel base)
  int pty[NP], ptx[NP];
  bool pok[NP];
#pragma unroll
  for (int P = 0; P < NP; ++P) {
    if (P < NA) {
      const int ch = co0 + 64 * P + 8 * lchunk;
      pok[P] = ch < cout8;
      poff[P] = (S.cdy0 + ch) * 2;
      pty[P] = ptx[P] = 0;
    } else {
      const int col = col0 + 64 * (P - NA) + 8 * lchunk;
      pok[P] = col < cols;
      const int t = pok[P] ? col / A.Cin : 0;
      const int ci = col - t * A.Cin;
      pty[P] = S.ty[t];
      ptx[P] = S.tx[t];
      poff[P] = ((pty[P] * A.IW + ptx[P]) * A.ldx + A.cx0 + ci) * 2;
    }
  }
  // grid point of the next step to issue
  int pn, pgy, pgx;
  {
    const int p = min(pbeg + R, M - 1);
    pn = p / GHW;
    const int rr = p - pn * GHW;
    pgy = rr / A.GW;
    pgx = rr - pgy * A.GW;
  }
  int pnext = pbeg + R;
#if defined(__HIP_DEVICE_COMPILE__)
  const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)A.x, (short)0, (int)WB.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t drsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)S.dy, (short)0, (int)WB.dy_bytes[sub], 0x00020000);
#endif

  auto issue = [&](uint4* dst) {
    const bool pv = pnext < pend;
    const unsigned dbase =
        (unsigned)((((pn * S.OH + pgy * S.oys + S.oyo) * S.OW + pgx * S.oxs + S.oxo) * S.lddy) * 2);
    const int iy0 = pgy * A.sy, ix0 = pgx * A.sx;
    const int xbase = (((pn * A.IH + iy0) * A.IW + ix0) * A.ldx) * 2;
    unsigned voff[JPW];
#pragma unroll
    for (int j = 0; j < JPW; ++j) {
      const int P = panel_of(j);  // wave-uniform (compile-time for KP 64)
      voff[j] = 0x80000000u;
      if (P < NA) {
        if (pv && pok[P]) voff[j] = dbase + (unsigned)poff[P];
      } else if (P < NP) {
        const int iy = iy0 + pty[P], ix = ix0 + ptx[P];
        if (pv && pok[P] && (unsigned)iy < (unsigned)A.IH && (unsigned)ix < (unsigned)A.IW)
          voff[j] = (unsigned)(xbase + poff[P]);
      }
    }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int j = 0; j < JPW; ++j) {
      const int P = panel_of(j);
      if (P >= NP) continue;
      auto* d = (__attribute__((address_space(3))) void*)((unsigned char*)dst + P * PB + rowblk * 1024);
      if (P < NA) __builtin_amdgcn_raw_ptr_buffer_load_lds(drsrc, d, 16, voff[j], 0, 0, 0);
      else __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, d, 16, voff[j], 0, 0, 0);
    }
#endif
    pnext += KP;
    if (A.GW >= 16) {  // at most KP / 16 row wraps per step: predicated, no loop
      pgx += KP;
#pragma unroll
      for (int it = 0; it < KP / 16; ++it) {
        if (pgx >= A.GW) {
          pgx -= A.GW;
          if (++pgy == A.GH) {
            pgy = 0;
            ++pn;
          }
        }
      }
    } else {  // tiny grids (1x1 image-pool branch): divide
      const int p = min(pnext, M - 1);
      pn = p / GHW;
      const int rr = p - pn * GHW;
      pgy = rr / A.GW;
      pgx = rr - pgy * A.GW;
    }
  };

  f32x4 acc[4][4 * WN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4 * WN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // fragment read addresses: lane (g, 4q+p) -> row 8g + q, byte 8p of the 16-column block,
  // 16-column block ii at chunk pair 2*(ii ^ s'), s' = s(R) / 2 (independent of the +4 / +32
  // row offsets, which are immediates)
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int sh = (((q4 >> 1) & 1) | ((g & 1) << 1));
  unsigned ra[4];
#pragma unroll
  for (int ii = 0; ii < 4; ++ii) ra[ii] = (unsigned)(wa * PB) + (unsigned)(128 * (8 * g + q4) + 8 * p4 + 32 * (ii ^ sh));
  // column panel w of this wave = panel NA + wb * WN + w: an immediate offset w * PB

  auto step = [&](auto cur_c, auto nxt_c, int ks) {
    const bool more = ks + (STAGES - 1) < nK;
    if constexpr (ZP_ABL != 1) {
      if (more) issue(bufp(nxt_c));
    }
    const unsigned cb = lds_addr(bufp(cur_c));
    unsigned pa[4], pb[4];
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      pa[ii] = cb + ra[ii];
      pb[ii] = pa[ii] + (unsigned)((NA + wb * WN - wa) * PB);
    }
    static_for<KP / 32>([&](auto s2) {
      uint4 af[4], bfr[4 * WN];
      static_for<4>([&](auto ii) {
        const uint2 a0 = ds_read_tr8<s2 * 4096>(pa[ii]);
        const uint2 a1 = ds_read_tr8<s2 * 4096 + 512>(pa[ii]);
        af[ii] = make_uint4(a0.x, a0.y, a1.x, a1.y);
        static_for<WN>([&](auto w) {
          const uint2 b0 = ds_read_tr8<w * PB + s2 * 4096>(pb[ii]);
          const uint2 b1 = ds_read_tr8<w * PB + s2 * 4096 + 512>(pb[ii]);
          bfr[w * 4 + ii] = make_uint4(b0.x, b0.y, b1.x, b1.y);
        });
      });
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      if constexpr (ZP_ABL != 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4 * WN; ++j) MfmaTraits<bf16_t>::mma(acc[i][j], af[i], bfr[j]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][0][0] += __uint_as_float(af[i].x ^ bfr[i].y);
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(0);
    });
    if (more) vm_wait<JPW * (STAGES - 2)>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  if (nK > 0) {
    issue(lds0);
    if (STAGES == 3 && nK > 1) {
      issue(lds1);
      vm_wait<JPW * (STAGES - 2)>();
    } else {
      vm_wait<0>();
    }
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (STAGES == 3) {
    for (int ks = 0; ks < nK; ks += 3) {
      step(I0{}, I2{}, ks);
      if (ks + 1 >= nK) break;
      step(I1{}, I0{}, ks + 1);
      if (ks + 2 >= nK) break;
      step(I2{}, I1{}, ks + 2);
    }
  } else {
    for (int ks = 0; ks < nK; ks += 2) {
      step(I0{}, I1{}, ks);
      if (ks + 1 >= nK) break;
      step(I1{}, I0{}, ks + 1);
    }
  }
  // partial tile -> ws[((split*nsub + sub)*Cout + co)*cols_max + col]
  float* W = ws + ((size_t)split * A.nsub + sub) * (size_t)A.Cout * cols_max;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4 * WN; ++j) {
      const int col = col0 + wb * WN * 64 + j * 16 + (lane & 15);
      if (col >= cols) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wa * 64 + i * 16 + g * 4 + r;
        if (co < A.Cout) W[(size_t)co * cols_max + col] = acc[i][j][r];
      }
    }
}

// ------------------------------------------------------------------------------------
// k_wgrad2: k_wgrad_lds's product (same tiles, same panels, same fragment reads, same partial
// layout) with a lean issue path for the common geometry: one sub-problem, stride 1, dy on the
// input grid (same-size convs: every 3x3 d-conv and 1x1 of the network), W in {32, 64, 128},
// images a multiple of the 64-pixel step, Cin and the dy channel slice 64-aligned.  Then the
// pixel offset of a lane's row in dy and x is LINEAR in the pixel index: the per-step offset is
// one scalar (p * ld * 2) added by the buffer unit; per lane only constant row / channel /
// tap offsets are kept, and a tap's row validity is wave-uniform per step (a 64-pixel step is
// one image row at W 64, half a row at W 128, two rows at W 32 whose halves are waves 0-3 and
// 4-7), its column validity a per-lane constant (W 128: one of two).  k_wgrad_lds, profiled on
// the 256->256 3x3 at 128x128 (bs 32), spent 1.4 VALU + 1.0 SALU per MFMA on per-step pixel
// arithmetic and ran the MFMA pipe 34% busy.
// Stride 2 (round 6; the input grid twice the output grid): a lane's x pixel is (S (gy + rh) + ty,
// S gx + tx) -- per lane (S rh + ty) IW + S gx + tx, per step the image and row (n IH + S gy) IW
// (+ S 64 for the second half of a W 128 row).  That covers the stride-2 convs and, with x and dy
// exchanged, the ConvTranspose2d(3, s2, p1, op1) weight gradient: dW[ci][co][ky][kx] = sum_g
// x[g][ci] dy[2 g + (ky, kx) - 1][co] is the weight gradient of the stride-2 conv over dy whose
// output gradient is x (geometry.convT_dgrad's plan; the engine's _wgrad).
// ------------------------------------------------------------------------------------
template <int NA, int NB, int STAGES, int WN>
__global__ void __launch_bounds__(512) k_wgrad2(const zp_wgrad_args A, float* __restrict__ ws, int pix_per_split,
                                                int col_tiles, int tiles_per_sub, int cols_max, const wg_bounds WB) {
  constexpr int KP = 64;
  static_assert(NA * NB == 8 * WN, "8 waves of 64 x (64 WN)");
  constexpr int NBW = NB / WN;
  constexpr int NP = NA + NB;   // panels per stage; wave w fills rows 8w..8w+7 of every panel
  constexpr int PB = KP * 128;  // panel bytes
  constexpr int SB = NP * PB;   // stage bytes
  static_assert(SB * STAGES <= 160 * 1024, "LDS");
  __shared__ uint4 lds[STAGES * SB / 16];

  // XCD-aware order (bijective for any total): each XCD walks a contiguous run of (split, tile),
  // tiles fastest, so the tiles of one split (same dy / x pixel rows) share an L2
  const int total = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, pos = bid >> 3, q8 = total >> 3, r8 = total & 7;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + pos;
  const int tile = lin % tiles_per_sub;
  const int split = lin / tiles_per_sub;  // one sub-problem
  const auto& S = A.sub[0];
  const int cols = S.ntaps * A.Cin;
  const int ct = tile % col_tiles, cot = tile / col_tiles;
  const int col0 = ct * 64 * NB, co0 = cot * 64 * NA;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wa = wid / NBW, wb = wid % NBW;
  const int W = A.GW, GHW = A.GH * A.GW;
  const int M = A.N * GHW;
  const int pbeg = split * pix_per_split;
  const int pend = min(M, pbeg + pix_per_split);
  const int nK = pend > pbeg ? (pend - pbeg) / KP : 0;

  const int R = wid * 8 + (lane >> 3);  // this lane's pixel row within a step
  const int lchunk = (lane & 7) ^ wg_swz(R);
  const int cout8 = (A.Cout + 7) & ~7;
  const int rh = W == 32 ? (wid >> 2) : 0;  // image-row offset of this wave's rows (wave-uniform)
  const int gxl = W == 32 ? (R & 31) : R;   // column (W 128: + 64 * xh)
  const int SS = A.sy;                      // input stride (1, or 2 with IH = 2 GH, IW = 2 GW)
  // per panel: lane offsets (dy: row + channel; x: row + tap + channel, with column validity folded
  // in as an out-of-range offset), tap row of x panels (wave-uniform)
  unsigned vdy[NA];
  int vx[NB];                // x: row + tap + channel offset (bytes; may be negative, the step adds p)
  bool okx0[NB], okx1[NB];   // column validity (W 128: column half 0 / 1)
  int tyP[NB];
#pragma unroll
  for (int P = 0; P < NA; ++P) {
    const int ch = co0 + 64 * P + 8 * lchunk;
    vdy[P] = ch < cout8 ? (unsigned)((R * S.lddy + S.cdy0 + ch) * 2) : 0x80000000u;
  }
#pragma unroll
  for (int P = 0; P < NB; ++P) {
    const int col = col0 + 64 * P + 8 * lchunk;
    const bool ok = col < cols;
    const int t = ok ? col / A.Cin : 0;
    const int ci = col - t * A.Cin;
    const int ty = S.ty[t], tx = S.tx[t];
    tyP[P] = __builtin_amdgcn_readfirstlane(S.ty[(col0 + 64 * P) / A.Cin < S.ntaps ? (col0 + 64 * P) / A.Cin : 0]);
    vx[P] = ((SS * rh + ty) * A.IW + SS * gxl + tx) * A.ldx * 2 + (A.cx0 + ci) * 2;
    okx0[P] = ok && (unsigned)(SS * gxl + tx) < (unsigned)A.IW;
    okx1[P] = ok && (unsigned)(SS * (gxl + 64) + tx) < (unsigned)A.IW;
  }
#if defined(__HIP_DEVICE_COMPILE__)
  const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)A.x, (short)0, (int)WB.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t drsrc = __builtin_amdgcn_make_buffer_rsrc((void*)S.dy, (short)0, (int)WB.dy_bytes[0], 0x00020000);
#endif
  // scalar walk: pixel p of the next step to issue, its image row gy and (W 128) column half xh
  int p_is = pbeg;
  int gy_is, xh_is, n_is = pbeg / GHW;
  {
    const int r = pbeg % GHW;
    gy_is = r / W;
    xh_is = W == 128 ? (r / 64) & 1 : 0;
  }
  const int ldy2 = S.lddy * 2, ldx2 = A.ldx * 2;
  auto issue = [&](auto slot_c) {
    constexpr int SL = decltype(slot_c)::value;
    const int sdy = p_is * ldy2;
    const int sx = ((n_is * A.IH + SS * gy_is) * A.IW + SS * 64 * xh_is) * ldx2;  // (S 1: p_is * ldx2)
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int P = 0; P < NA; ++P) {
      auto* d = (__attribute__((address_space(3))) void*)((unsigned char*)lds + SL * SB + P * PB + wid * 1024);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(drsrc, d, 16, vdy[P], sdy, 0, 0);
    }
#pragma unroll
    for (int P = 0; P < NB; ++P) {
      // the full (non-negative when valid) offset in the VGPR: a lane offset below zero is never
      // handed to the buffer unit, whatever its range check does with the scalar part
      const bool rowok = (unsigned)(SS * (gy_is + rh) + tyP[P]) < (unsigned)A.IH;  // wave-uniform
      const bool ok = rowok && (xh_is ? okx1[P] : okx0[P]);
      const unsigned v = ok ? (unsigned)(vx[P] + sx) : 0x80000000u;
      auto* d = (__attribute__((address_space(3))) void*)((unsigned char*)lds + SL * SB + (NA + P) * PB + wid * 1024);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, d, 16, v, 0, 0, 0);
    }
#endif
    // advance one 64-pixel step (images are whole steps: GHW % 64 == 0)
    p_is += KP;
    if (W == 128) {
      xh_is ^= 1;
      if (xh_is == 0) ++gy_is;
    } else {
      gy_is += KP / W;
    }
    if (gy_is >= A.GH) {
      gy_is = 0;
      ++n_is;
    }
  };

  f32x4 acc[4][4 * WN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4 * WN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int sh = (((q4 >> 1) & 1) | ((g & 1) << 1));
  const unsigned l0 = lds_addr(lds);
  unsigned pa[STAGES][4], pb[STAGES][4];  // per ring slot (slot offsets exceed the ds immediate)
#pragma unroll
  for (int sl = 0; sl < STAGES; ++sl)
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      pa[sl][ii] = l0 + (unsigned)(sl * SB + wa * PB) + (unsigned)(128 * (8 * g + q4) + 8 * p4 + 32 * (ii ^ sh));
      pb[sl][ii] = pa[sl][ii] + (unsigned)((NA + wb * WN - wa) * PB);
    }
  auto step = [&](auto cur_c, auto nxt_c, int ks) {
    constexpr int CUR = decltype(cur_c)::value;
    const bool more = ks + (STAGES - 1) < nK;
    if constexpr (ZP_ABL != 1) {
      if (more) issue(nxt_c);
    }
    static_for<KP / 32>([&](auto s2) {
      uint4 af[4], bfr[4 * WN];
      static_for<4>([&](auto ii) {
        const uint2 a0 = ds_read_tr8<s2 * 4096>(pa[CUR][ii]);
        const uint2 a1 = ds_read_tr8<s2 * 4096 + 512>(pa[CUR][ii]);
        af[ii] = make_uint4(a0.x, a0.y, a1.x, a1.y);
        static_for<WN>([&](auto w) {
          const uint2 b0 = ds_read_tr8<w * PB + s2 * 4096>(pb[CUR][ii]);
          const uint2 b1 = ds_read_tr8<w * PB + s2 * 4096 + 512>(pb[CUR][ii]);
          bfr[w * 4 + ii] = make_uint4(b0.x, b0.y, b1.x, b1.y);
        });
      });
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      if constexpr (ZP_ABL != 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4 * WN; ++j) MfmaTraits<bf16_t>::mma(acc[i][j], af[i], bfr[j]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][0][0] += __uint_as_float(af[i].x ^ bfr[i].y);
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(0);
    });
    if (more) vm_wait<NP * (STAGES - 2)>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  if (nK > 0) {
    issue(I0{});
    if (STAGES == 3 && nK > 1) {
      issue(I1{});
      vm_wait<NP * (STAGES - 2)>();
    } else {
      vm_wait<0>();
    }
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (STAGES == 3) {
    for (int ks = 0; ks < nK; ks += 3) {
      step(I0{}, I2{}, ks);
      if (ks + 1 >= nK) break;
      step(I1{}, I0{}, ks + 1);
      if (ks + 2 >= nK) break;
      step(I2{}, I1{}, ks + 2);
    }
  } else {
    for (int ks = 0; ks < nK; ks += 2) {
      step(I0{}, I1{}, ks);
      if (ks + 1 >= nK) break;
      step(I1{}, I0{}, ks + 1);
    }
  }
  float* Wp = ws + (size_t)split * (size_t)A.Cout * cols_max;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4 * WN; ++j) {
      const int col = col0 + wb * WN * 64 + j * 16 + (lane & 15);
      if (col >= cols) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wa * 64 + i * 16 + g * 4 + r;
        if (co < A.Cout) Wp[(size_t)co * cols_max + col] = acc[i][j][r];
      }
    }
}

// ws (summed over splits) -> dw in the weight's own layout.  Per element the splits are summed into
// 8 partial sums (split k into q[k % 8] for the whole batches of 8, the rest into q[0]), combined as
// ((q0 + q1) + (q2 + q3)) + ((q4 + q5) + (q6 + q7)): fixed order, deterministic.  (Round 5) up to 32
// splits' loads are issued before their adds (the same adds in the same order as batches of 8; one
// batch of 8 in flight left the launch bound by 3-4 dependent memory round trips per thread), and
// the element index is 32-bit.
__global__ void __launch_bounds__(256) k_wgrad_reduce(const zp_wgrad_args A, const float* __restrict__ ws, int splits,
                                                      int cols_max) {
  const int sub = blockIdx.y;
  const auto& S = A.sub[sub];
  const unsigned cols = (unsigned)(S.ntaps * A.Cin);
  const unsigned total = (unsigned)A.Cout * cols;
  const size_t stride = (size_t)A.nsub * A.Cout * cols_max;
  for (unsigned e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const unsigned co = e / cols, col = e - co * cols;
    const int t = (int)(col / (unsigned)A.Cin), ci = (int)col - t * A.Cin;
    const int ky = S.ky[t], kx = S.kx[t];
    if (ci >= A.Cw || ky < 0) continue;  // padded input channels / padding taps
    const float* p = ws + ((size_t)sub * A.Cout + co) * cols_max + col;
    float q[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int k = 0;
    for (; k + 32 <= splits; k += 32) {
      float v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = p[(size_t)(k + u) * stride];
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int u = 0; u < 8; ++u) q[u] += v[8 * b + u];
    }
    if (k + 16 <= splits) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = p[(size_t)(k + u) * stride];
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int u = 0; u < 8; ++u) q[u] += v[8 * b + u];
      k += 16;
    }
    if (k + 8 <= splits) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[(size_t)(k + u) * stride];
#pragma unroll
      for (int u = 0; u < 8; ++u) q[u] += v[u];
      k += 8;
    }
    {
      float v[7];  // the remaining < 8 splits, loaded together, added to q[0] in split order
#pragma unroll
      for (int u = 0; u < 7; ++u) v[u] = k + u < splits ? p[(size_t)(k + u) * stride] : 0.f;
#pragma unroll
      for (int u = 0; u < 7; ++u)
        if (k + u < splits) q[0] += v[u];
    }
    const float s = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
    size_t idx = A.transposed_w ? (((size_t)ci * A.Cout + co) * A.kh + ky) * A.kw + kx
                                : (((size_t)co * A.Cw + ci) * A.kh + ky) * A.kw + kx;
    if (A.accumulate) A.dw[idx] += s;
    else A.dw[idx] = s;
  }
}

}  // namespace zp

using namespace zp;

// ------------------------------------------------------------------------------------ host
static int conv_flags();

template <typename T, int WC, int NWP, int STAGES, bool SMALLC>
static void launch_conv(const zp_conv_args& a, const conv_taps& tg, int gx, int gy, hipStream_t st) {
  hipLaunchKernelGGL((k_conv<T, WC, 4, NWP, STAGES, SMALLC>), dim3(gx, gy, a.nsub), dim3(128 * NWP), 0, st,
                     a, tg, conv_flags());
}
// 256 x 256 tile (bf16 only): 64 KB per LDS stage, so a 2-deep ring
template <typename T>
static void launch_conv_tc256(const zp_conv_args& a, const conv_taps& tg, int gx, int gy, hipStream_t st) {
  if constexpr (sizeof(T) == 2) launch_conv<T, 8, 4, 2, false>(a, tg, gx, gy, st);
}

// Tuning overrides for sweeps (read once): ZP_CONV_TP=128|256 forces the pixel tile,
// ZP_CONV_STAGES=2|3 forces the LDS ring depth, ZP_CONV_TC256=0 disables the 256-channel tile.
// 0 = heuristic.
static int env_int(const char* name) {
  const char* v = getenv(name);
  return v ? atoi(v) : 0;
}
static bool conv_tc256_enabled() {
  static const bool v = getenv("ZP_CONV_TC256") ? env_int("ZP_CONV_TC256") != 0 : true;
  return v;
}
// runtime tuning knobs (zp_conv_tuning): minimum workgroup count for the 256-channel tile
static int g_tc256_min_blocks = 1024;

// cout tile: 256 (the whole layer: activations are staged once per pixel tile instead of once per
// 128-channel tile, and 64 MFMAs per wave per LDS step instead of 32) for bf16 layers with
// Cout % 256 == 0; else 128 / 64 / 32.
// Measured (R34 bs 32, profiles/r01_conv_sweep.md): a win when the launch still has >= 1024
// workgroups of 256 pixels (64x64 / 128x128 layers, the 64x64 transposed-conv phases: 1.1-1.2x),
// a loss on 32x32 layers (128 workgroups for 256 CUs), on the 32x32 transposed-conv phases (512
// workgroups: 78.7 us vs 70.7 us on the 128-channel tile) and on the ASPP launch, whose four
// sub-problems (1 vs 9 taps) are too unbalanced for 512 large tiles.
static bool strip_eligible(const zp_conv_args& a, strip_geo* sg);
static bool quad_plan(const zp_conv_args& a, quad_geo* qg);
static int g_quad_min_blocks = 256;  // zp_conv_tuning key 6: fewest workgroups k_conv_quad runs with
static int g_strip_c64 = 1;  // zp_conv_tuning key 2: 64-channel layers on the strip kernel (TC 64; 27.5 -> 22.2 us at 64x64)
// strip tile width: 128 channels, or 64 when 128-channel tiles would leave part of the 256 CUs
// idle (128 -> 128 at 32x32, bs 32: 128 workgroups; 24.2 -> 22.7 us).  64-channel layers stay on
// k_conv's 128-pixel tiles (27.5 us there vs 29.2 us as a 64-channel strip).
static int strip_tc(const zp_conv_args& a) {
  static const int en64 = getenv("ZP_STRIP_TC64") ? env_int("ZP_STRIP_TC64") : 1;
  if (a.Cout <= 64) return 64;
  if (!en64) return 128;
  const long tiles = (long)a.N * a.GH * a.GW / 256;
  if (tiles * ((a.Cout + 127) / 128) < 256) return 64;
  return 128;
}
static int conv_tc(const zp_conv_args& a) {
  if (a.dtype == ZP_F32X3 || a.dtype == ZP_F32H2) return conv3_tc(a);  // k_conv3 / k_conv3s
  if (quad_plan(a, nullptr)) return 64;  // k_conv_quad: 64 channels x 4 phases
  // strip-eligible layers take k_conv_strip's 128-channel tile: it stages fewer bytes per FLOP than
  // the 256-channel k_conv tile, and a 256-channel strip tile does not fit the register file
  // (35 spilled VGPRs)
  if (strip_eligible(a, nullptr)) return strip_tc(a);
  if (a.dtype != ZP_F32 && a.Cout % 256 == 0 && a.Cin >= 64 && conv_tc256_enabled()) {
    const long M = (long)a.N * a.GH * a.GW;
    int tmin = ZP_MAX_TAPS, tmax = 0;
    for (int s = 0; s < a.nsub; ++s) {
      tmin = a.sub[s].ntaps < tmin ? a.sub[s].ntaps : tmin;
      tmax = a.sub[s].ntaps > tmax ? a.sub[s].ntaps : tmax;
    }
    if (ceil_div(M, 256) * (long)a.nsub >= g_tc256_min_blocks && tmax <= 4 * tmin) return 256;
  }
  return a.Cout > 64 ? 128 : (a.Cout > 32 ? 64 : 32);
}
static int conv_tp_override() {
  static const int v = env_int("ZP_CONV_TP");
  return v;
}
static int conv_stages_override() {
  static const int v = env_int("ZP_CONV_STAGES");
  return v;
}

// conv schedule switches: bit 1 XCD-aware tile order, bit 2 s_setprio(1) around the MFMA
// cluster, bit 3 ping-pong (staggered wave groups), bit 4 tap-row trimming (tap rows that read only
// padding for a whole tile are skipped), bit 5 spread strip DMA (k_conv_strip only; slower), bit 6
// k_conv_strip2 instead of k_conv_strip, bit 7 k_conv_quad for the four phases of stride-2 transposed
// structures (ConvTranspose2d forward, stride-2 conv data gradient), bit 8 k_conv_strip2 issues the
// next strip's DMA between the MFMAs of a group's first step (DM 2).  Default (measured, profiles/r01_conv_sweep.md,
// profiles/r02_conv_ab.md): XCD order + setprio + ping-pong + trimming + k_conv_strip2 (94).
// ZP_CONV_FLAGS / zp_conv_tuning(1, .) override for sweeps.
static int g_conv_flags = -1;  // zp_conv_tuning key 1 (runtime A/B in one process); -1 = env / default
static int conv_flags() {
  static const int v = getenv("ZP_CONV_FLAGS") ? env_int("ZP_CONV_FLAGS") : 94 + 128 + 256;
  return g_conv_flags >= 0 ? g_conv_flags : v;
}

// 3x3 stride-1 same-size bf16 convs on full-width tiles (W 32 / 64 / 128) whose strip of
// TR x (W + 2 pad) pixels fits the 320-row LDS slot run k_conv_strip (256-pixel tiles).
// ZP_CONV_STRIP=0 disables.
static bool strip_eligible(const zp_conv_args& a, strip_geo* sg) {
  static const int en = getenv("ZP_CONV_STRIP") ? env_int("ZP_CONV_STRIP") : 1;
  if (!en || a.dtype == ZP_F32 || a.dtype == ZP_F32X3 || a.dtype == ZP_F32H2 || a.nsub != 1 || a.Cin % 64 != 0 || a.Cout % 64 != 0)
    return false;
  if (a.Cout <= 64 && !g_strip_c64) return false;
  if (a.sy != 1 || a.sx != 1 || a.GH != a.IH || a.GW != a.IW) return false;
  const zp_conv_sub& S = a.sub[0];
  if (S.ntaps != 9 || S.oys != 1 || S.oxs != 1 || S.oyo != 0 || S.oxo != 0 || S.OH != a.GH || S.OW != a.GW)
    return false;
  const int ty0 = S.ty[0], tx0 = S.tx[0], dty = S.ty[3] - S.ty[0], dtx = S.tx[1] - S.tx[0];
  for (int t = 0; t < 9; ++t)
    if (S.ty[t] != ty0 + (t / 3) * dty || S.tx[t] != tx0 + (t % 3) * dtx) return false;
  const int W = a.GW;
  if (W != 32 && W != 64 && W != 128) return false;
  if (((long)a.GH * a.GW) % 256 != 0) return false;
  int pad = 0;
  for (int k = 0; k < 3; ++k) {
    pad = max(pad, abs(ty0 + k * dty));
    pad = max(pad, abs(tx0 + k * dtx));
  }
  const int TR = 256 / W, SW = W + 2 * pad, SR = TR * SW;
  if (SR > 320) return false;
  if (sg) {
    sg->W = W;
    sg->TR = TR;
    sg->SW = SW;
    sg->SR = SR;
    sg->SPW = 5;
    sg->ty0 = ty0;
    sg->dty = dty;
    sg->tx0 = tx0;
    sg->dtx = dtx;
    sg->pad = pad;
  }
  return true;
}

// k_conv_quad eligibility: 16-bit, the four phases (py, px) = (0,0), (0,1), (1,0), (1,1) of a
// stride-2 transposed structure over an input the size of the grid (W 32 / 64), 1 / 2 / 2 / 4 taps
// at input offsets in {0,1}^2 (geometry.py _phases with k = 3, p = 1), channels in whole chunks, and
// enough workgroups to cover the CUs.  qg: the byte offset of each schedule slot's tap.
static bool quad_plan(const zp_conv_args& a, quad_geo* qg) {
  if (!(conv_flags() & 128)) return false;
  if (a.dtype == ZP_F32 || a.dtype == ZP_F32X3 || a.dtype == ZP_F32H2 || a.nsub != 4 || a.Cin % 64 != 0 || a.Cout % 64 != 0) return false;
  if (a.sy != 1 || a.sx != 1 || a.GH != a.IH || a.GW != a.IW) return false;
  if (a.GW != 32 && a.GW != 64) return false;
  if (((long)a.GH * a.GW) % 256 != 0) return false;
  if ((long)a.N * a.GH * a.GW / 256 * (a.Cout / 64) < g_quad_min_blocks) return false;
  static const int ntap[4] = {1, 2, 2, 4};
  for (int s = 0; s < 4; ++s) {
    const zp_conv_sub& S = a.sub[s];
    if (S.oys != 2 || S.oxs != 2 || S.oyo != s / 2 || S.oxo != s % 2 || S.ntaps != ntap[s]) return false;
    if (S.OH < 2 * a.GH || S.OW < 2 * a.GW) return false;
  }
  // slot -> (ty, tx) (the sub is quad_phase(slot))
  static const int shift[9][2] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 1}, {0, 1}, {1, 0}, {1, 0}, {1, 1}};
  int used[4] = {0, 0, 0, 0};
  for (int k = 0; k < 9; ++k) {
    const int ph = quad_phase(k);
    const zp_conv_sub& S = a.sub[ph];
    int t = 0;
    while (t < S.ntaps && !(S.ty[t] == shift[k][0] && S.tx[t] == shift[k][1])) ++t;
    if (t == S.ntaps || (used[ph] >> t) & 1) return false;
    used[ph] |= 1 << t;
    if (qg) qg->koff[k] = t * a.Cin * 2;
  }
  return true;
}

// pixel tile: 256 (8 waves) whenever the cout tile allows it.  Measured on MI355X (R34 bs32,
// profiles/r01_conv_sweep.md): the 8-wave 3-stage tile beats the 4-wave tiles even on the
// 32x32 layers where it leaves part of the chip idle (fewer workgroups, but 2x the MFMA work
// per LDS byte and deeper prefetch)
static int conv_tp(const zp_conv_args& a) {
  if (a.dtype == ZP_F32X3 || a.dtype == ZP_F32H2) return conv3_tp(a, conv3_tc(a));
  int tc = a.Cout > 64 ? 128 : (a.Cout > 32 ? 64 : 32);
  if (tc == 32) return 128;  // 32 + 256 rows do not split over 8 waves in 8-row groups
  if (strip_eligible(a, nullptr) || quad_plan(a, nullptr)) return 256;
  if (conv_tc(a) == 256) return 256;  // the 256-channel tile exists only with 256-pixel tiles
  const int ov = conv_tp_override();
  if (ov == 128 || ov == 256) return ov;
  // Cout <= 128 (one cout tile): 128-pixel tiles double the workgroup count of the 32x32 / 64x64
  // layers (tools/conv_micro.py: 128->128 @32x32 36 -> 24 us, 64->64 @64x64 28.6 -> 26.3 us);
  // the small-Cin stem keeps 256
  const int E = a.dtype == ZP_F32 ? 4 : 8;
  if (a.Cout <= 128 && a.Cin >= 8 * E) return 128;
  return 256;
}

// LDS ring depth: 3, except for the two launches with very few or gather-bound K steps, where the
// 2-deep ring's smaller LDS footprint (more resident workgroups) wins (R34 bs 32, layer report):
// the small-Cin stem (7x7, per-lane tap gather: 100 -> 75 us) and the 32-channel-tile head
// (1x1 320 -> 17 at 128x128, 5 K steps, HBM-bound: 99 -> 90 us).  Every other k_conv launch loses
// with 2 stages (ASPP 217 -> 329 us).
static int conv_stages(const zp_conv_args& a, int tc) {
  const int ov = conv_stages_override();
  if (ov == 2 || ov == 3) return ov;
  const int ke = a.dtype == ZP_F32 ? 32 : 64;  // elements per K step
  if (a.Cin < ke || tc <= 32) return 2;
  return 3;
}

extern "C" int zp_conv2d_stat_parts(const zp_conv_args* a);

// k_conv1x1n's geometry (ZP_CONV1X1N=0 turns it off)
static int num_cus();
static bool conv1x1n_ok(const zp_conv_args& a) {
  static const int en1n = getenv("ZP_CONV1X1N") ? env_int("ZP_CONV1X1N") : 1;
  const zp_conv_sub& S = a.sub[0];
  return en1n && (a.dtype == ZP_BF16 || a.dtype == ZP_F16) && a.nsub == 1 && S.ntaps == 1 && S.ty[0] == 0 &&
         S.tx[0] == 0 && (a.Cin == 32 || a.Cin == 64) && a.Cout % 64 == 0 && a.Cout / 16 <= C1N_MAXCB &&
         a.w_rows >= a.Cout && a.k_pad >= a.Cin && !a.stats && !a.bnr_part && !a.res && !a.relu &&
         a.out_mode == ZP_OUT_NHWC && !S.scale && !S.shift && S.ldy % 8 == 0 && S.cy0 % 8 == 0 && a.ldx % 8 == 0 &&
         a.cx0 % 8 == 0 && a.sy == 1 && a.sx == 1 && a.GH == a.IH && a.GW == a.IW && S.OH == a.GH && S.OW == a.GW &&
         S.oys == 1 && S.oxs == 1 && S.oyo == 0 && S.oxo == 0 && (long)a.N * a.GH * a.GW >= 65536;
}

extern "C" int zp_conv2d_grid(const zp_conv_args* a) {
  if (!a) return 0;
  long M = (long)a->N * a->GH * a->GW;
  return ceil_div(M, conv_tp(*a));
}

extern "C" int zp_conv2d(const zp_conv_args* ap, void* stream) {
  ZP_CHECK_ARG(ap != nullptr, "zp_conv2d: null args");
  const zp_conv_args& a = *ap;
  ZP_CHECK_ARG(a.dtype == ZP_F32 || a.dtype == ZP_BF16 || a.dtype == ZP_F16 || a.dtype == ZP_F32X3 ||
                   a.dtype == ZP_F32H2,
               "zp_conv2d: bad dtype %d", a.dtype);
  ZP_CHECK_ARG(a.nsub >= 1 && a.nsub <= ZP_MAX_SUB, "zp_conv2d: nsub %d", a.nsub);
  ZP_CHECK_ARG(a.x && a.N > 0 && a.GH > 0 && a.GW > 0 && a.IH > 0 && a.IW > 0 && a.Cout > 0,
               "zp_conv2d: bad geometry");
  ZP_CHECK_ARG(!a.bnr_part || (a.bnr_x && a.bnr_save && (a.dtype == ZP_F32 || a.dtype == ZP_BF16) && !a.stats &&
                                !a.res && !a.relu && a.out_mode == ZP_OUT_NHWC && a.Cout % 4 == 0),
               "zp_conv2d: bnr_* (fused BN backward reduce) needs a plain f32 / bf16 NHWC store (no stats, "
               "residual, ReLU), bnr_x and bnr_save, Cout %% 4 == 0");
  if (a.dtype == ZP_F32X3 || a.dtype == ZP_F32H2) return conv3_launch(a, (hipStream_t)stream, conv_flags());
  const int E = a.dtype == ZP_F32 ? 4 : 8, KE = 8 * E;
  const bool smallc = a.Cin < KE;
  ZP_CHECK_ARG(a.Cin > 0 && a.Cin % E == 0 && (smallc || a.Cin % KE == 0),
               "zp_conv2d: Cin %d must be a multiple of %d (or < %d and a multiple of %d)", a.Cin, KE, KE, E);
  ZP_CHECK_ARG(a.ldx >= a.cx0 + a.Cin && a.cx0 % E == 0 && a.ldx % E == 0, "zp_conv2d: bad ldx/cx0");
  ZP_CHECK_ARG(a.k_pad % KE == 0, "zp_conv2d: k_pad %d not a multiple of %d", a.k_pad, KE);
  ZP_CHECK_ARG(a.w_rows % conv_tc(a) == 0 && a.w_rows >= a.Cout, "zp_conv2d: w_rows %d", a.w_rows);
  ZP_CHECK_ARG((a.out_mode >= 0 && a.out_mode <= 2) || ((a.out_mode == ZP_OUT_NHWC_X3 || a.out_mode == ZP_OUT_NHWC_H2) && a.dtype == ZP_F32 && !a.stats),
               "zp_conv2d: out_mode %d", a.out_mode);
  ZP_CHECK_ARG(!(a.stats || a.bnr_part) || (!a.res && !a.relu && a.out_mode != ZP_OUT_HEAD_NCHW && !a.sub[0].scale &&
                            !a.sub[0].shift),
               "zp_conv2d: stats are taken on the raw conv output (no scale/shift/residual/relu/head)");
  for (int s = 0; s < a.nsub; ++s) {
    const zp_conv_sub& S = a.sub[s];
    ZP_CHECK_ARG(S.w && S.y, "zp_conv2d: sub %d null w/y", s);
    ZP_CHECK_ARG(!a.bnr_part || (!S.scale && !S.shift), "zp_conv2d: bnr_* with a scale / shift epilogue");
    ZP_CHECK_ARG(S.ntaps >= 1 && S.ntaps <= ZP_MAX_TAPS, "zp_conv2d: ntaps %d", S.ntaps);
    if (smallc) {
      ZP_CHECK_ARG(S.kw > 0 && (long)S.ntaps * a.Cin <= a.k_pad, "zp_conv2d: small-Cin taps/k_pad");
    } else {
      ZP_CHECK_ARG((long)S.ntaps * a.Cin <= a.k_pad, "zp_conv2d: k_pad %d < ntaps*Cin", a.k_pad);
    }
    if (a.out_mode != ZP_OUT_HEAD_NCHW) {
      ZP_CHECK_ARG(S.ldy >= S.cy0 + a.Cout && S.cy0 % 4 == 0 && S.ldy % 4 == 0, "zp_conv2d: bad ldy/cy0");
    } else {
      ZP_CHECK_ARG(S.y2 || a.Cout == 1, "zp_conv2d: head needs y2");
    }
  }
  if (a.res) ZP_CHECK_ARG(a.ldr >= a.cr0 + a.Cout && a.cr0 % 4 == 0, "zp_conv2d: bad residual ld");
  conv_taps tg{};
  {
    const long long xb = (long long)a.N * a.IH * a.IW * a.ldx * (E == 8 ? 2 : 4);
    const long long wb = (long long)a.w_rows * a.k_pad * (E == 8 ? 2 : 4);
    ZP_CHECK_ARG(xb < (1ll << 31) && wb < (1ll << 31),
                 "zp_conv2d: input (%lld B) / weights (%lld B) must stay below 2 GiB per launch (split the batch)",
                 xb, wb);
    tg.x_bytes = (unsigned)xb;
    tg.rflag = a.out_mode == ZP_OUT_NHWC_H2 ? range_flag() : nullptr;
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
      if (smallc) continue;  // the small-Cin path decodes (kw, dil, pad) per lane instead
      bool grid = ny * nx == S.ntaps && ny <= 32 && nx <= 32;
      for (int t = 0; grid && t < S.ntaps; ++t)
        grid = S.ty[t] == tg.ty0[s] + (t / nx) * tg.dty[s] && S.tx[t] == tg.tx0[s] + (t % nx) * tg.dtx[s];
      ZP_CHECK_ARG(grid, "zp_conv2d: sub %d taps must form a (row x column) grid of at most 32 x 32, rows outer", s);
    }
  }
  // narrow-K 1x1 convs with a wide output (k_conv1x1n: the head's data gradient in training)
  {
    if (conv1x1n_ok(a)) {
      const long groups = ((long)a.N * a.GH * a.GW + 15) / 16;
      const long want = (groups + 3) / 4;
      const int blocks = (int)(want < 2L * num_cus() ? want : 2L * num_cus());  // (~200 VGPRs: 2 blocks per CU)
#define ZP_C1N(NCB)                                                                                           \
  case NCB:                                                                                                   \
    if (a.dtype == ZP_F16) hipLaunchKernelGGL((k_conv1x1n<f16_t, NCB>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, a); \
    else hipLaunchKernelGGL((k_conv1x1n<bf16_t, NCB>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, a);    \
    break;
      switch (a.Cout / 16) { ZP_C1N(4) ZP_C1N(8) ZP_C1N(12) ZP_C1N(16) ZP_C1N(20) ZP_C1N(24) }
#undef ZP_C1N
      ZP_LAUNCH_CHECK("zp_conv2d 1x1 narrow-K");
      return ZP_OK;
    }
  }
  // tiny-M 1x1 convs (the ASPP image-pool conv): one wave per (grid point, 16 output channels)
  {
    const long mpix = (long)a.N * a.GH * a.GW;
    const zp_conv_sub& S = a.sub[0];
    if (E == 8 && !smallc && mpix <= 64 && a.nsub == 1 && S.ntaps == 1 && !a.stats && !a.bnr_part && !a.res &&
        a.out_mode == ZP_OUT_NHWC && a.w_rows >= ((a.Cout + 63) / 64) * 64 && (conv_flags() & 1024) != 0) {
      const dim3 grid((a.Cout + 63) / 64, (unsigned)mpix);
      if (a.dtype == ZP_F16) hipLaunchKernelGGL(k_conv_smallm<f16_t>, grid, dim3(256), 0, (hipStream_t)stream, a);
      else hipLaunchKernelGGL(k_conv_smallm<bf16_t>, grid, dim3(256), 0, (hipStream_t)stream, a);
      ZP_LAUNCH_CHECK("zp_conv2d small-M");
      return ZP_OK;
    }
  }
  const int tc = conv_tc(a);
  const int gx = zp_conv2d_grid(&a), gy = ceil_div(a.Cout, tc);
  hipStream_t st = (hipStream_t)stream;
  strip_geo sg{};
  if (tc <= 128 && strip_eligible(a, &sg)) {
    sg.x_bytes = tg.x_bytes;
    sg.w_bytes = tg.w_bytes[0];
    const int sgx = (int)(((long)a.N * a.GH * a.GW) / 256);
    const dim3 grid(sgx, gy, 1);
    const int fl0 = conv_flags();
    // train-mode statistics: the caller sized the partials buffer with zp_conv2d_stat_parts; the
    // launch must emit exactly that many parts (NWP = 4 wave-halves per 256-pixel tile)
    ZP_CHECK_ARG(!a.bnr_part || (fl0 & 64) || 4 * sgx == zp_conv2d_stat_parts(&a), "zp_conv2d: strip bnr parts");
    ZP_CHECK_ARG(!a.stats || ((fl0 & 64) ? 1 : 4) * sgx == zp_conv2d_stat_parts(&a),
                 "zp_conv2d: strip launch emits %d stat parts, zp_conv2d_stat_parts says %d", 4 * sgx,
                 zp_conv2d_stat_parts(&a));
    const int fl = conv_flags();
    if (fl & 64) {  // k_conv_strip2 (lean main loop); flags & 32: strip DMA spread over the group
      const zp_head_args H0{};
#define ZP_STRIP2(T, WC)                                                                               \
  if (fl & 256) hipLaunchKernelGGL((k_conv_strip2<T, WC, 5, 2>), grid, dim3(512), 0, st, a, sg, fl, H0); \
  else if (fl & 32) hipLaunchKernelGGL((k_conv_strip2<T, WC, 5, 1>), grid, dim3(512), 0, st, a, sg, fl, H0); \
  else hipLaunchKernelGGL((k_conv_strip2<T, WC, 5, 0>), grid, dim3(512), 0, st, a, sg, fl, H0);
#define ZP_STRIP2B(T, WC)                                                                              \
  if (fl & 256) hipLaunchKernelGGL((k_conv_strip2<T, WC, 5, 2, false, true>), grid, dim3(512), 0, st, a, sg, fl, H0); \
  else if (fl & 32) hipLaunchKernelGGL((k_conv_strip2<T, WC, 5, 1, false, true>), grid, dim3(512), 0, st, a, sg, fl, H0); \
  else hipLaunchKernelGGL((k_conv_strip2<T, WC, 5, 0, false, true>), grid, dim3(512), 0, st, a, sg, fl, H0);
      if (a.bnr_part) {  // (bf16 only: zp_conv2d's bnr check)
        if (tc == 64) { ZP_STRIP2B(bf16_t, 2) } else { ZP_STRIP2B(bf16_t, 4) }
      } else if (a.dtype == ZP_F16) {
        if (tc == 64) { ZP_STRIP2(f16_t, 2) } else { ZP_STRIP2(f16_t, 4) }
      } else {
        if (tc == 64) { ZP_STRIP2(bf16_t, 2) } else { ZP_STRIP2(bf16_t, 4) }
      }
#undef ZP_STRIP2
#undef ZP_STRIP2B
    } else if (a.dtype == ZP_F16) {
      if (tc == 64) hipLaunchKernelGGL((k_conv_strip<f16_t, 2, 3, 5>), grid, dim3(512), 0, st, a, sg, fl);
      else hipLaunchKernelGGL((k_conv_strip<f16_t, 4, 3, 5>), grid, dim3(512), 0, st, a, sg, fl);
    } else {
      if (tc == 64) hipLaunchKernelGGL((k_conv_strip<bf16_t, 2, 3, 5>), grid, dim3(512), 0, st, a, sg, fl);
      else hipLaunchKernelGGL((k_conv_strip<bf16_t, 4, 3, 5>), grid, dim3(512), 0, st, a, sg, fl);
    }
    ZP_LAUNCH_CHECK("zp_conv2d strip");
    return ZP_OK;
  }
  quad_geo qg{};
  if (quad_plan(a, &qg)) {
    qg.x_bytes = tg.x_bytes;
    qg.w_bytes = tg.w_bytes[0];
    const int qgx = (int)(((long)a.N * a.GH * a.GW) / 256);
    const dim3 grid(qgx, gy, 1);
    ZP_CHECK_ARG(!(a.stats || a.bnr_part) || 4 * qgx == zp_conv2d_stat_parts(&a),
                 "zp_conv2d: quad launch emits %d stat parts, zp_conv2d_stat_parts says %d", 4 * qgx,
                 zp_conv2d_stat_parts(&a));
    const int fl = conv_flags();
#define ZP_QUAD(T)                                                                             \
  if (a.GW == 32 && (fl & 256)) hipLaunchKernelGGL((k_conv_quad<T, 32, true>), grid, dim3(512), 0, st, a, qg, fl); \
  else if (a.GW == 32) hipLaunchKernelGGL((k_conv_quad<T, 32, false>), grid, dim3(512), 0, st, a, qg, fl); \
  else if (fl & 256) hipLaunchKernelGGL((k_conv_quad<T, 64, true>), grid, dim3(512), 0, st, a, qg, fl); \
  else hipLaunchKernelGGL((k_conv_quad<T, 64, false>), grid, dim3(512), 0, st, a, qg, fl);
    if (a.dtype == ZP_F16) { ZP_QUAD(f16_t) } else { ZP_QUAD(bf16_t) }
#undef ZP_QUAD
    ZP_LAUNCH_CHECK("zp_conv2d quad");
    return ZP_OK;
  }
  const int nwp = conv_tp(a) / 64;
  const int stages = conv_stages(a, tc);
  {
    ZP_CHECK_ARG(!(a.stats || a.bnr_part) || gx * a.nsub == zp_conv2d_stat_parts(&a),
                 "zp_conv2d: launch emits %d stat parts, zp_conv2d_stat_parts says %d", gx * a.nsub,
                 zp_conv2d_stat_parts(&a));
  }
#define ZP_DISPATCH_ST(T, WC, NWP, ST)                                   \
  if (smallc) launch_conv<T, WC, NWP, ST, true>(a, tg, gx, gy, st);      \
  else launch_conv<T, WC, NWP, ST, false>(a, tg, gx, gy, st);
#define ZP_DISPATCH_NWP(T, WC, NWP)                                      \
  if (stages == 3) { ZP_DISPATCH_ST(T, WC, NWP, 3) } else { ZP_DISPATCH_ST(T, WC, NWP, 2) }
#define ZP_DISPATCH(T)                                                   \
  if (tc == 256) {                                                       \
    launch_conv_tc256<T>(a, tg, gx, gy, st);                             \
  } else if (tc == 128) {                                                \
    if (nwp == 4) { ZP_DISPATCH_NWP(T, 4, 4) } else { ZP_DISPATCH_NWP(T, 4, 2) } \
  } else if (tc == 64) {                                                 \
    if (nwp == 4) { ZP_DISPATCH_NWP(T, 2, 4) } else { ZP_DISPATCH_NWP(T, 2, 2) } \
  } else {                                                               \
    ZP_DISPATCH_NWP(T, 1, 2)                                             \
  }
  if (a.dtype == ZP_BF16) {
    ZP_DISPATCH(bf16_t)
  } else if (a.dtype == ZP_F16) {
    ZP_DISPATCH(f16_t)
  } else {
    ZP_DISPATCH(float)
  }
#undef ZP_DISPATCH_ST
#undef ZP_DISPATCH_NWP
#undef ZP_DISPATCH
  ZP_LAUNCH_CHECK("zp_conv2d");
  return ZP_OK;
}

static void wgrad_plan(const zp_wgrad_args& a, int* splits, int* col_tiles, int* cols_max, int* pix_per) {
  long M = (long)a.N * a.GH * a.GW;
  int cm = 0;
  for (int s = 0; s < a.nsub; ++s) cm = cm > a.sub[s].ntaps * a.Cin ? cm : a.sub[s].ntaps * a.Cin;
  int ct = ceil_div(cm, WG_TILE);
  int tiles = ct * ceil_div(a.Cout, WG_TILE) * a.nsub;
  const int KP = a.dtype == ZP_BF16 ? 32 : 16;
  // aim for >= 1024 workgroups, but keep >= 8 K steps per split
  long sp = (1024 + tiles - 1) / tiles;
  long maxsp = M / (8 * KP);
  if (maxsp < 1) maxsp = 1;
  if (sp > maxsp) sp = maxsp;
  if (sp > 256) sp = 256;
  long pp = (M + sp - 1) / sp;
  pp = (pp + KP - 1) / KP * KP;
  sp = (M + pp - 1) / pp;
  *splits = (int)sp;
  *col_tiles = ct;
  *cols_max = cm;
  *pix_per = (int)pp;
}

// bf16: the LDS-DMA kernel (k_wgrad_lds).  Tile 128 co x 256 col (3 stages), or 64 x 512 (2 stages)
// when Cout <= 64; KP 64.  One workgroup per CU (144 KB LDS): aim for ~2 workgroups per CU
// over the launch, each with >= 16 K steps.  ZP_WGRAD=0 selects the register-staged k_wgrad.
static bool wgrad_lds(const zp_wgrad_args& a) {
  static const int v = getenv("ZP_WGRAD") ? env_int("ZP_WGRAD") : 1;
  return a.dtype == ZP_BF16 && v != 0;
}
// tile: 0 = 64 co x 512 col (Cout <= 64), 1 = 128 x 256, 2 = 256 x 256 (Cout >= 256: fewer staged
// bytes per FLOP -- the L2 -> LDS stream, not the MFMA, bounds this kernel).  Round 5: a k_wgrad2
// launch whose 256 x 256 plan would give each split under 2048 pixels takes 128 x 256 instead --
// few tiles (a 3x3 256 -> 256 at 32 x 32 has 9) mean ~28 splits, and each split writes a 256 KB f32
// partial slab (64 MB per launch, re-read by k_wgrad_reduce) for 1216 pixels of MFMA work:
// measured 739 -> 679 us over layer4's 11 wgrads, the 1 x 1 convs 43 -> 32 us; the 128 x 128
// decoder / layer5 wgrads (18724 / 4681 pixels per split) stay on 256 x 256 (1116 vs 1328 us).
// ZP_WGRAD_BIG=0: always 128 x 256; 2: always 256 x 256 (A/B)
static bool wgrad2_eligible(const zp_wgrad_args& a);
static int num_cus();
extern int g_wgrad2_rounds_v;
static int wgrad_cfg(const zp_wgrad_args& a) {
  static const int big = getenv("ZP_WGRAD_BIG") ? env_int("ZP_WGRAD_BIG") : 1;
  if (a.Cout <= 64) return 0;
  if (a.Cout < 256 || !big) return 1;
  // (round 6) a Cout the 256-row tiles would pad by more than the 128-row ones (320: 512 against
  // 384 rows -- the ConvT weight gradient as the stride-2 conv over dy) takes 128 x 256: measured
  // 276 -> 261 us for up2's ConvT (tools/wgrad_ab.py, profiles/r06_conv_ablations.md)
  if (big == 1 && (a.Cout + 255) / 256 * 256 > (a.Cout + 127) / 128 * 128) return 1;
  if (big == 1 && wgrad2_eligible(a)) {
    long M = (long)a.N * a.GH * a.GW;
    int cm = 0;
    for (int s = 0; s < a.nsub; ++s) cm = cm > a.sub[s].ntaps * a.Cin ? cm : a.sub[s].ntaps * a.Cin;
    const long tiles = (long)ceil_div(cm, 256) * ceil_div(a.Cout, 256);
    long sp = (long)g_wgrad2_rounds_v * num_cus() / tiles;
    const long maxsp = M / (16 * 64) > 0 ? M / (16 * 64) : 1;
    sp = sp < 1 ? 1 : (sp > maxsp ? maxsp : sp);
    if (M / sp < 2048) return 1;
  }
  return 2;
}
// k_wgrad2 (lean issue path) for the common geometry -- see the kernel's header comment.
// zp_conv_tuning key 3: 0 disables it; key 4: its workgroup rounds over the CUs (default 1: fewer,
// longer workgroups than k_wgrad_lds's 1024 -- the split-K partial slabs are written and re-read
// in full -- and never a partial extra round; one round measured fastest).
static int g_wgrad2 = 1, g_wgrad2_rounds = 1, g_wgrad_lds_rounds = 1;
int g_wgrad2_rounds_v = 1;  // (g_wgrad2_rounds, read by wgrad_cfg above)
static int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}
static bool wgrad2_eligible(const zp_wgrad_args& a) {
  if (!g_wgrad2 || a.dtype != ZP_BF16 || a.nsub != 1 || a.sy != a.sx || (a.sy != 1 && a.sy != 2)) return false;
  if (a.IH != a.sy * a.GH || a.IW != a.sx * a.GW || (a.GW != 32 && a.GW != 64 && a.GW != 128)) return false;
  if (((long)a.GH * a.GW) % 64 != 0 || a.Cin % 64 != 0) return false;
  const auto& S = a.sub[0];
  return S.oys == 1 && S.oxs == 1 && S.oyo == 0 && S.oxo == 0 && S.OH == a.GH && S.OW == a.GW;
}
static void wgrad_plan_lds(const zp_wgrad_args& a, int* splits, int* col_tiles, int* cols_max, int* pix_per) {
  long M = (long)a.N * a.GH * a.GW;
  int cm = 0;
  for (int s = 0; s < a.nsub; ++s) cm = cm > a.sub[s].ntaps * a.Cin ? cm : a.sub[s].ntaps * a.Cin;
  const int cfg = wgrad_cfg(a);
  const int tco = cfg == 0 ? 64 : (cfg == 1 ? 128 : 256), tcol = cfg == 0 ? 512 : 256, KP = 64;
  int ct = ceil_div(cm, tcol);
  int tiles = ct * ceil_div(a.Cout, tco) * a.nsub;
  // target workgroup count: 1024 (R34 bs 32 train step 19.93 -> 19.71 ms vs 512; 2048: 19.81).
  // ZP_WGRAD_WG overrides for sweeps (read once, so the workspace size query agrees)
  static const int target_lds = getenv("ZP_WGRAD_WG") ? env_int("ZP_WGRAD_WG") : 1024;
  const bool lean = wgrad2_eligible(a);
  // k_wgrad2: workgroups (one per CU at a time: 96-144 KB of LDS) in whole rounds over the CUs --
  // a grid one workgroup past a round costs a full extra workgroup lifetime (513 vs 512 ran 1.6x)
  // k_wgrad_lds: the same whole-round plan when zp_conv_tuning key 5 > 0, else ~target_lds workgroups
  long sp = lean ? (long)g_wgrad2_rounds * num_cus() / tiles
                 : g_wgrad_lds_rounds > 0 ? (long)g_wgrad_lds_rounds * num_cus() / tiles
                                          : (target_lds + tiles - 1) / tiles;
  if (sp < 1) sp = 1;
  long maxsp = M / (16 * KP);
  if (maxsp < 1) maxsp = 1;
  if (sp > maxsp) sp = maxsp;
  if (sp > 256) sp = 256;
  long pp = (M + sp - 1) / sp;
  pp = (pp + KP - 1) / KP * KP;
  sp = (M + pp - 1) / pp;  // never more than requested: pp only grew
  // k_wgrad_lds: pad the split count so the launch is a multiple of 8 workgroups (its XCD-aware
  // order needs it); padding splits have an empty pixel range and write zero partials
  if (!lean && g_wgrad_lds_rounds <= 0)
    while ((sp * tiles) % 8) ++sp;
  *splits = (int)sp;
  *col_tiles = ct;
  *cols_max = cm;
  *pix_per = (int)pp;
}

extern "C" long long zp_conv2d_wgrad_ws_bytes(const zp_wgrad_args* a) {
  if (!a || a->nsub < 1 || a->nsub > ZP_MAX_SUB) return -1;
  int sp, ct, cm, pp;
  if (wgrad_lds(*a)) wgrad_plan_lds(*a, &sp, &ct, &cm, &pp);
  else wgrad_plan(*a, &sp, &ct, &cm, &pp);
  return (long long)sp * a->nsub * a->Cout * (long long)cm * 4;
}

extern "C" int zp_conv2d_wgrad(const zp_wgrad_args* ap, void* ws, void* stream) {
  ZP_CHECK_ARG(ap && ws, "zp_conv2d_wgrad: null args/workspace");
  const zp_wgrad_args& a = *ap;
  ZP_CHECK_ARG(a.dtype == ZP_F32 || a.dtype == ZP_BF16, "zp_conv2d_wgrad: dtype");
  ZP_CHECK_ARG(a.nsub >= 1 && a.nsub <= ZP_MAX_SUB && a.dw && a.x, "zp_conv2d_wgrad: bad args");
  const int E = a.dtype == ZP_BF16 ? 8 : 4;
  ZP_CHECK_ARG(a.Cin % E == 0 && a.cx0 % E == 0 && a.ldx % E == 0, "zp_conv2d_wgrad: Cin/cx0/ldx alignment");
  ZP_CHECK_ARG(a.Cw >= 1 && a.Cw <= a.Cin, "zp_conv2d_wgrad: Cw");
  for (int s = 0; s < a.nsub; ++s) {
    ZP_CHECK_ARG(a.sub[s].dy && a.sub[s].ntaps >= 1 && a.sub[s].ntaps <= ZP_MAX_TAPS, "zp_conv2d_wgrad: sub %d", s);
    ZP_CHECK_ARG(a.sub[s].cdy0 % E == 0 && a.sub[s].lddy % E == 0 &&
                 a.sub[s].lddy >= a.sub[s].cdy0 + ((a.Cout + E - 1) / E) * E,
                 "zp_conv2d_wgrad: dy ld must cover Cout rounded to %d", E);
  }
  int sp, ct, cm, pp;
  hipStream_t st = (hipStream_t)stream;
  if (wgrad_lds(a)) {
    wgrad_plan_lds(a, &sp, &ct, &cm, &pp);
    wg_bounds wb{};
    const long long xb = (long long)a.N * a.IH * a.IW * a.ldx * 2;
    ZP_CHECK_ARG(xb < (1ll << 31), "zp_conv2d_wgrad: input %lld B must stay below 2 GiB (split the batch)", xb);
    wb.x_bytes = (unsigned)xb;
    for (int s = 0; s < a.nsub; ++s) {
      const long long db = (long long)a.N * a.sub[s].OH * a.sub[s].OW * a.sub[s].lddy * 2;
      ZP_CHECK_ARG(db < (1ll << 31), "zp_conv2d_wgrad: dy %lld B must stay below 2 GiB", db);
      wb.dy_bytes[s] = (unsigned)db;
    }
    const int cfg = wgrad_cfg(a);
    if (wgrad2_eligible(a)) {
      const int tiles = ct * ceil_div(a.Cout, cfg == 0 ? 64 : (cfg == 1 ? 128 : 256));
      if (cfg == 0)
        hipLaunchKernelGGL((k_wgrad2<1, 8, 2, 1>), dim3(sp * tiles), dim3(512), 0, st, a, (float*)ws, pp, ct, tiles, cm, wb);
      else if (cfg == 1)
        hipLaunchKernelGGL((k_wgrad2<2, 4, 3, 1>), dim3(sp * tiles), dim3(512), 0, st, a, (float*)ws, pp, ct, tiles, cm, wb);
      else
        hipLaunchKernelGGL((k_wgrad2<4, 4, 2, 2>), dim3(sp * tiles), dim3(512), 0, st, a, (float*)ws, pp, ct, tiles, cm, wb);
    } else if (cfg == 0) {
      const int tiles = ct * ceil_div(a.Cout, 64);
      hipLaunchKernelGGL((k_wgrad_lds<64, 1, 8, 2, 1>), dim3(sp * a.nsub * tiles), dim3(512), 0, st, a, (float*)ws,
                         pp, ct, tiles, cm, wb);
    } else if (cfg == 1) {
      const int tiles = ct * ceil_div(a.Cout, 128);
      hipLaunchKernelGGL((k_wgrad_lds<64, 2, 4, 3, 1>), dim3(sp * a.nsub * tiles), dim3(512), 0, st, a, (float*)ws,
                         pp, ct, tiles, cm, wb);
    } else {
      const int tiles = ct * ceil_div(a.Cout, 256);
      hipLaunchKernelGGL((k_wgrad_lds<64, 4, 4, 2, 2>), dim3(sp * a.nsub * tiles), dim3(512), 0, st, a, (float*)ws,
                         pp, ct, tiles, cm, wb);
    }
  } else {
    wgrad_plan(a, &sp, &ct, &cm, &pp);
    dim3 grid(sp, ct * ceil_div(a.Cout, WG_TILE), a.nsub);
    if (a.dtype == ZP_BF16)
      hipLaunchKernelGGL(k_wgrad<bf16_t>, grid, dim3(256), 0, st, a, (float*)ws, pp, ct, cm);
    else
      hipLaunchKernelGGL(k_wgrad<float>, grid, dim3(256), 0, st, a, (float*)ws, pp, ct, cm);
  }
  ZP_LAUNCH_CHECK("zp_conv2d_wgrad");
  long tot = (long)a.Cout * cm;
  int rb = (int)((tot + 255) / 256);
  if (rb > 4096) rb = 4096;
  hipLaunchKernelGGL(k_wgrad_reduce, dim3(rb, a.nsub), dim3(256), 0, st, a, (const float*)ws, sp, cm);
  ZP_LAUNCH_CHECK("zp_conv2d_wgrad reduce");
  return ZP_OK;
}

extern "C" int zp_conv2d_stat_parts(const zp_conv_args* a) {
  if (!a) return 0;
  if (a->dtype == ZP_F32X3 || a->dtype == ZP_F32H2) return (conv_tp(*a) / 64) * zp_conv2d_grid(a) * a->nsub;
  // round 5: k_conv_strip2, k_conv_quad and k_conv merge their wave halves in LDS -- one part per tile
  // (k_conv_quad: per tile and phase); k_conv_strip (flags & 64 off) keeps one per wave half
  if (conv_tc(*a) <= 128 && strip_eligible(*a, nullptr))
    return (int)(((long)a->N * a->GH * a->GW) / 256) * ((conv_flags() & 64) ? 1 : 4);
  if (quad_plan(*a, nullptr)) return 4 * (int)(((long)a->N * a->GH * a->GW) / 256);
  return zp_conv2d_grid(a) * a->nsub;
}

extern "C" int zp_conv2d_bnr_parts(const zp_conv_args* a) {
  if (!a) return 0;
  // k_conv_strip2 sums its wave halves in LDS: one part per 256-pixel tile
  if (a->dtype != ZP_F32 && conv_tc(*a) <= 128 && strip_eligible(*a, nullptr) && (conv_flags() & 64))
    return (int)(((long)a->N * a->GH * a->GW) / 256);
  return zp_conv2d_stat_parts(a);
}

// the 16-bit fused head: a 3x3 stride-1 conv on the 128-channel strip tile (k_conv_strip2, two cout
// tiles for Cout 256)
static bool head16_ok(const zp_conv_args& a) {
  if ((a.dtype != ZP_BF16 && a.dtype != ZP_F16) || a.nsub != 1 || a.Cout != 256 || a.out_mode != ZP_OUT_NHWC ||
      a.stats || !(conv_flags() & 64))
    return false;
  if (a.res && (a.ldr % 8 != 0 || a.cr0 % 8 != 0)) return false;
  return strip_eligible(a, nullptr) && conv_tc(a) == 128;
}

extern "C" int zp_conv2d_head_ok(const zp_conv_args* a) {
  if (!a) return 0;
  if (a->dtype == ZP_BF16 || a->dtype == ZP_F16) return head16_ok(*a);
  return a->dtype == ZP_F32H2 && a->nsub == 1 && a->Cout == 256 && a->out_mode == ZP_OUT_NHWC &&
         conv3_tc(*a) == 256 && conv3w_tp_head(*a) == 256 && conv3w_splitk(*a) == 1;
}

extern "C" long long zp_conv2d_head_ws(const zp_conv_args* a) {
  if (!a || !(a->dtype == ZP_BF16 || a->dtype == ZP_F16)) return 0;
  return 2LL * 32 * (long long)a->N * a->GH * a->GW * 4;
}

extern "C" int zp_conv2d_head(const zp_conv_args* a, const zp_head_args* h, void* stream) {
  ZP_CHECK_ARG(a && h, "zp_conv2d_head: null args");
  ZP_CHECK_ARG(zp_conv2d_head_ok(a), "zp_conv2d_head: not a fused-head geometry (zp_conv2d_head_ok)");
  if (a->dtype == ZP_F32H2) return conv3_launch(*a, (hipStream_t)stream, conv_flags(), h);
  // ZP_BF16 / ZP_F16: the strip kernel with the head epilogue, then the cout tiles' combine
  const zp_conv_args& A = *a;
  ZP_CHECK_ARG(h->w && h->mask && (h->code || h->cout == 1) && h->cout >= 1 && h->cout <= 32 && h->ws,
               "zp_conv2d_head: bad head (16-bit: needs ws, zp_conv2d_head_ws bytes)");
  ZP_CHECK_ARG(h->C2 >= 0 && h->C2 % 32 == 0 && h->k_pad % 8 == 0 && h->k_pad >= A.Cout + h->C2,
               "zp_conv2d_head: C2 %d / k_pad %d", h->C2, h->k_pad);
  ZP_CHECK_ARG(h->C2 == 0 || (h->x2 && h->ldx2 % 8 == 0 && h->cx20 % 8 == 0 && h->ldx2 >= h->cx20 + h->C2),
               "zp_conv2d_head: x2 layout");
  ZP_CHECK_ARG(A.Cin > 0 && A.Cin % 64 == 0 && A.ldx >= A.cx0 + A.Cin && A.cx0 % 8 == 0 && A.ldx % 8 == 0 &&
                   A.k_pad % 64 == 0 && A.w_rows % 128 == 0 && A.w_rows >= A.Cout && A.sub[0].w && A.sub[0].ntaps == 9,
               "zp_conv2d_head: conv operands");
  ZP_CHECK_ARG(A.sub[0].OH == A.GH && A.sub[0].OW == A.GW, "zp_conv2d_head: output grid");
  const long long xb = (long long)A.N * A.IH * A.IW * A.ldx * 2, wb = (long long)A.w_rows * A.k_pad * 2;
  ZP_CHECK_ARG(xb < (1ll << 31) && wb < (1ll << 31), "zp_conv2d_head: input / weights must stay below 2 GiB");
  strip_geo sg{};
  ZP_CHECK_ARG(strip_eligible(A, &sg), "zp_conv2d_head: not a strip geometry");
  sg.x_bytes = (unsigned)xb;
  sg.w_bytes = (unsigned)wb;
  hipStream_t st = (hipStream_t)stream;
  const int fl = conv_flags();
  const dim3 grid((unsigned)(((long)A.N * A.GH * A.GW) / 256), 2u, 1u);
  if (A.dtype == ZP_F16) hipLaunchKernelGGL((k_conv_strip2<f16_t, 4, 5, 2, true>), grid, dim3(512), 0, st, A, sg, fl, *h);
  else hipLaunchKernelGGL((k_conv_strip2<bf16_t, 4, 5, 2, true>), grid, dim3(512), 0, st, A, sg, fl, *h);
  ZP_LAUNCH_CHECK("zp_conv2d_head (16-bit conv + head partials)");
  const int M = A.N * A.GH * A.GW;
  hipLaunchKernelGGL(k_head_combine16, dim3((M + 255) / 256), dim3(256), 0, st, h->ws, M, A.GH * A.GW, h->cout, h->bias,
                     h->mask, h->code);
  ZP_LAUNCH_CHECK("zp_conv2d_head (combine)");
  return ZP_OK;
}

/* launch configuration zp_conv2d picks for these args (for kernel labels in reports) */
extern "C" int zp_conv2d_config(const zp_conv_args* a, int* tc, int* tp, int* stages, int* variant) {
  ZP_CHECK_ARG(a && tc && tp && stages && variant, "zp_conv2d_config: null args");
  *tc = conv_tc(*a);
  *tp = conv_tp(*a);
  *stages = *tc == 256 ? 2 : conv_stages(*a, *tc);
  *variant = (a->dtype == ZP_F32X3 || a->dtype == ZP_F32H2) ? (*tc == 256 ? 6 : conv3_nsplit(*a) == 1 && conv3_strip_ok(*a, *tc) ? 5 : 4) : conv1x1n_ok(*a) ? 7 : quad_plan(*a, nullptr) ? 3 : *tc <= 128 && strip_eligible(*a, nullptr) ? ((conv_flags() & 64) ? 2 : 1) : 0;
  return ZP_OK;
}

/* runtime tuning knobs (tests / sweeps).  key 0: minimum workgroups for the 256-channel conv tile
 * (default 1024); key 1: conv schedule flags (-1 = ZP_CONV_FLAGS / default); key 2: 64-channel
 * layers on the strip kernel (default 1); key 3: k_wgrad2 (default 1); key 4: k_wgrad2's
 * workgroup rounds over the CUs (default 1); key 5: k_wgrad_lds's workgroup rounds (default 1; 0 =
 * the older ~1024-workgroup target padded to a multiple of 8); key 6: the fewest workgroups
 * k_conv_quad runs with (default 256); key 7: split-fp32 strip kernel k_conv3s (0 off, 1 the
 * 64-channel tiles, 2 also the 128-channel tiles; -1 = ZP_CONV3_STRIP / default 1); key 8: the
 * fewest workgroups a split-fp32 launch runs 128-channel tiles with (fewer: 64-channel tiles);
 * keys 10-12: the wide two-plane tile (on / fewest workgroups / split-K); key 13: its accumulation
 * form (0 flushed correction accumulator, 1 one scaled accumulator, 2 per-step partial sums, the
 * default; -1 = ZP_CONV3W_ACC); key 14: its 256 x 128 pixel tile (0 off, 1 on; -1 = ZP_CONV3W_TP128);
 * key 15: zp_bn_train_finalize's statistics merge in one launch (1, default) or two (0; -1 = ZP_BN_FUSED);
 * key 16: k_conv3's multi-sub launches (the merged ASPP) with a tile's subs adjacent on one XCD (1) or
 * the sub slowest (0, default: measured faster; -1 = ZP_CONV3_SUBINT); key 17: k_conv3w's multi-sub
 * launches (the ConvT phases) with a pixel tile's phases adjacent on one XCD (1) or phase by phase,
 * longest first (0, default: measured faster; -1 = ZP_CONV3W_SUBINT); key 18: k_conv3w's 256 x 256 tile
 * on v_mfma_f32_32x32x16_f16 (k_conv3w32; 1) or 16 x 16 x 32 (0, default; -1 = ZP_CONV3W_MF32);
 * key 19: ring depth (2, 3, 4) of k_conv3's register-pipelined two-plane 64-channel tile (-1 =
 * ZP_CONV3_PIPE_ST or 2, the default: measured fastest); key 20: persistent workgroups per CU of the two-plane stem (1 or 2; -1 = ZP_STEM_WGS or 1); key 21: the wide strip tile's next-step pixel
 * fragments read before the step's barrier (1) or after it (0; -1 = ZP_CONV3W_PFB or 1).
 * Returns the previous value. */
/* split-fp32 split-K workspace: bytes of f32 slices zp_conv2d uses for these args when a.stats
 * points to that many (0: the launch is not split) */
extern "C" long long zp_conv2d_split_ws(const zp_conv_args* a) {
  if (!a || (a->dtype != ZP_F32X3 && a->dtype != ZP_F32H2)) return 0;
  const int ns = conv3_nsplit(*a);
  return ns > 1 ? (long long)ns * a->nsub * a->N * a->GH * a->GW * a->Cout * 4 : 0;
}

extern "C" int zp_conv_tuning(int key, int value) {
  if (key == 0) {
    const int old = g_tc256_min_blocks;
    g_tc256_min_blocks = value;
    return old;
  }
  if (key == 1) {
    const int old = g_conv_flags;
    g_conv_flags = value;
    return old;
  }
  if (key == 2) {
    const int old = g_strip_c64;
    g_strip_c64 = value;
    return old;
  }
  if (key == 3) {
    const int old = g_wgrad2;
    g_wgrad2 = value;
    return old;
  }
  if (key == 5) {
    const int old = g_wgrad_lds_rounds;
    g_wgrad_lds_rounds = value >= 0 ? value : 1;
    return old;
  }
  if (key == 6) {
    const int old = g_quad_min_blocks;
    g_quad_min_blocks = value;
    return old;
  }
  if (key == 7) return conv3_strip_mode(value);
  if (key == 8) return conv3_min_blocks(value);
  if (key == 9) return conv3_splitk_mode(value);
  if (key == 10) return conv3w_mode(value);
  if (key == 11) return conv3w_min_blocks(value);
  if (key == 12) return conv3w_splitk_mode(value);
  if (key == 13) return conv3w_acc_mode(value);
  if (key == 14) return conv3w_tp128_mode(value);
  if (key == 15) return bn_fused_mode(value);
  if (key == 16) return conv3_subint_mode(value);
  if (key == 17) return conv3w_subint_mode(value);
  if (key == 18) return conv3w_mf32_mode(value);
  if (key == 19) return conv3_pipe_st_mode(value);
  if (key == 20) return stem_wgs_mode(value);
  if (key == 21) return conv3w_pfb_mode(value);
  if (key == 4) {
    const int old = g_wgrad2_rounds;
    g_wgrad2_rounds = value > 0 ? value : 1;
    g_wgrad2_rounds_v = g_wgrad2_rounds;
    return old;
  }
  return -1;
}
