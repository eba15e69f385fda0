// k_conv3w32: k_conv3w's 256 x 256 two-plane tile on v_mfma_f32_32x32x16_f16 (round 6; A/B,
// zp_conv_tuning key 18).
//
// Why (DESIGN.md §4 "What bounds the two-plane kernels", profiles/r06_sq_counters.md): with two waves
// per SIMD, k_conv3w's vector issue port is ~97% busy per K step -- an MFMA holds it for 8 cycles
// (16x16x32: 8 of 16, 32x32x16: 8 of 32; MI355X_MICROARCH.md cycle constants), and the flushed
// correction accumulator adds one FMA per output element and K step.  A 32 x 32 block does the same
// MACs in half the MFMA instructions: per K step and wave 48 MFMAs instead of 96, the same 128 flush
// FMAs, the same 24 fragment reads (ds_read_b128), so the issue port drops from ~2980 to ~2210 of the
// 3072 MFMA-pipe cycles per step and SIMD.
//
// Same staging (the LDS images are k_conv3w's: 16-row x 32-element tiles, [k group][row] inside a
// tile), same DMA schedule, same numerics as k_conv3w's default (ACC_FLUSH: hi*lo', then lo'*hi into a
// fresh correction accumulator per block and K step, hi*hi into acc, acc = fma(c2, 2^-11, acc) once
// the block's step is done), the same epilogue arithmetic.  What changes:
//   - a wave owns 4 cout blocks x 2 pixel blocks of 32 x 32 (128 accumulator registers, as before);
//   - v_mfma_f32_32x32x16_f16 reads A row (lane & 31), k = (lane >> 5) * 8 .. + 7 of a K half: in the
//     16-row tile image that is tile (lane & 31) >> 4, k group 2 h + (lane >> 5), row lane & 15 -- one
//     per-lane base for A, B and both halves, the rest immediates;
//   - the K step (32 channels) is two K halves; a (cout block, half) unit streams its weight
//     fragments through a 3-slot register ring, the pixel fragments of both halves are held;
//   - epilogue: lane l holds rows 8 (i >> 2) + 4 (l >> 5) + (i & 3) of pixel l & 31 for accumulator
//     element i; v_permlane32_swap pairs, then a v_permlane16_swap, give every lane 8 consecutive output
//     channels of one pixel with 4 lanes covering a pixel's 32 channels: 16-byte stores per lane and
//     plane, 64 contiguous bytes per pixel per instruction, as k_conv3w.
// Eval forward only (NHWC output, one sub-problem or the ConvT phases, no split-K, no fused head).
#include "zp_conv_kern.h"
#include "zp_conv3.h"

namespace zp {

typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ void mma32(f32x16& acc, const uint4& a, const uint4& b) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), acc, 0, 0, 0);
}

__device__ __forceinline__ void wbarrier32() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <bool STR>
__global__ void __launch_bounds__(512) k_conv3w32(const zp_conv_args A, const conv_taps TG, const int flags) {
  constexpr int NPL = 2;
  constexpr int TC = 256, TP = 256;
  constexpr int NTW = TC / 16, NT = (TC + TP) / 16;  // 16-row tiles per plane: weights / all
  constexpr int UNITS = NPL * NT;
  constexpr int TPW = NT / 8;   // DMA tiles per wave: 2 weight + 2 activation
  constexpr int CB = 4, PB = 2;  // per wave: 4 cout blocks x 2 pixel blocks of 32 x 32
  constexpr int SPMAX = 20;
  constexpr int APL = STR ? NTW : NT;
  constexpr int ASTG = NPL * APL;
  constexpr int LDSU = STR ? 2 * ASTG + 2 * NPL * SPMAX : 2 * UNITS;
  __shared__ uint4 lds[LDSU * 64];
  static_assert(LDSU * 1024 <= 160 * 1024, "LDS");
  int tb = (int)blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid >> 2, wp = wid & 3;
  const int GHW = A.GH * A.GW;
  const int M = A.N * GHW;
  int bx = blockIdx.x, by = blockIdx.y;
  if (flags & 2) {  // XCD-aware order (k_conv3w): consecutive pixel tiles on one XCD
    const int total = gridDim.x * gridDim.y;
    const int bid = blockIdx.x + gridDim.x * blockIdx.y;
    const int lin = (total & 7) ? bid : (bid & 7) * (total >> 3) + (bid >> 3);
    bx = lin / gridDim.y;
    by = lin - bx * gridDim.y;
  }
  tb = __builtin_amdgcn_readfirstlane(tb);
  const zp_conv_sub& S = A.sub[tb];
  const int p0 = bx * TP, c0 = by * TC;
  const int CBK = A.Cin / 32;
  const int ny = TG.ny[tb], nx = TG.nx[tb], dty = TG.dty[tb], dtx = TG.dtx[tb];
  const int nK = S.ntaps * CBK;
  const int lr = lane & 15, lk = (lane >> 4) * 8;
  const unsigned psx_b = (unsigned)((long)A.N * A.IH * A.IW * A.ldx * 2);
  const unsigned psw_b = (unsigned)((long)A.w_rows * A.k_pad * 2);

  // DMA: k_conv3w's (tile t = wid + 8 k: k 0, 1 weight tiles, 2, 3 activation tiles; both planes)
  unsigned ubase[TPW], uym[TPW], uxm[TPW];
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    const int t = wid + 8 * k;
    uym[k] = uxm[k] = 0u;
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
  // STR: k_conv3w's strip pieces; sjj[J]: the strip pixel of this lane's pixel (lane & 31) of block J
  int nsp = 16, SW = 0, sh0 = 0;
  unsigned sbase[3], sym[3];
  int sjj[PB];
  if constexpr (STR) {
    const int sx0 = min(TG.tx0[tb], TG.tx0[tb] + (nx - 1) * dtx);
    sh0 = TG.tx0[tb] - sx0;
    SW = A.GW + (nx - 1) * (dtx < 0 ? -dtx : dtx);
    const int TR = TP / A.GW;
    nsp = (TR * SW + 15) >> 4;
    const int n = p0 / GHW, oy0 = (p0 - n * GHW) / A.GW;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int sp = (wid + 8 * k) * 16 + lr;
      const int r = sp / SW, c = sp - (sp / SW) * SW;
      const int ix = c + sx0, iyb = oy0 + r + TG.ty0[tb];
      unsigned ym = 0;
      for (int q = 0; q < ny; ++q) ym |= (unsigned)((unsigned)(iyb + q * dty) < (unsigned)A.IH) << q;
      sym[k] = (r < TR && (unsigned)ix < (unsigned)A.IW) ? ym : 0u;
      sbase[k] = (unsigned)(((((long)n * A.IH + iyb) * A.IW + ix) * A.ldx + A.cx0 + lk) * 2);
    }
#pragma unroll
    for (int J = 0; J < PB; ++J) {
      const int q = wp * 64 + J * 32 + (lane & 31);
      sjj[J] = (q / A.GW) * SW + q % A.GW;
    }
  }
#if defined(__HIP_DEVICE_COMPILE__)
  const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)A.x, (short)0, (int)TG.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)S.w, (short)0, (int)TG.w_bytes[tb], 0x00020000);
#endif
  int w_cb = 0, w_tyi = 0, w_txi = 0;
  const int step_x = dtx * A.ldx * 2, step_y = dty * A.IW * A.ldx * 2;
  int act_off = ((TG.ty0[tb] * A.IW + TG.tx0[tb]) * A.ldx) * 2;
  int w_koff = 0;
  const int cin2 = A.Cin * 2;
  struct DmaStep {
    unsigned voff[TPW];
    int koff;
  };
  auto prep = [&](DmaStep& d) {
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      const bool ok = (uym[k] >> w_tyi) & (uxm[k] >> w_txi) & 1u;
      d.voff[k] = k < 2 ? ubase[k] : (ok ? ubase[k] + (unsigned)act_off : 0x80000000u);
    }
    d.koff = w_koff;
    w_koff += cin2;
    act_off += step_x;
    if (++w_txi == nx) {
      w_txi = 0;
      act_off += step_y - nx * step_x;
      if (++w_tyi == ny) {
        w_tyi = 0;
        ++w_cb;
        act_off += 64 - ny * step_y;
        w_koff = w_cb * 64;
      }
    }
  };
  auto piece = [&](auto q_c, int stage, const DmaStep& d) {
    constexpr int q = decltype(q_c)::value, k = q / 2, pl = q % 2;
    if constexpr (STR && k >= 2) return;  // (the strips carry the activations)
    const int t = wid + 8 * k;
#if defined(__HIP_DEVICE_COMPILE__)
    auto* dst = (__attribute__((address_space(3))) void*)&lds[(stage * ASTG + pl * APL + t) * 64];
    if constexpr (k < 2) __builtin_amdgcn_raw_ptr_buffer_load_lds(wrsrc, dst, 16, d.voff[k], pl * psw_b + d.koff, 0, 0);
    else __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, dst, 16, d.voff[k], pl * psx_b, 0, 0);
#else
    (void)t; (void)stage; (void)d;
#endif
  };
  auto issue = [&](int stage) {
    DmaStep d;
    prep(d);
    static_for<2 * TPW>([&](auto q_c) { piece(q_c, stage, d); });
  };
  int g_cb = 0, g_tyi = 0;
  auto strip_issue = [&](int gst) {
    const unsigned goff = (unsigned)(g_tyi * step_y + g_cb * 64);
    static_for<3>([&](auto k_c) {
      constexpr int k = decltype(k_c)::value;
      const int P = wid + 8 * k;
      if (k < 2 || P < nsp) {
        const unsigned vo = ((sym[k] >> g_tyi) & 1u) ? sbase[k] + goff : 0x80000000u;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) {
          auto* dst = (__attribute__((address_space(3))) void*)&lds[(2 * ASTG + (gst * NPL + pl) * SPMAX + P) * 64];
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, dst, 16, vo, pl * psx_b, 0, 0);
        }
#else
        (void)vo;
#endif
      }
    });
    if (++g_tyi == ny) {
      g_tyi = 0;
      ++g_cb;
    }
  };
  int r_txi = 0, r_gs = 0;

  f32x16 acc[CB][PB];
#pragma unroll
  for (int i = 0; i < CB; ++i)
#pragma unroll
    for (int j = 0; j < PB; ++j) acc[i][j] = (f32x16){};

  // per-lane fragment base: tile (lane & 31) >> 4, k group (lane >> 5) (+ 2 h: immediate), row lane & 15
  const unsigned lb = (unsigned)(((lane & 31) >> 4) * 1024 + (lane >> 5) * 256 + (lane & 15) * 16);
  const unsigned abase0 = lds_addr(lds) + lb + (unsigned)(wc * 8) * 1024u;
  const unsigned bbase0 = lds_addr(lds) + lb + (unsigned)(NTW + wp * 4) * 1024u;
  const unsigned abase1 = abase0 + ASTG * 1024u, bbase1 = bbase0 + UNITS * 1024u;
  const unsigned sl0 = lds_addr(lds) + (unsigned)(2 * ASTG) * 1024u + (unsigned)(lane >> 5) * 256u;
  constexpr int NU = CB * 2;  // (cout block, K half) units per step
  f32x16 c2[PB];  // the current cout block's correction sums (this K step), flushed one unit later
#pragma unroll
  for (int J = 0; J < PB; ++J) c2[J] = (f32x16){};
  auto flush = [&](f32x16 (&a)[PB]) {  // a = fma(c2, 2^-11, a): one rounding, k_conv3w's flushed form
#pragma unroll
    for (int J = 0; J < PB; ++J) {
#pragma unroll
      for (int r = 0; r < 16; ++r) a[J][r] = __builtin_fmaf(c2[J][r], SplitF32<2>::CS, a[J][r]);
      asm volatile("" : "+v"(a[J]));
    }
  };

  auto step = [&](auto s_c, const bool more, const bool strip_now) {
    constexpr int s = decltype(s_c)::value;
    DmaStep dn;
    prep(dn);
    if (!more) {
#pragma unroll
      for (int k = 0; k < TPW; ++k) dn.voff[k] = 0x80000000u;
      dn.koff = 0;
    }
    const unsigned ab = s ? abase1 : abase0, bb = s ? bbase1 : bbase0;
    uint4 bf[NPL][PB][2];  // pixel fragments [plane][block][K half], held for the step
    uint4 af[3][NPL];      // weight fragments of a unit: a 3-slot ring
    if constexpr (STR) {
      const unsigned sb = sl0 + (unsigned)r_gs * (unsigned)(NPL * SPMAX * 1024);
      const int sh = sh0 + r_txi * dtx;
      static_for<PB>([&](auto j_c) {
        constexpr int J = decltype(j_c)::value;
        const int sp = sjj[J] + sh;
        const unsigned ad = sb + ((unsigned)(sp >> 4) << 10) + ((unsigned)(sp & 15) << 4);
        static_for<NPL>([&](auto p_c) {
          constexpr int p = decltype(p_c)::value;
          bf[p][J][0] = ds_read16<p * SPMAX * 1024>(ad);
          bf[p][J][1] = ds_read16<p * SPMAX * 1024 + 512>(ad);
        });
      });
    } else {
      static_for<NPL>([&](auto p_c) {
        constexpr int p = decltype(p_c)::value;
        static_for<PB>([&](auto j_c) {
          constexpr int J = decltype(j_c)::value;
          bf[p][J][0] = ds_read16<(p * NT + 2 * J) * 1024>(bb);
          bf[p][J][1] = ds_read16<(p * NT + 2 * J) * 1024 + 512>(bb);
        });
      });
    }
    // unit u = (cout block u >> 1, K half u & 1): A tile 2 (u >> 1) of the wave's 8, k groups 2 (u & 1) ..
    static_for<2>([&](auto q_c) {
      constexpr int q = decltype(q_c)::value;
      static_for<NPL>([&](auto p_c) {
        constexpr int p = decltype(p_c)::value;
        af[q][p] = ds_read16<(p * APL + 2 * (q >> 1)) * 1024 + (q & 1) * 512>(ab);
      });
    });
    // unit u = (cout block I = u >> 1, K half h = u & 1).  h = 0: hi*hi of block I first, then the
    // previous block's corrections are flushed (its MFMAs have finished under block I's), then block
    // I's corrections of this half start a fresh c2; h = 1: the corrections, then hi*hi.  Block 3's
    // corrections are flushed at the next step's first unit (c2 lives across the barrier; after the
    // last step, below the loop).
    static_for<NU>([&](auto u_c) {
      constexpr int u = decltype(u_c)::value, I = u >> 1, h = u & 1;
      if constexpr (u + 2 < NU) {
        static_for<NPL>([&](auto p_c) {
          constexpr int p = decltype(p_c)::value;
          af[(u + 2) % 3][p] = ds_read16<(p * APL + 2 * ((u + 2) >> 1)) * 1024 + ((u + 2) & 1) * 512>(ab);
        });
      }
      constexpr int after = (u + 1 < NU ? NPL : 0) + (u + 2 < NU ? NPL : 0);
      asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(after) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (h == 0) {
#pragma unroll
        for (int J = 0; J < PB; ++J) mma32(acc[I][J], af[u % 3][0], bf[0][J][h]);
        flush(acc[(I + CB - 1) % CB]);  // (u = 0: block 3 of the previous step; zero before the first)
        __builtin_amdgcn_sched_barrier(0);  // (the flush reads c2 before the fresh c2 is written: no second set)
#pragma unroll
        for (int J = 0; J < PB; ++J) {
          c2[J] = (f32x16){};
          mma32(c2[J], af[u % 3][0], bf[1][J][h]);  // hi*lo', then lo'*hi: k_conv3's term order
          mma32(c2[J], af[u % 3][1], bf[0][J][h]);
        }
      } else {
#pragma unroll
        for (int J = 0; J < PB; ++J) {
          mma32(c2[J], af[u % 3][0], bf[1][J][h]);
          mma32(c2[J], af[u % 3][1], bf[0][J][h]);
        }
#pragma unroll
        for (int J = 0; J < PB; ++J) mma32(acc[I][J], af[u % 3][0], bf[0][J][h]);
      }
      if constexpr (u == 0)  // the next step's DMA (8 pieces) after the first unit's MFMAs
        static_for<2 * TPW>([&](auto q_c) { piece(q_c, s ^ 1, dn); });
      if constexpr (STR && u == 2) {
        if (strip_now) strip_issue(r_gs ^ 1);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  issue(0);
  if constexpr (STR) strip_issue(0);
  vm_wait<0>();
  wbarrier32();
  __builtin_amdgcn_sched_barrier(0);
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  auto end_step = [&](const bool sn) {
    if (STR && sn && nx > 1) vm_wait<4>();
    else vm_wait<0>();
    wbarrier32();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (STR) {
      if (++r_txi == nx) {
        r_txi = 0;
        r_gs ^= 1;
      }
    }
  };
  for (int ks = 0; ks < nK; ks += 2) {
    const bool sn0 = STR && r_txi == 0 && ks + nx < nK;
    step(I0{}, ks + 1 < nK, sn0);
    end_step(sn0);
    if (ks + 1 >= nK) break;
    const bool sn1 = STR && r_txi == 0 && ks + 1 + nx < nK;
    step(I1{}, ks + 2 < nK, sn1);
    end_step(sn1);
  }
  flush(acc[CB - 1]);  // the last step's block 3

  // ---------------- epilogue: v_permlane32_swap pairs element groups (q, q + 1) ----------------
  using SP = SplitF32<NPL>;
  bool bad = false;
  const long psy = (long)A.N * S.OH * S.OW * S.ldy;
  const long psr = (long)A.N * S.OH * S.OW * A.ldr;
  // Lane layout after the swaps: v_permlane32_swap of element groups (0, 1) and (2, 3) gives lane l
  // channels 8 q + 8 (l >> 5) .. + 7 of pixel l & 31 (q = 0, 2); a v_permlane16_swap of those two
  // results then gives rows {0, 2, 1, 3}[l >> 4] of 8 channels of pixel l & 15 (first) and 16 + (l & 15)
  // (second): each store instruction writes the 64 contiguous bytes of 32 channels of 16 pixels, as
  // k_conv3w's -- with the first pairing alone a store wrote 32-byte halves of 32 pixels, and its
  // non-temporal stores ran ConvT launches at half speed (tools/conv3_ab.py, round 6).
  const int csl = ((lane >> 4) & 1) * 16 + (lane >> 5) * 8;  // this lane's channel group in a 32-block
  size_t pixv[PB][2];
  bool pokv[PB][2];
#pragma unroll
  for (int J = 0; J < PB; ++J)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int p = p0 + wp * 64 + J * 32 + hf * 16 + (lane & 15);
      pokv[J][hf] = p < M;
      const int pp = pokv[J][hf] ? p : 0;
      const int n = pp / GHW, rr = pp - n * GHW;
      const int gy = rr / A.GW, gx = rr - gy * A.GW;
      pixv[J][hf] = ((size_t)n * S.OH + (gy * S.oys + S.oyo)) * S.OW + (gx * S.oxs + S.oxo);
    }
#pragma unroll
  for (int I = 0; I < CB; ++I) {
    const int cs = c0 + wc * 128 + I * 32 + csl;  // this lane's 8 channels
    const bool cok = cs < A.Cout;
    float sc[8], sh[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      sc[r] = 1.f;
      sh[r] = 0.f;
    }
    if (cok && S.scale) {
      const float4 s0 = *(const float4*)(S.scale + cs), s1 = *(const float4*)(S.scale + cs + 4);
      sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w;
      sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
    }
    if (cok && S.shift) {
      const float4 s0 = *(const float4*)(S.shift + cs), s1 = *(const float4*)(S.shift + cs + 4);
      sh[0] = s0.x; sh[1] = s0.y; sh[2] = s0.z; sh[3] = s0.w;
      sh[4] = s1.x; sh[5] = s1.y; sh[6] = s1.z; sh[7] = s1.w;
    }
#pragma unroll
    for (int J = 0; J < PB; ++J) {
      float v[2][8];  // [pixel half][channel]
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // all lanes active here (cross-lane ops)
        const auto a0 = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[I][J][r]), __float_as_uint(acc[I][J][4 + r]),
                                                         false, false);
        const auto a2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[I][J][8 + r]),
                                                         __float_as_uint(acc[I][J][12 + r]), false, false);
        const auto b0 = __builtin_amdgcn_permlane16_swap(a0[0], a2[0], false, false);
        const auto b1 = __builtin_amdgcn_permlane16_swap(a0[1], a2[1], false, false);
        v[0][r] = __uint_as_float(b0[0]);
        v[1][r] = __uint_as_float(b0[1]);
        v[0][r + 4] = __uint_as_float(b1[0]);
        v[1][r + 4] = __uint_as_float(b1[1]);
      }
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        if (!(pokv[J][hf] && cok)) continue;
        const size_t pix = pixv[J][hf];
        float* vv = v[hf];
#pragma unroll
        for (int r = 0; r < 8; ++r) vv[r] = vv[r] * sc[r] + sh[r];
        if (A.res) {
          const unsigned short* R = (const unsigned short*)A.res + pix * A.ldr + A.cr0 + cs;
          uint4 rq[NPL];
#pragma unroll
          for (int pl = 0; pl < NPL; ++pl) rq[pl] = *(const uint4*)(R + pl * psr);
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            unsigned short qv[NPL];
#pragma unroll
            for (int pl = 0; pl < NPL; ++pl) {
              const uint32_t w4[4] = {rq[pl].x, rq[pl].y, rq[pl].z, rq[pl].w};
              qv[pl] = (unsigned short)(w4[r >> 1] >> ((r & 1) * 16));
            }
            vv[r] += SP::join(qv);
          }
        }
        if (A.relu) {
#pragma unroll
          for (int r = 0; r < 8; ++r) vv[r] = fmaxf(vv[r], 0.f);
        }
        uint32_t o[NPL][4];
#pragma unroll
        for (int r = 0; r < 8; r += 2) {
          unsigned short q0[NPL], q1[NPL];
          SP::split(vv[r], q0);
          SP::split(vv[r + 1], q1);
          bad |= h2_overflow(vv[r]) || h2_overflow(vv[r + 1]);
#pragma unroll
          for (int pl = 0; pl < NPL; ++pl) o[pl][r >> 1] = (uint32_t)q0[pl] | ((uint32_t)q1[pl] << 16);
        }
        unsigned short* Y = (unsigned short*)S.y + pix * S.ldy + S.cy0 + cs;
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) {
          if (!(flags & 1)) {  // non-temporal stores, as k_conv3w (flags & 1: plain)
            typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 v4 = {o[pl][0], o[pl][1], o[pl][2], o[pl][3]};
            __builtin_nontemporal_store(v4, (u32x4*)(Y + pl * psy));
          } else {
            *(uint4*)(Y + pl * psy) = make_uint4(o[pl][0], o[pl][1], o[pl][2], o[pl][3]);
          }
        }
      }
    }
  }
  raise_range_flag(TG.rflag, bad);
}

// zp_conv_tuning key 18: the 32 x 32 MFMA form of the 256 x 256 tile (1) or k_conv3w's 16 x 16 one
// (0, default) (-1: ZP_CONV3W_MF32 or 0)
static int g_conv3w_mf32 = -1;
int conv3w_mf32_mode(int v) {
  const int old = g_conv3w_mf32;
  g_conv3w_mf32 = v;
  return old;
}
bool conv3w_mf32_on() {
  static const int env = getenv("ZP_CONV3W_MF32") ? atoi(getenv("ZP_CONV3W_MF32")) : 0;
  return (g_conv3w_mf32 >= 0 ? g_conv3w_mf32 : env) != 0;
}

void conv3w32_launch(const zp_conv_args& a, const conv_taps& tg, hipStream_t st, int fl, bool str) {
  const dim3 grid((unsigned)(((long)a.N * a.GH * a.GW + 255) / 256), (unsigned)(a.Cout / 256), (unsigned)a.nsub);
  if (str) hipLaunchKernelGGL((k_conv3w32<true>), grid, dim3(512), 0, st, a, tg, fl);
  else hipLaunchKernelGGL((k_conv3w32<false>), grid, dim3(512), 0, st, a, tg, fl);
}

}  // namespace zp
