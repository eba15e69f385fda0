// k_conv3w: the wide-tile two-plane split-fp32 (ZP_F32H2) convolution for gfx950 -- 256 output
// channels x 256 pixels per workgroup (k_conv3's tile is 128 x 256).
//
// Why: k_conv3<h2, 128 x 256> is bound by its staging, not by its MFMAs.
// A K step (one tap x 32 channels) stages 48 KB (two planes of 128 weight rows + 256 pixel rows)
// for 1536 MFMA cycles per SIMD, and the ablations (profiles/r03_conv3_ablation.txt) show the
// kernel running as long without its MFMAs as with them.  Staged bytes per FLOP scale as
// 1/TC + 1/TP: the 256 x 256 tile stages 64 KB per K step for 3072 MFMA cycles per SIMD, two
// thirds of the bytes per FLOP, and halves the per-step fixed costs (barrier, first-read latency,
// DMA issue) per FLOP.
//
// Numerics (template NUM; zp_conv_tuning key 13).  Every product a*b = hi*hi + (hi*lo' + lo'*hi) *
// 2^-11 of exact fp16 products on v_mfma_f32_16x16x32_f16 (SplitF32<2> operands).  The default
// (ACC_FLUSH, round 5) is k_conv3's: the two correction products of a 16 x 16 block go into a fresh
// accumulator c2, hi*hi into acc, and c2 joins acc one cout block later by a rounding FMA
// (acc = fma(c2, 2^-11, acc)) -- bit-identical to k_conv3<h2>.  Round 4's ACC_SA put all three
// products into ONE accumulator on the 2^11 scale ((2^11 w_hi)*x_hi + w_hi*x_lo' + w_lo'*x_hi, 2^11
// w_hi by v_pk_mul_f16; the epilogue folds 2^-11 into the BN scale): 4-6% faster on the big 3x3s, but
// the MFMA aligns the small correction products to the large running sum and truncates their low
// bits, a systematic bias of about -1e-7 relative per conv (r05: -1.0e-7 against
// -1.4e-9 flushed and 9e-10 for exact f32 on a K = 144 conv, tests/test_gpu_x3.py
// test_wide_accumulation_forms).  ACC_PS (per-step partial sums from zero, added by v_add_f32) has
// the smallest rms but still truncates the corrections against the step's main partial (-2e-8) and
// ran slowest; it stays for A/B.
// Tile: 8 waves = 2 (cout halves of 128) x 4 (pixel quarters of 64); a wave owns 8 x 4 blocks of
// 16 x 16 (128 accumulator registers).  Its 8 weight fragments are streamed through a 3-deep
// register ring, the 4 pixel fragments of both planes are held for the step: ~210 VGPRs, no spill
// at two waves per SIMD.
// Staging: per plane, a 16-row x 32-element tile (1 KB) is ONE buffer_load ... lds of 64 lanes
// (lane l: row l & 15, elements (l >> 4) * 8 ..), so the LDS image is in MFMA fragment order and
// every fragment read is a lane-linear conflict-free ds_read_b128.  2-stage ring of 64 KB: the DMA
// of step k + 1 is issued at the top of step k into the buffer step k - 1 read (every wave passed
// the barrier that ended step k - 1) and has the whole step to land.
// Epilogue: v_permlane16_swap pairs the lane groups of cout blocks (i, i + 1) so that a lane holds
// 8 consecutive output channels of one pixel: 16 B stores per lane and plane (k_conv3 stores 8 B),
// 16 B residual loads.
#include "zp_conv_kern.h"
#include "zp_conv3.h"

namespace zp {

// accumulation forms of the two-plane products (template NUM; zp_conv_tuning key 13)
constexpr int ACC_FLUSH = 0;  // k_conv3's: correction accumulator flushed per step by a scaled FMA
constexpr int ACC_SA = 1;     // one scaled accumulator (round 4): biased, see the numerics note
constexpr int ACC_PS = 2;     // per-step partial from zero, added by a rounding v_add_f32 (round 5)
constexpr int ACC_FS = 3;     // ACC_FLUSH with acc on the 2^11 scale: the flush is a plain v_add_f32
constexpr int ACC_P2 = 4;     // round 6: a persistent second accumulator for the corrections, joined once
                              // after the K loop (the 256 x 128 tile only: 64 more accumulator VGPRs)

__device__ __forceinline__ void wbarrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ABL: diagnostic ablations (timing only, wrong results): 1 no DMA after the prologue, 2 no MFMA, 3 no
// barrier in the main loop, 4 / 5 no weight / activation DMA after the prologue
// DM: the next step's 8 DMA pieces are issued over the first DM cout blocks of a step (8 / DM per
// block, after its correction MFMAs)
// HEAD: the fused 1x1 head (zp_conv2d_head): the conv output feeds the head's MFMAs instead of
// being stored
// nsplit > 1 (small grids, e.g. bs = 1): blockIdx.z = sub * nsplit + K slice; the slice's raw f32
// sums go to ws [nsub][nsplit][M][Cout] and k_splitk_epi (zp_conv3.hip) finishes them
// SGB: the cout block's MFMAs and the previous block's flush FMAs interleaved by
// sched_group_barrier (1 MFMA, 2 VALU, ...) instead of the compiler's own order
// PF: L2 prefetch of the next chunk's activation rows (see prep below; measured no gain, off)
// BF: the activation pieces of a step issued before its weight pieces
// STR: strip staging of the activations (stride-1 convs with >= 2 tap columns, conv3w_strip_ok):
//   the input rows of a (32-channel chunk, tap row) group -- TR = 256 / GW output rows' input row
//   plus the tap-column halo, TR x (GW + (nx - 1) dtx) pixels -- are staged ONCE per group, in
//   1 KB pieces of 16 pixels, and the group's nx steps read their pixel fragments from it at a
//   shift of txi * dtx pixels.  For a 3x3 conv that is a third of the activation pieces of the
//   per-step tiles (the part of the staging that costs: tools/conv3_ab.py ablations), and a
//   strip is issued a step and a half before its first use.
// SA: one scaled accumulator per block (see the numerics note above); SA = false: k_conv3's
//   correction accumulator c2, flushed one cout block later (acc = fma(c2, 2^-11, acc))
#ifdef ZP_STAMP
// Diagnostic build only (tools/stamp_build.sh -> tools/stamp/libzp_stamp.so, loaded through ZP_LIB; the
// product libzp.so never defines ZP_STAMP): per wave of the plain wide tile, the shader clock
// (s_memtime) summed over the K loop's segments -- [0] step start -> first fragments landed,
// [1] -> end of the step's MFMA blocks, [2] -> the next step's DMA landed (vm_wait), [3] -> past the
// barrier -- and [4] the whole K loop, written by lane 0 of every wave of the LAST launch.
constexpr int ZP_STAMP_WAVES = 1 << 17;
__device__ unsigned long long zp_stamp_buf[ZP_STAMP_WAVES * 8];
#endif

template <int ABL, int DM, bool HEAD, bool SGB = false, bool PF = false, bool BF = false, bool STR = false,
          int NUM = ACC_FLUSH, int TPX = 256, bool PFB = false>
__global__ void __launch_bounds__(512) k_conv3w(const zp_conv_args A, const conv_taps TG, const int flags,
                                                const zp_head_args H, float* __restrict__ ws, const int nsplit) {
  constexpr int NPL = 2;
  constexpr int TC = 256, TP = TPX;
  static_assert(TP == 256 || TP == 128, "pixel tile");
  static_assert(TP == 256 || (!HEAD && !BF && DM == 1), "the 256 x 128 tile: plain epilogue, default DMA order");
  constexpr bool SA = NUM == ACC_SA || NUM == ACC_PS || NUM == ACC_FS;  // accumulators on the 2^11 scale
  constexpr bool P2 = NUM == ACC_P2;
  static_assert(!P2 || (TPX == 128 && !HEAD), "the persistent correction accumulator: 256 x 128 tiles");
  // PFB (round 6, zp_conv_tuning key 21): the next step's pixel fragments read from the strip BEFORE the
  // barrier that ends a step -- by plain LDS loads the compiler tracks (they are carried across the
  // barrier and the loop edge) -- instead of after it, where all eight waves' fragment reads hit the
  // LDS at once (shader-clock stamps: ~16% of the K loop from a step's start to its first fragments,
  // tools/stamp_conv3w.py).  Legal for 3 x 3 convs (three tap columns): the next step reads the current
  // strip, or the next group's, issued in the group's first step and complete and visible since the
  // barrier of its second.  One sub, no split-K (conv3w_launch checks)
  static_assert(!PFB || (STR && !P2 && NUM == ACC_FLUSH && TPX == 256), "pixel-fragment prefetch: the strip tile");
  constexpr int NTW = TC / 16, NT = (TC + TP) / 16;  // weight tiles / all tiles per plane (16 rows each)
  constexpr int UNITS = NPL * NT;                    // 1 KB DMA units per stage
  constexpr int WC = 8, WP = TP / 64;                // per wave: 8 cout blocks x 4 (TP 128: 2) pixel blocks
  constexpr int TPW = NT / 8;                        // tiles per wave: 2 weight + 2 (TP 128: 1) activation
  constexpr int NPC = 2 * TPW;                       // DMA pieces per wave and step (both planes)
  static_assert(NPC % DM == 0 && NPC <= 2 * WC, "DMA pieces over the first DM cout blocks");
  using MT = MfmaTraits<f16_t>;
  constexpr int SPMAX = 20;              // STR: strip pieces per plane (320 pixels)
  constexpr int APL = STR ? NTW : NT;    // units per plane of a stage of the per-step ring
  constexpr int ASTG = NPL * APL;        // units per stage of the per-step ring (STR: weights only)
  constexpr int LDSU = STR ? 2 * ASTG + 2 * NPL * SPMAX : 2 * UNITS;
  __shared__ uint4 lds[LDSU * 64];
  static_assert(LDSU * 1024 <= 160 * 1024, "LDS");
  static_assert(((NPL - 1) * NT + NT - 1) * 1024 < 65536, "ds_read immediate range");
  int tb = (int)blockIdx.z / nsplit;
  const int kz = (int)blockIdx.z - tb * nsplit;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid >> 2, wp = wid & 3;
  const int GHW = A.GH * A.GW;
  const int M = A.N * GHW;
  int bx = blockIdx.x, by = blockIdx.y;
  const int total = gridDim.x * gridDim.y;
  if ((flags & 32768) && nsplit == 1 && A.nsub > 1 && (total & 7) == 0) {
    // sub-interleaved order (round 6, zp_conv_tuning key 17; measured slower, off): the subs of a
    // pixel tile are dispatched back to back on one XCD (dispatch id % 8 picks the XCD), longest
    // first, so the input strip all four phases read is fetched from HBM once and hit in that
    // XCD's L2 by the others (phase-major order re-read the input once per phase: up2's ConvT read
    // 721 MB for a 168 MB input, profiles/r06a_fp32_dispatches.csv); the phases' weights (2.9 MB in
    // all for up2) stay L2-resident.  Consecutive pixel tiles (shared halo rows) stay on one XCD.
    const int gid = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int q = gid >> 3;
    tb = q % A.nsub;
    const int tile = (gid & 7) * (total >> 3) + q / A.nsub;
    bx = tile / gridDim.y;
    by = tile - bx * gridDim.y;
  } else if (flags & 2) {  // XCD-aware order (k_conv): consecutive pixel tiles (shared halo rows) on one XCD
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
  // this slice's K steps [ks0, ks0 + nK) (STR: whole groups of nx steps)
  const int kq = STR ? nx : 1, nq = nK_all / kq;
  const int ks0 = (int)((long)kz * nq / nsplit) * kq;
  const int nK = (int)((long)(kz + 1) * nq / nsplit) * kq - ks0;
  const int lr = lane & 15, lk = (lane >> 4) * 8;
  const unsigned psx_b = (unsigned)((long)A.N * A.IH * A.IW * A.ldx * 2);
  const unsigned psw_b = (unsigned)((long)A.w_rows * A.k_pad * 2);

  // DMA tiles of this wave: t = wid + 8 k (k 0, 1: weight tiles; 2, 3: activation tiles), both
  // planes each; per-lane plane-0 byte offsets and the activation tiles' tap validity masks
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
  // STR: this wave's strip pieces P = wid + 8 k (k < 3, P < nsp; both planes): lane (lr, lk) loads
  // strip pixel s = 16 P + lr = r * SW + c (output row r of the tile, input column c + tx0) at the
  // group's tap row; sym: tap rows whose input row is in the image (0: column / row outside)
  int nsp = 16, SW = 0, sh0 = 0;
  unsigned sbase[3], sym[3];
  int sj[WP];  // the strip pixel of this lane's pixel block j at the strip's first column
  if constexpr (STR) {
    // the strip's columns start at the leftmost tap column (the ConvT phases list theirs right to
    // left: dtx = -1); tap column txi reads at a shift of sh0 + txi * dtx pixels
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
    for (int j = 0; j < WP; ++j) {
      const int q = wp * 16 * WP + j * 16 + lr;
      sj[j] = (q / A.GW) * SW + q % A.GW;
    }
  }
#if defined(__HIP_DEVICE_COMPILE__)
  const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)A.x, (short)0, (int)TG.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)S.w, (short)0, (int)TG.w_bytes[tb], 0x00020000);
#endif
  // scalar walk of the next step to issue: 32-channel chunk outer, taps inner (k_conv3's order: the
  // taps of one chunk re-read nearly the same input rows from L2)
  // (the walk starts at step ks0 = (chunk w_cb, tap w_tyi * nx + w_txi))
  const int t0 = ks0 % S.ntaps;
  int w_cb = ks0 / S.ntaps, w_tyi = t0 / nx, w_txi = t0 - (t0 / nx) * nx;
  const int step_x = dtx * A.ldx * 2, step_y = dty * A.IW * A.ldx * 2;
  int act_off = ((TG.ty0[tb] * A.IW + TG.tx0[tb]) * A.ldx) * 2 + w_tyi * step_y + w_txi * step_x + w_cb * 64;
  int w_koff = (t0 * A.Cin + w_cb * 32) * 2;
  const int cin2 = A.Cin * 2;
  // the DMA of one K step as 8 pieces (tile k = q / 2 of this wave, plane q % 2): prep() forms the
  // per-lane offsets of the next step to issue and advances the walk; piece<q>() issues one piece
  struct DmaStep {
    unsigned voff[TPW];
    int koff;
  };
  // L2 prefetch of the next 32-channel chunk's activation rows.  Measured (flags 4194304 / 8388608:
  // builds without the weight / the activation DMA): the weight pieces (L2-resident, read by every
  // workgroup) cost nothing, the activation pieces 25% of the kernel -- each chunk's first tap
  // misses L2 (~14% of the activation rows per launch, TCC counters) and the step's barrier waits
  // for the slowest piece.  So at the first tap of chunk cb, one dword per 64-byte row of chunk
  // cb + 1's first tap (this wave's two activation tiles x two planes = the 64 lanes) is loaded and
  // discarded: nine steps later those rows are L2 hits.
  unsigned pf_sink = 0;
  const bool pf_hi = (lane >> 5) & 1;  // lane groups 0, 1 -> activation tile 2; 2, 3 -> tile 3
  constexpr int PFT = TPW - 1;  // (TP 128: one activation tile)
  const unsigned pf_base = pf_hi ? ubase[PFT] : ubase[2], pf_ym = pf_hi ? uym[PFT] : uym[2], pf_xm = pf_hi ? uxm[PFT] : uxm[2];
  const unsigned pf_plane = ((lane >> 4) & 1) ? psx_b : 0u;
  auto prep = [&](DmaStep& d) {
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      bool ok = (uym[k] >> w_tyi) & (uxm[k] >> w_txi) & 1u;
      if constexpr (ABL == 6) ok = ok && w_txi == 0;  // diagnostic: activation pieces at one tap column in 3
      d.voff[k] = k < 2 ? ubase[k] : (ok ? ubase[k] + (unsigned)act_off : 0x80000000u);
    }
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (PF) {  // every step (no branch, no merge that would wait for the value): out of range
      const bool ok = w_tyi == 0 && w_txi == 0 && w_cb + 1 < CB && (pf_ym & pf_xm & 1u);  // except at chunk starts
      const unsigned vo = ok ? pf_base + (unsigned)(act_off + 64) + pf_plane : 0x80000000u;
      pf_sink = __builtin_amdgcn_raw_buffer_load_b32(xrsrc, vo, 0, 0);
    }
#endif
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
    if constexpr ((ABL == 4 && k < 2) || (ABL == 5 && k >= 2)) return;  // diagnostic: no weight / activation DMA
    if constexpr (STR && k >= 2) return;                                   // (the strips carry the activations)
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
  // STR: the strip walk (next group to issue: chunk g_cb, tap row g_tyi) and its issue into strip
  // stage gst (4 pieces per wave, 6 on the waves with a third piece)
  int g_cb = ks0 / S.ntaps, g_tyi = (ks0 - (ks0 / S.ntaps) * S.ntaps) / nx;
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
  // STR: the step being computed reads strip stage r_gs at tap column r_txi
  int r_txi = 0, r_gs = 0;
  const unsigned sl0 = lds_addr(lds) + (unsigned)(2 * ASTG) * 1024u + (unsigned)(lane >> 4) * 256u;

  f32x4 acc[WC][WP];
#ifdef ZP_STAMP
  constexpr bool STAMP = !HEAD && NUM == ACC_FLUSH && TPX == 256 && ABL == 0;
  unsigned long long st_seg[4] = {0, 0, 0, 0}, st_t = 0, st_loop0 = 0;
  auto stamp = [&](int k) {
    if constexpr (STAMP) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      if (k >= 0) st_seg[k] += now - st_t;
      st_t = now;
    }
  };
#define ZP_STAMP_AT(k)                  \
  do {                                  \
    __builtin_amdgcn_sched_barrier(0);  \
    stamp(k);                           \
    __builtin_amdgcn_sched_barrier(0);  \
  } while (0)
#else
#define ZP_STAMP_AT(k) \
  do {                 \
  } while (0)
#endif
  // P2 (ACC_P2): the correction products' own running sums, one per block, for the whole K loop --
  // no per-step flush (4 v_fma_f32 per block and step, which with 2 waves per SIMD kept the vector
  // issue port ~95% busy beside the MFMAs: tools/conv3_ab.py ablations)
  f32x4 c2acc[P2 ? WC : 1][P2 ? WP : 1];
#pragma unroll
  for (int i = 0; i < WC; ++i)
#pragma unroll
    for (int j = 0; j < WP; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if constexpr (P2) {
#pragma unroll
    for (int i = 0; i < WC; ++i)
#pragma unroll
      for (int j = 0; j < WP; ++j) c2acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }

  // fragment reads: inline-asm ds_read_b128 with explicit lgkmcnt waits.  Plain LDS loads would
  // make the compiler put an s_waitcnt vmcnt(0) in front of every fragment read issued after the
  // LDS-DMA of the next step (it cannot tell the DMA's LDS destination from the buffer being read),
  // i.e. wait for the next step's staging before computing this one.
  const unsigned l0 = lds_addr(lds) + (unsigned)lane * 16u;
  const unsigned abase0 = l0 + (unsigned)(wc * WC) * 1024u, bbase0 = l0 + (unsigned)(NTW + wp * WP) * 1024u;
  const unsigned abase1 = abase0 + ASTG * 1024u, bbase1 = bbase0 + UNITS * 1024u;
  // one K step on stage buffer s: the 4 pixel fragments of both planes held for the step, the 8
  // weight fragments streamed 2 ahead; per block: c2 = hi*lo' + lo'*hi, acc += hi*hi, and the flush
  // acc = fma(c2, 2^-11, acc) one cout block later (its MFMAs have finished by then)
  constexpr bool abl_dma = ABL == 1, abl_mfma = ABL == 2, abl_bar = ABL == 3;
  // a cout block's per-step sums into its accumulators (NUM 2: one rounding add; NUM 0: the scaled
  // correction FMA); the asm pins each add here -- sunk into the next step, every block's c2 would
  // stay live (333 spilled VGPRs)
  auto flush = [&](f32x4 (&a)[WP], const f32x4 (&c)[WP]) {
#pragma unroll
    for (int j = 0; j < WP; ++j) {
      if constexpr (NUM == ACC_PS || NUM == ACC_FS) {
        // (rebuilt as a whole vector: element-wise updates of a[j] spilled 130+ VGPRs, and a vector
        // add becomes v_pk_add_f32, which costs ~13 cycles more than two v_add_f32 beside MFMAs)
        const f32x4 t = {a[j].x + c[j].x, a[j].y + c[j].y, a[j].z + c[j].z, a[j].w + c[j].w};
        a[j] = t;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) a[j][r] = __builtin_fmaf(c[j][r], SplitF32<2>::CS, a[j][r]);
      }
      asm volatile("" : "+v"(a[j]));
    }
  };
  uint4 bfo[NPL][WP];  // PFB: the pixel fragments of the step about to run
  auto load_bf = [&](int gs, int txi) {
    if constexpr (PFB) {
      // (the strip fragment addresses of the asm reads below, as uint4 indices into lds)
      const int base = 2 * ASTG * 64 + (lane >> 4) * 16 + gs * (NPL * SPMAX * 64);
      const int sh = sh0 + txi * dtx;
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        const int sp = sj[j] + sh;
        const int ix = base + (sp >> 4) * 64 + (sp & 15);
#pragma unroll
        for (int p = 0; p < NPL; ++p) bfo[p][j] = lds[ix + p * SPMAX * 64];
      }
    }
  };
  auto step = [&](auto s_c, const bool more, const bool strip_now) {
    const int s = (int)s_c;  // (a compile-time stage, or -- P2's one-step loop -- a runtime one)
    // the next step's DMA (into the other buffer: every wave has passed the barrier that ended the
    // step which read it): one piece per cout block, after that block's correction MFMAs, so that
    // the issue cost (~60 cycles per piece beside MFMAs) is spread over the step
    DmaStep dn;
    prep(dn);
    if (!more) {  // no next step: every piece's offset out of the buffers' range (the unit returns, stores nothing)
#pragma unroll
      for (int k = 0; k < TPW; ++k) dn.voff[k] = 0x80000000u;
      dn.koff = 0;
    }
    const unsigned ab = s ? abase1 : abase0, bb = s ? bbase1 : bbase0;
    uint4 bfl[NPL][WP];
    uint4(&bf)[NPL][WP] = *(PFB ? &bfo : &bfl);  // PFB: loaded by the previous step / the prologue
    uint4 af[3][NPL];  // weight fragments: a 3-slot ring
    if constexpr (PFB) {
    } else if constexpr (STR) {  // pixel fragments from the strip: 16 consecutive strip pixels, conflict-free
      const unsigned sb = sl0 + (unsigned)r_gs * (unsigned)(NPL * SPMAX * 1024);
      const int sh = sh0 + r_txi * dtx;
      static_for<WP>([&](auto j_c) {
        constexpr int j = decltype(j_c)::value;
        const int sp = sj[j] + sh;
        const unsigned ad = sb + ((unsigned)(sp >> 4) << 10) + ((unsigned)(sp & 15) << 4);
        static_for<NPL>([&](auto p_c) {
          constexpr int p = decltype(p_c)::value;
          bf[p][j] = ds_read16<p * SPMAX * 1024>(ad);
        });
      });
    } else {
      static_for<NPL>([&](auto p_c) {
        constexpr int p = decltype(p_c)::value;
        static_for<WP>([&](auto j_c) {
          constexpr int j = decltype(j_c)::value;
          bf[p][j] = ds_read16<(p * NT + j) * 1024>(bb);
        });
      });
    }
    static_for<2>([&](auto q_c) {
      constexpr int q = decltype(q_c)::value;
      static_for<NPL>([&](auto p_c) {
        constexpr int p = decltype(p_c)::value;
        af[q][p] = ds_read16<(p * APL + q) * 1024>(ab);
      });
    });
    f32x4 c2p[WP];  // NUM 0 / 2: the previous cout block's per-step sums (flushed one block later)
    static_for<WC>([&](auto i_c) {
      constexpr int i = decltype(i_c)::value;
      if constexpr (i + 2 < WC) {
        static_for<NPL>([&](auto p_c) {
          constexpr int p = decltype(p_c)::value;
          af[(i + 2) % 3][p] = ds_read16<(p * APL + i + 2) * 1024>(ab);
        });
      }
      // reads issued after cout block i's: blocks i + 1 and i + 2 (two planes each)
      constexpr int after = (i + 1 < WC ? NPL : 0) + (i + 2 < WC ? NPL : 0);
      asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(after) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (i == 0) ZP_STAMP_AT(0);
      // NUM 2 (ACC_PS): the three products of the block, on the 2^11 scale, into a fresh c2 --
      // lo'*hi + hi*lo' + (2^11 hi)*hi, the small terms first -- and acc += c2 (v_add_f32, round to
      // nearest) one cout block later.  NUM 1 (ACC_SA): the same three products straight into acc.
      // NUM 0 (ACC_FLUSH): the corrections into a fresh c2 (k_conv3's term order, Terms<2>: hi*lo',
      // then lo'*hi), hi*hi into acc, acc = fma(c2, 2^-11, acc) one block later.
      f32x4 c2[WP];
      uint4 hs;
      if constexpr (SA) hs = scale_hi(af[i % 3][0]);
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        if constexpr (NUM != ACC_SA) c2[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
        if constexpr (abl_mfma) {
          // (the fragment reads are asm volatile: they still issue)
        } else if constexpr (NUM == ACC_SA) {
          MT::mma(acc[i][j], af[i % 3][1], bf[0][j]);
        } else if constexpr (NUM == ACC_PS) {
          MT::mma(c2[j], hs, bf[0][j]);
        } else if constexpr (P2) {  // hi*lo', then lo'*hi (k_conv3's term order) into the block's running sum
          MT::mma(c2acc[i][j], af[i % 3][0], bf[1][j]);
          MT::mma(c2acc[i][j], af[i % 3][1], bf[0][j]);
        } else {
          MT::mma(c2[j], af[i % 3][0], bf[1][j]);
          MT::mma(c2[j], af[i % 3][1], bf[0][j]);
        }
      }
      if constexpr ((NUM == ACC_SA || NUM == ACC_PS) && !abl_mfma) {
#pragma unroll
        for (int j = 0; j < WP; ++j) {
          if constexpr (NUM == ACC_SA) MT::mma(acc[i][j], af[i % 3][0], bf[1][j]);
          else MT::mma(c2[j], af[i % 3][0], bf[1][j]);
        }
      }
      if constexpr (i < DM && !abl_dma)  // (no branch: after the last step the pieces are out of range -> no-ops)
        static_for<NPC / DM>([&](auto q_c) {
          constexpr int q = i * (NPC / DM) + decltype(q_c)::value;
          piece(std::integral_constant<int, BF ? (q + NPC / 2) % NPC : q>{}, s ^ 1, dn);
        });
      if constexpr (STR && i == 1 && !abl_dma) {
        if (strip_now) strip_issue(r_gs ^ 1);
      }
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        if constexpr (abl_mfma) {
          if constexpr (SA) asm volatile("" ::"v"(hs.x), "v"(hs.y), "v"(hs.z), "v"(hs.w));
        } else if constexpr (NUM == ACC_SA) {
          MT::mma(acc[i][j], hs, bf[0][j]);
        } else if constexpr (NUM == ACC_PS) {
          MT::mma(c2[j], af[i % 3][1], bf[0][j]);
        } else if constexpr (NUM == ACC_FS) {
          MT::mma(acc[i][j], hs, bf[0][j]);
        } else {
          MT::mma(acc[i][j], af[i % 3][0], bf[0][j]);
        }
      }
      if constexpr (NUM == ACC_PS) flush(acc[i], c2);  // (the same block: the other wave's MFMAs cover the wait)
      if constexpr ((NUM == ACC_FLUSH || NUM == ACC_FS) && i > 0) flush(acc[i - 1], c2p);
      if constexpr (NUM == ACC_FLUSH || NUM == ACC_FS) {
#pragma unroll
        for (int j = 0; j < WP; ++j) c2p[j] = c2[j];
      }
      if constexpr (SGB) {
        static_for<4>([&](auto) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);  // 1 VALU
        });
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    if constexpr (NUM == ACC_FLUSH || NUM == ACC_FS) flush(acc[WC - 1], c2p);
    ZP_STAMP_AT(1);
    if constexpr (PFB) {  // the next step's pixel fragments (past the last step: harmless reads, unused)
      int ntxi = r_txi + 1, ngs = r_gs;
      if (ntxi == nx) {
        ntxi = 0;
        ngs ^= 1;
      }
      __builtin_amdgcn_sched_barrier(0);
      load_bf(ngs, ntxi);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // prologue: step 0's DMA into buffer 0 (STR: and group 0's strip into strip stage 0)
  issue(0);
  if constexpr (STR) strip_issue(0);
  vm_wait<0>();
  wbarrier();
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (PFB) load_bf(r_gs, r_txi);
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  if (flags & 65536) {  // static priority for the second-dispatched half (MI355X_MICROARCH.md item 4)
    if (wid >= 4) __builtin_amdgcn_s_setprio(1);
  }
  // STR: a step that issued the next group's strip waits for its own per-step pieces only (issued
  // before the strip's 4 .. 6: vmcnt counts in order); the strip lands by the next step's full wait
  auto end_step = [&](const bool sn) {
    if (STR && sn && nx > 1) vm_wait<4>();  // (one-column groups: the strip is read at the next step)
    else vm_wait<0>();
    asm volatile("" ::"v"(pf_sink));  // the prefetch's (discarded) value: consumed after the wait
    ZP_STAMP_AT(2);
    if constexpr (!abl_bar) wbarrier();
    __builtin_amdgcn_sched_barrier(0);
    ZP_STAMP_AT(3);
    if constexpr (STR) {
      if (++r_txi == nx) {
        r_txi = 0;
        r_gs ^= 1;
      }
    }
  };
  if constexpr (P2) {
    // one step per iteration, the stage a runtime value: in the two-step unrolled loop LLVM gave the
    // 128 loop-carried sums different registers in the two copies and spilled 52-61 VGPRs
    for (int ks = 0; ks < nK; ++ks) {
      const bool sn = STR && r_txi == 0 && ks + nx < nK;
      step(ks & 1, ks + 1 < nK, sn);
      end_step(sn);
    }
  } else {
#ifdef ZP_STAMP
  ZP_STAMP_AT(-1);
  st_loop0 = st_t;
#endif
  for (int ks = 0; ks < nK; ks += 2) {
    // step ks on buffer 0, issuing the DMA of step ks + 1 into buffer 1
    const bool sn0 = STR && r_txi == 0 && ks + nx < nK;
    step(I0{}, ks + 1 < nK, sn0);
    end_step(sn0);
    if (ks + 1 >= nK) break;
    const bool sn1 = STR && r_txi == 0 && ks + 1 + nx < nK;
    step(I1{}, ks + 2 < nK, sn1);
    end_step(sn1);
  }
#ifdef ZP_STAMP
  if constexpr (STAMP) {
    const unsigned long long tot = __builtin_amdgcn_s_memtime() - st_loop0;
    const long wv = ((long)blockIdx.x + (long)gridDim.x * ((long)blockIdx.y + (long)gridDim.y * blockIdx.z)) * 8 + wid;
    if (lane == 0 && wv < ZP_STAMP_WAVES) {
      unsigned long long* o = zp_stamp_buf + wv * 8;
      o[0] = st_seg[0]; o[1] = st_seg[1]; o[2] = st_seg[2]; o[3] = st_seg[3]; o[4] = tot; o[5] = (unsigned long long)nK;
    }
  }
#endif
  }
#undef ZP_STAMP_AT
  if constexpr (P2) {  // the corrections join the main sums once: acc = fma(c2, 2^-11, acc) (one rounding)
#pragma unroll
    for (int i = 0; i < WC; ++i)
#pragma unroll
      for (int j = 0; j < WP; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = __builtin_fmaf(c2acc[i][j][r], SplitF32<2>::CS, acc[i][j][r]);
  }

  if (!HEAD && nsplit > 1) {  // split-K slice: raw f32 sums (acc[i][j] = 4 channels x one grid point)
    float* wsl = ws + ((size_t)tb * nsplit + kz) * M * A.Cout;
#pragma unroll
    for (int j = 0; j < WP; ++j) {
      const int p = p0 + wp * 16 * WP + j * 16 + lr;
      if (p >= M) continue;
#pragma unroll
      for (int i = 0; i < WC; ++i) {
        const int cf = c0 + wc * 16 * WC + i * 16 + (lane >> 4) * 4;
        constexpr float cs = SA ? SplitF32<2>::CS : 1.f;  // (SA: the accumulators are on the 2^11 scale)
        *(float4*)(wsl + (size_t)p * A.Cout + cf) =
            make_float4(acc[i][j][0] * cs, acc[i][j][1] * cs, acc[i][j][2] * cs, acc[i][j][3] * cs);
      }
    }
    return;
  }

  // ---------------- epilogue: paired lane groups, 16 B per lane and plane ----------------
  using SP = SplitF32<NPL>;
  bool bad = false;
  const int g = lane >> 4;
  const long psy = (long)A.N * S.OH * S.OW * S.ldy;
  const long psr = (long)A.N * S.OH * S.OW * A.ldr;
  // output pixel of the lane in pixel block j: image, row, column, in range (the HEAD variant
  // recomputes it per use -- register pressure -- the plain epilogue keeps the four)
  struct PixInfo {
    int n, oy, ox;
    bool ok;
  };
  auto pixinfo = [&](int j) {
    const int p = p0 + wp * 16 * WP + j * 16 + lr;
    PixInfo q;
    q.ok = p < M;
    const int pp = q.ok ? p : 0;
    const int n = pp / GHW, rr = pp - n * GHW;
    const int gy = rr / A.GW, gx = rr - gy * A.GW;
    q.n = n;
    q.oy = gy * S.oys + S.oyo;
    q.ox = gx * S.oxs + S.oxo;
    return q;
  };
  PixInfo pi[WP];
  if constexpr (!HEAD) {
#pragma unroll
    for (int j = 0; j < WP; ++j) pi[j] = pixinfo(j);
  }
  // HEAD: the 1x1 head's sums (rows hb * 16 + 4 g + q, pixel block j) over this wave's channels
  f32x4 hacc[2][WP];
  // HEAD: the head weights ([NPL][32 rows][k_pad], 40 KB at k_pad 320) staged in LDS -- free after
  // the main loop's last barrier -- by LDS-DMA in MFMA fragment order: piece (plane, row half hb,
  // 32-channel chunk q) holds lane l's 8 weights of row hb * 16 + (l & 15) at the channels lane
  // group l >> 4 carries in the epilogue's paired layout (conv channels: (g & 1) * 16 + (g >> 1) * 8;
  // the x_128 part: g * 8), so every use is a lane-linear ds_read_b128 (they were global loads, one
  // L1 round trip each)
  const int hnq = H.k_pad / 32;  // 32-channel chunks of a head weight row
  if constexpr (HEAD) {
#pragma unroll
    for (int hb = 0; hb < 2; ++hb)
#pragma unroll
      for (int j = 0; j < WP; ++j) hacc[hb][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#if defined(__HIP_DEVICE_COMPILE__)
    const __amdgpu_buffer_rsrc_t hrsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)H.w, (short)0, NPL * 32 * H.k_pad * 2, 0x00020000);
    const int gq = lane >> 4;
    for (int pc = wid; pc < NPL * 2 * hnq; pc += 8) {  // (wave-uniform)
      const int q = pc % hnq, hb = (pc / hnq) & 1, pl = pc / (2 * hnq);
      const int koff = q * 32 + (q * 32 < A.Cout ? (gq & 1) * 16 + (gq >> 1) * 8 : gq * 8);
      const unsigned vo = (unsigned)(((pl * 32 + hb * 16 + (lane & 15)) * H.k_pad + koff) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(hrsrc, (__attribute__((address_space(3))) void*)&lds[pc * 64], 16, vo, 0, 0, 0);
    }
#endif
    vm_wait<0>();
    __syncthreads();
  }
  // one 32-channel K slice q of the head: weight fragments wf[hb][plane] (k slot g of lane group g),
  // activation fragment planes (xh, xl) of pixel block j
  auto head_mma = [&](const int q, const uint4& xh, const uint4& xl, const int j) {
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      uint4 wf[2][NPL];
      // (inline-asm reads waited on here: plain LDS loads were hoisted over the pixel blocks and
      // spilled the accumulators)
      const unsigned ha = lds_addr(lds) + (unsigned)(((hb * hnq + q) * 64 + lane) * 16);
      wf[hb][0] = ds_read16<0>(ha);
      wf[hb][1] = ds_read16<0>(ha + (unsigned)(2 * hnq * 1024));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      f32x4 c2 = (f32x4){0.f, 0.f, 0.f, 0.f};
      MT::mma(c2, wf[hb][0], xl);
      MT::mma(c2, wf[hb][1], xh);
      MT::mma(hacc[hb][j], wf[hb][0], xh);
#pragma unroll
      for (int r = 0; r < 4; ++r) hacc[hb][j][r] = __builtin_fmaf(c2[r], SplitF32<2>::CS, hacc[hb][j][r]);
    }
  };
#pragma unroll
  for (int i = 0; i < WC; i += 2) {
    // (HEAD: one channel pair at a time -- loads hoisted over the pairs would keep every pair's head
    // weights live beside the accumulators)
    if constexpr (HEAD) __builtin_amdgcn_sched_barrier(0);
    const int cs = c0 + wc * 16 * WC + (i + (g & 1)) * 16 + (g >> 1) * 8;  // this lane's 8 channels
    const bool cok = cs < A.Cout;
    // BN scale / shift of the lane's 8 channels (HEAD: re-read per pixel block from L1, register pressure)
    float sc[8], sh[8];
    auto load_bn = [&]() {
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
      if constexpr (SA) {
#pragma unroll
        for (int r = 0; r < 8; ++r) sc[r] *= SplitF32<2>::CS;  // the accumulators are on the 2^11 scale (exact)
      }
    };
    if constexpr (!HEAD) load_bn();
    // HEAD: the head weights of these 32 channels in the lanes' channel order (lane group g holds
    // channels (g & 1) * 16 + (g >> 1) * 8 .. + 7 of the slice; the MFMA reads them as k slot g)
    const int hq = (wc * 16 * WC + i * 16) / 32;  // the head-weight chunk of this channel pair
#pragma unroll
    for (int j = 0; j < WP; ++j) {
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // all lanes active here (cross-lane op)
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][j][r]), __float_as_uint(acc[i + 1][j][r]),
                                                         false, false);
        v[r] = __uint_as_float(sw[0]);
        v[r + 4] = __uint_as_float(sw[1]);
      }
      if constexpr (HEAD) {
        pi[j] = pixinfo(j);
        load_bn();
      }
      const bool live = pi[j].ok && cok;
      if (!HEAD && !live) continue;
      const size_t pix = ((size_t)pi[j].n * S.OH + pi[j].oy) * S.OW + pi[j].ox;
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = v[r] * sc[r] + sh[r];
      if (A.res && live) {
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
      if (HEAD && !live) {
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = 0.f;
      }
      uint32_t o[NPL][4];
#pragma unroll
      for (int r = 0; r < 8; r += 2) {
        unsigned short q0[NPL], q1[NPL];
        SP::split(v[r], q0);
        SP::split(v[r + 1], q1);
        bad |= h2_overflow(v[r]) || h2_overflow(v[r + 1]);
#pragma unroll
        for (int p = 0; p < NPL; ++p) o[p][r >> 1] = (uint32_t)q0[p] | ((uint32_t)q1[p] << 16);
      }
      if constexpr (HEAD) {  // the conv output is not stored: it feeds the head
        head_mma(hq, make_uint4(o[0][0], o[0][1], o[0][2], o[0][3]), make_uint4(o[1][0], o[1][1], o[1][2], o[1][3]), j);
        __builtin_amdgcn_sched_barrier(0);  // one pixel block at a time (register pressure)
        continue;
      }
      if ((flags & 16384) && v[0] != 1.f) continue;  // diagnostic: no stores (unless a value is exactly 1)
      unsigned short* Y = (unsigned short*)S.y + pix * S.ldy + S.cy0 + cs;
#pragma unroll
      for (int p = 0; p < NPL; ++p) {
        // non-temporal stores (flags & 1: plain, A/B): the output is read by the next layer, not
        // by this kernel; measured up2's ConvT 665 -> 568 us, its 3x3 1392 -> 1372, up1's 350 -> 343
        if (!(flags & 1)) {
          typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
          const u32x4 v4 = {o[p][0], o[p][1], o[p][2], o[p][3]};
          __builtin_nontemporal_store(v4, (u32x4*)(Y + p * psy));
        } else {
          *(uint4*)(Y + p * psy) = make_uint4(o[p][0], o[p][1], o[p][2], o[p][3]);
        }
      }
    }
  }
  raise_range_flag(TG.rflag, bad);
  if constexpr (HEAD) {
    // the second concat part (x2: the skip features, already split NHWC on the output grid) in the
    // cout-half-0 waves, its weights at k = Cout + c
    if (wc == 0) {
      const long psx2 = (long)A.N * S.OH * S.OW * H.ldx2;
      for (int q = 0; q < H.C2 / 32; ++q) {
        const int hq = A.Cout / 32 + q;
#pragma unroll
        for (int j = 0; j < WP; ++j) {
          uint4 xq[NPL];
          const PixInfo q2 = pixinfo(j);
          const size_t pix = ((size_t)q2.n * S.OH + q2.oy) * S.OW + q2.ox;
          const unsigned short* X2 = (const unsigned short*)H.x2 + pix * H.ldx2 + H.cx20 + q * 32 + g * 8;
#pragma unroll
          for (int pl = 0; pl < NPL; ++pl) xq[pl] = q2.ok ? *(const uint4*)(X2 + pl * psx2) : make_uint4(0u, 0u, 0u, 0u);
          head_mma(hq, xq[0], xq[1], j);
        }
      }
    }
    // the two cout halves' sums meet in LDS (free: every wave passed the main loop's last barrier)
    f32x4* red = (f32x4*)(lds + 4096);  // [wp][hb][j][lane], past the staged head weights (64 KB in)
    if (wc == 1) {
#pragma unroll
      for (int hb = 0; hb < 2; ++hb)
#pragma unroll
        for (int j = 0; j < WP; ++j) red[((wp * 2 + hb) * WP + j) * 64 + lane] = hacc[hb][j];
    }
    __syncthreads();
    if (wc == 0) {
      const size_t plane = (size_t)S.OH * S.OW;
#pragma unroll
      for (int hb = 0; hb < 2; ++hb)
#pragma unroll
        for (int j = 0; j < WP; ++j) {
          const f32x4 o = red[((wp * 2 + hb) * WP + j) * 64 + lane];
          const PixInfo q2 = pixinfo(j);
          if (!q2.ok) continue;
          const size_t sp = (size_t)q2.oy * S.OW + q2.ox;
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            const int r = hb * 16 + g * 4 + qq;
            if (r >= H.cout) continue;
            const float val = (hacc[hb][j][qq] + o[qq]) + (H.bias ? H.bias[r] : 0.f);
            if (r == 0) H.mask[(size_t)q2.n * plane + sp] = val;
            else H.code[((size_t)q2.n * (H.cout - 1) + (r - 1)) * plane + sp] = val;
          }
        }
    }
  }
}

// eligibility of the wide tile: two planes, NHWC output with 16-byte-aligned channel slices, Cout a
// multiple of 256 and a grid of at least g_conv3w_min workgroups (fewer: k_conv3's 128 x 256 tile
// keeps more CUs busy)
int conv3w_splitk(const zp_conv_args& a);
static int g_conv3w = -1;       // zp_conv_tuning key 10 (-1: ZP_CONV3W or the default 1)
static int g_conv3w_min = 256;  // zp_conv_tuning key 11
static int g_conv3w_acc = -1;   // zp_conv_tuning key 13: accumulation form (-1: ZP_CONV3W_ACC or ACC_FLUSH)
static int g_conv3w_tp128 = -1; // zp_conv_tuning key 14: 256 x 128 tiles (-1: ZP_CONV3W_TP128 or 0)

int conv3w_acc_mode(int v) {
  const int old = g_conv3w_acc;
  g_conv3w_acc = v;
  return old;
}
int conv3w_tp128_mode(int v) {
  const int old = g_conv3w_tp128;
  g_conv3w_tp128 = v;
  return old;
}
static int conv3w_acc() {
  static const int env = getenv("ZP_CONV3W_ACC") ? atoi(getenv("ZP_CONV3W_ACC")) : ACC_FLUSH;
  const int v = g_conv3w_acc >= 0 ? g_conv3w_acc : env;
  return (v == ACC_PS || v == ACC_SA || v == ACC_FS || v == ACC_P2) ? v : ACC_FLUSH;
}
static bool conv3w_tp128_on() {
  static const int env = getenv("ZP_CONV3W_TP128") ? atoi(getenv("ZP_CONV3W_TP128")) : 0;
  return (g_conv3w_tp128 >= 0 ? g_conv3w_tp128 : env) != 0;
}

int conv3w_mode(int v) {
  const int old = g_conv3w;
  g_conv3w = v;
  return old;
}
int conv3w_min_blocks(int v) {
  const int old = g_conv3w_min;
  g_conv3w_min = v;
  return old;
}

static int conv3w_tp_base(const zp_conv_args& a);
bool conv3w_ok(const zp_conv_args& a) {
  static const int env = getenv("ZP_CONV3W") ? atoi(getenv("ZP_CONV3W")) : 1;
  const int en = g_conv3w >= 0 ? g_conv3w : env;
  if (!en || a.dtype != ZP_F32H2 || a.out_mode != ZP_OUT_NHWC || a.Cout % 256 != 0 || a.Cin % 32 != 0) return false;
  if (a.w_rows % 256 != 0) return false;
  for (int s = 0; s < a.nsub; ++s)
    if (a.sub[s].ldy % 8 != 0 || a.sub[s].cy0 % 8 != 0) return false;
  if (a.res && (a.ldr % 8 != 0 || a.cr0 % 8 != 0)) return false;
  // several sub-problems in one launch: the ConvT phases (1..4 taps) run here, longest first
  // (conv3w_launch).  The merged ASPP's 1 + 9 + 9 + 9 taps stay on k_conv3's tiles: 583-593 us
  // against 607 us wide at bs 32 (tools/conv3_ab.py aspp, profiles/r04_conv3_ab.txt round-close
  // sweeps), with the flushed accumulator
  if (a.nsub > 1)
    for (int s = 0; s < a.nsub; ++s)
      if (a.sub[s].ntaps > 4) return false;
  const long blocks = (((long)a.N * a.GH * a.GW + 255) / 256) * (a.Cout / 256) * a.nsub;
  return blocks >= g_conv3w_min || conv3w_splitk(a) > 1 || conv3w_tp_base(a) == 128;
}

// pixel tile of the wide kernel: 256, or 128 for a one-sub launch whose 256 x 256 grid would leave
// CUs idle (fewer than g_conv3w_min tiles, no split-K) while its 256 x 128 grid fills them (bs 32:
// layer4's 256 -> 256 3 x 3s at 32 x 32 and conv_1x1_3, 128 -> 256 tiles; they ran on k_conv3's
// 128 x 256 tile).  k_conv3w<TP = 128>: a wave owns 8 x 2 blocks, 6 DMA pieces per step.
// ACC_P2 (key 13 = 4) runs every unsplit launch on the 256 x 128 tile (its persistent correction
// accumulator does not fit the 256 x 256 tile's registers); the fused head keeps the 256 x 256 tile
int conv3w_tp(const zp_conv_args& a) {
  if (conv3w_acc() == ACC_P2 && conv3w_splitk(a) == 1) return 128;
  return conv3w_tp_base(a);
}
int conv3w_tp_head(const zp_conv_args& a) { return conv3w_tp_base(a); }
static int conv3w_tp_base(const zp_conv_args& a) {
  const long M = (long)a.N * a.GH * a.GW;
  if (((M + 255) / 256) * (a.Cout / 256) * a.nsub >= g_conv3w_min) return 256;
  if (!conv3w_tp128_on() || a.nsub != 1 || conv3w_splitk(a) > 1) return 256;
  return ((M + 127) / 128) * (a.Cout / 256) >= g_conv3w_min ? 128 : 256;
}

// split-K of the wide tile (zp_conv_tuning key 12, default 1): a one-sub NHWC launch under 64 tiles
// (bs = 1: up2's 3 x 3 at 128 x 128 is 64 tiles, layer5's 512 -> 512 32) is cut along K into up to
// 8 slices of >= 12 steps, for 256..512 workgroups; mode 2 also cuts grids under g_conv3w_min tiles
// in two (bs = 32: layer4's 256 -> 256 at 32 x 32 is 128 tiles; measured 137 us vs k_conv3's 128:
// not the default)
static int g_conv3w_splitk = 1;
int conv3w_splitk_mode(int v) {
  const int old = g_conv3w_splitk;
  g_conv3w_splitk = v;
  return old;
}
int conv3w_splitk(const zp_conv_args& a) {
  if (!g_conv3w_splitk || a.nsub != 1 || a.out_mode != ZP_OUT_NHWC || a.dtype != ZP_F32H2 || a.Cout % 256 != 0)
    return 1;
  const long blocks = (((long)a.N * a.GH * a.GW + 255) / 256) * (a.Cout / 256);
  const int nK = a.sub[0].ntaps * (a.Cin / 32);
  if (blocks > 64) return (g_conv3w_splitk == 2 && blocks < g_conv3w_min && nK / 2 >= 12) ? 2 : 1;
  // under 32 tiles even 8 slices leave CUs idle: k_conv3's smaller tiles (and its own split-K) win
  // (bs = 1, tools/conv3_ab.py --batch 1: layer5's 8 tiles 58.6 us wide vs 45.1 us, up1's 16 tiles
  // 59.1 vs 45.3; up2's 64 tiles 86.4 vs 87.7)
  if (blocks < 32) return 1;
  int ns = 1;
  while (ns < 8 && blocks * ns * 2 <= 512 && nK / (ns * 2) >= 12) ns *= 2;
  return ns;
}

// the strip staging (STR): one sub-problem of stride 1 with >= 2 tap columns, tiles of whole output
// rows (GW a multiple of 16 dividing 256, whole tiles per image) and a strip of <= 320 pixels
// (flag 268435456: off, for A/B)
// (several sub-problems -- the ConvT phases, 1 x 1 / 1 x 2 / 2 x 1 / 2 x 2 taps over the input grid
// -- each with its own strip geometry; one-column subs stage a halo-free strip per step)
static bool conv3w_strip_ok(const zp_conv_args& a, const conv_taps& tg, int fl, int ns, int tp = 256) {
  (void)ns;
  if ((fl & 268435456) || a.sx != 1 || a.sy != 1) return false;
  if (a.GW % 16 != 0 || tp % a.GW != 0 || ((long)a.GH * a.GW) % tp != 0) return false;
  int nxmax = 0;
  for (int s = 0; s < a.nsub; ++s) {
    if (a.sub[s].ntaps != tg.ny[s] * tg.nx[s] || (tg.nx[s] > 1 && tg.dtx[s] == 0)) return false;
    if ((tp / a.GW) * (a.GW + (tg.nx[s] - 1) * abs(tg.dtx[s])) > 320) return false;
    nxmax = max(nxmax, tg.nx[s]);
  }
  return nxmax >= 2;
}

// zp_conv_tuning key 17: the subs (ConvT phases) of a multi-sub launch interleaved per pixel tile on
// one XCD (1) or dispatched phase by phase, longest first (0, default) (-1: ZP_CONV3W_SUBINT or 0).
// Measured (round 6, tools/conv3_ab.py --wsubint 0,1, bs 32): up2's ConvT 593 -> 803 us, up1's
// 130 -> 170 us interleaved -- the input is read once instead of once per phase, but four phases'
// weight streams and the 537 MB output then share each XCD's L2, and every workgroup of a round runs
// a different phase: off
static int g_conv3w_subint = -1;
int conv3w_subint_mode(int v) {
  const int old = g_conv3w_subint;
  g_conv3w_subint = v;
  return old;
}
static bool conv3w_subint() {
  static const int env = getenv("ZP_CONV3W_SUBINT") ? atoi(getenv("ZP_CONV3W_SUBINT")) : 0;
  return (g_conv3w_subint >= 0 ? g_conv3w_subint : env) != 0;
}

#ifdef ZP_STAMP
}  // namespace zp
// diagnostic build only: copy the per-wave segment sums of the last plain wide-tile launch
extern "C" int zp_stamp_read(unsigned long long* dst, long long n) {
  if (n > (long long)zp::ZP_STAMP_WAVES * 8) n = (long long)zp::ZP_STAMP_WAVES * 8;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(zp::zp_stamp_buf), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
namespace zp {
#endif
// zp_conv_tuning key 21: the strip tile's next-step pixel fragments read before the step's barrier
// (PFB; 3 x 3 one-sub launches without split-K).  -1: ZP_CONV3W_PFB or 1.  Measured (tools/conv3_ab.py
// --pfb 0,1, 5 rounds, bit-identical): layer5 326.5 -> 324.3 us, up1's 3x3 350.3 -> 347.3, up2's
// 1418.1 -> 1414.7; stamps: the step-start wait 15.8% -> 5.8% of the K loop, most of it moved to the
// DMA wait the compiler puts before the plain LDS loads (2.1% -> 7.9%), 4741 -> 4660 cycles per step
static int g_conv3w_pfb = -1;
int conv3w_pfb_mode(int v) {
  const int old = g_conv3w_pfb;
  g_conv3w_pfb = v;
  return old;
}
static bool conv3w_pfb_on() {
  static const int env = getenv("ZP_CONV3W_PFB") ? atoi(getenv("ZP_CONV3W_PFB")) : 1;
  return (g_conv3w_pfb >= 0 ? g_conv3w_pfb : env) != 0;
}
void conv3w_launch(const zp_conv_args& a0, const conv_taps& tg0, hipStream_t st, int fl, float* ws, int ns) {
  // several sub-problems (the ConvT phases: 1 / 2 / 2 / 4 taps): dispatched longest first (the
  // dispatcher walks blockIdx.z slowest, so the 4-tap phase's workgroups start first and the
  // 1-tap phase's short ones fill the tail); flag 134217728 keeps the caller's order (A/B)
  zp_conv_args a = a0;
  conv_taps tg = tg0;
  if (a.nsub > 1 && !(fl & 134217728)) {
    int ord[ZP_MAX_SUB];
    for (int s = 0; s < a.nsub; ++s) ord[s] = s;
    for (int i = 1; i < a.nsub; ++i)  // stable insertion sort by descending tap count
      for (int j = i; j > 0 && a0.sub[ord[j]].ntaps > a0.sub[ord[j - 1]].ntaps; --j) {
        const int t = ord[j];
        ord[j] = ord[j - 1];
        ord[j - 1] = t;
      }
    for (int s = 0; s < a.nsub; ++s) {
      const int o = ord[s];
      a.sub[s] = a0.sub[o];
      tg.ny[s] = tg0.ny[o];
      tg.nx[s] = tg0.nx[o];
      tg.ty0[s] = tg0.ty0[o];
      tg.dty[s] = tg0.dty[o];
      tg.tx0[s] = tg0.tx0[o];
      tg.dtx[s] = tg0.dtx[o];
      tg.w_bytes[s] = tg0.w_bytes[o];
    }
  }
  const zp_head_args H{};
  const int acc = (fl & 536870912) ? ACC_FLUSH : conv3w_acc();  // (flag 536870912: the flushed form, as in round 4)
  if (a.nsub > 1 && ns == 1 && conv3w_subint()) fl |= 32768;  // the phases of a pixel tile adjacent on one XCD
  const bool str = conv3w_strip_ok(a, tg, fl, ns);
  if (ns == 1 && conv3w_tp(a) == 128) {  // the 256 x 128 tile (zp_conv_tuning key 14; key 13 = 4: ACC_P2)
    const dim3 g128((unsigned)(((long)a.N * a.GH * a.GW + 127) / 128), (unsigned)(a.Cout / 256), (unsigned)a.nsub);
    const bool s128 = conv3w_strip_ok(a, tg, fl, ns, 128);
    if (acc == ACC_P2) {
      if (s128) hipLaunchKernelGGL((k_conv3w<0, 1, false, false, false, false, true, ACC_P2, 128>), g128, dim3(512), 0, st, a, tg, fl, H, ws, ns);
      else hipLaunchKernelGGL((k_conv3w<0, 1, false, false, false, false, false, ACC_P2, 128>), g128, dim3(512), 0, st, a, tg, fl, H, ws, ns);
    } else if (s128) {
      hipLaunchKernelGGL((k_conv3w<0, 1, false, false, false, false, true, ACC_FLUSH, 128>), g128, dim3(512), 0, st, a, tg, fl, H, ws, ns);
    } else {
      hipLaunchKernelGGL((k_conv3w<0, 1, false, false, false, false, false, ACC_FLUSH, 128>), g128, dim3(512), 0, st, a, tg, fl, H, ws, ns);
    }
    return;
  }
  if (ns == 1 && acc == ACC_FLUSH && conv3w_mf32_on()) {  // the 32 x 32 MFMA form (zp_conv_tuning key 18)
    conv3w32_launch(a, tg, st, fl, str);
    return;
  }
  const dim3 grid((unsigned)(((long)a.N * a.GH * a.GW + 255) / 256), (unsigned)(a.Cout / 256), (unsigned)(a.nsub * ns));
  // flags 262144 / 524288: the DMA pieces over the first 2 / 8 cout blocks (default: the first one);
  // 1048576 / 2097152: DM 1 / 8 with the MFMA / flush interleave (SGB)
  if (fl & 4096) hipLaunchKernelGGL((k_conv3w<1, 1, false>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);  // diagnostic: no DMA
  else if (fl & 8192) hipLaunchKernelGGL((k_conv3w<2, 1, false>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);  // diagnostic: no MFMA
  else if (fl & 131072) hipLaunchKernelGGL((k_conv3w<3, 1, false>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);  // diagnostic: no barrier
  else if (fl & 4194304) hipLaunchKernelGGL((k_conv3w<4, 1, false>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);  // diagnostic: no weight DMA
  else if (fl & 8388608) hipLaunchKernelGGL((k_conv3w<5, 1, false>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);  // diagnostic: no activation DMA
  else if (fl & 262144) hipLaunchKernelGGL((k_conv3w<0, 2, false>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);
  else if (fl & 524288) hipLaunchKernelGGL((k_conv3w<0, 8, false>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);
  else if (fl & 1048576) {  // the MFMA / flush interleave (sched_group_barrier), strips as the default
    if (str) hipLaunchKernelGGL((k_conv3w<0, 1, false, true, false, false, true>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);
    else hipLaunchKernelGGL((k_conv3w<0, 1, false, true>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);
  } else if (fl & 2097152) hipLaunchKernelGGL((k_conv3w<0, 8, false, true>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);
  else if (fl & 16777216) hipLaunchKernelGGL((k_conv3w<0, 1, false, false, true>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);  // L2 prefetch
  else if (fl & 33554432) hipLaunchKernelGGL((k_conv3w<0, 1, false, false, false, true>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);  // activations first
  else if (fl & 67108864) hipLaunchKernelGGL((k_conv3w<6, 1, false, false, false>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);  // diagnostic: 1/3 of the activation pieces
  else if (acc == ACC_SA) {  // round 4's one scaled accumulator (A/B)
    if (str) hipLaunchKernelGGL((k_conv3w<0, 1, false, false, false, false, true, ACC_SA>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);
    else hipLaunchKernelGGL((k_conv3w<0, 1, false, false, false, false, false, ACC_SA>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);
  } else if (acc == ACC_PS) {  // per-step partial sums (A/B)
    if (str) hipLaunchKernelGGL((k_conv3w<0, 1, false, false, false, false, true, ACC_PS>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);
    else hipLaunchKernelGGL((k_conv3w<0, 1, false, false, false, false, false, ACC_PS>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);
  } else if (acc == ACC_FS) {  // the flushed form on the 2^11 scale
    if (str) hipLaunchKernelGGL((k_conv3w<0, 1, false, false, false, false, true, ACC_FS>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);
    else hipLaunchKernelGGL((k_conv3w<0, 1, false, false, false, false, false, ACC_FS>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);
  } else if (str && ns == 1 && a.nsub == 1 && tg.nx[0] == 3 && conv3w_pfb_on())  // (key 21: pixel-fragment prefetch)
    hipLaunchKernelGGL((k_conv3w<0, 1, false, false, false, false, true, ACC_FLUSH, 256, true>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);
  else if (str)  // the default: k_conv3's flushed correction accumulator (bit-identical to k_conv3<h2>)
    hipLaunchKernelGGL((k_conv3w<0, 1, false, false, false, false, true>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);
  else hipLaunchKernelGGL((k_conv3w<0, 1, false>), grid, dim3(512), 0, st, a, tg, fl, H, ws, ns);
}

void conv3w_head_launch(const zp_conv_args& a, const conv_taps& tg, const zp_head_args& h, hipStream_t st, int fl) {
  const dim3 grid((unsigned)(((long)a.N * a.GH * a.GW + 255) / 256), 1u, 1u);
  const bool str = conv3w_strip_ok(a, tg, fl, 1);
  int acc = (fl & 536870912) ? ACC_FLUSH : conv3w_acc();
  if (acc == ACC_P2) acc = ACC_FLUSH;  // (the 256 x 256 head tile: the flushed form)
  if (acc == ACC_SA) {  // (A/B)
    if (str) hipLaunchKernelGGL((k_conv3w<0, 1, true, false, false, false, true, ACC_SA>), grid, dim3(512), 0, st, a, tg, fl, h, nullptr, 1);
    else hipLaunchKernelGGL((k_conv3w<0, 1, true, false, false, false, false, ACC_SA>), grid, dim3(512), 0, st, a, tg, fl, h, nullptr, 1);
  } else if (acc == ACC_FS) {
    if (str) hipLaunchKernelGGL((k_conv3w<0, 1, true, false, false, false, true, ACC_FS>), grid, dim3(512), 0, st, a, tg, fl, h, nullptr, 1);
    else hipLaunchKernelGGL((k_conv3w<0, 1, true, false, false, false, false, ACC_FS>), grid, dim3(512), 0, st, a, tg, fl, h, nullptr, 1);
  } else if (str) {
    hipLaunchKernelGGL((k_conv3w<0, 1, true, false, false, false, true>), grid, dim3(512), 0, st, a, tg, fl, h, nullptr, 1);
  } else {
    hipLaunchKernelGGL((k_conv3w<0, 1, true>), grid, dim3(512), 0, st, a, tg, fl, h, nullptr, 1);
  }
}

}  // namespace zp
