// k_stem_h2: the ResNet stem conv (torchvision conv1: 7x7, stride 2, pad 3, 3 -> 64 channels;
// reference model/resnet.py:195, 233-236) + folded BN + ReLU for the two-plane split-fp32 engine
// (ZP_F32H2), straight from the f32 NHWC image.
//
// The round-3 split stem was two launches: zp_im2col_split wrote the 7 x 7 x 3 patches of every
// output pixel in split form (160 elements x 2 planes x 2 B = 640 B per pixel: 335 MB at bs 32, 171
// us), then a 1 x 1 split GEMM read them back (K = 160: five K steps per tile, ~190 us).  Here a
// workgroup stages the f32 input rows its 256 output pixels need (2 TR + 5 rows of 2 OW + 5 pixels,
// 3 channels: 28 KB at OW = 128) in LDS once, and every lane builds its own MFMA B fragments from
// them: the 16 x 16 x 32 B operand of lane l is pixel l & 15, patch elements (l >> 4) * 8 .. + 7 of
// the K step -- exactly what the lane itself can gather -- split into the two fp16 planes in
// registers.  No patch tensor exists.  Weights (packed for the im2col order k = tap * 3 + c,
// zp_pack_weight with cstride 3) are read as fragments from L2 / L1 (40 KB, every workgroup).
// Numerics: SplitF32<2> operands, hi*hi + (hi*lo' + lo'*hi) * 2^-11 per product, the correction
// accumulator flushed after each K step (k_conv3w's arithmetic).
// Tile: 4 waves, 64 output channels x 256 pixels (a wave: 64 x 64, 4 x 4 blocks of 16 x 16);
// persistent over tiles, one workgroup per CU (round 5), reading NCHW directly when ldx == 0.
#include "zp_conv_kern.h"

namespace zp {

constexpr int STEM_K = 7, STEM_S = 2, STEM_P = 3, STEM_C = 3, STEM_KP = 160;  // 147 patch elements -> 160

// NCHW: x is the reference's input tensor [B][3][H][W] (bop_dataset_pytorch.py:345; no NHWC copy),
// else f32 NHWC [B][H][W][ldx].  Persistent: a workgroup stages the weights once and walks tiles t,
// t + gridDim.x, ...; the next tile's input region is loaded into registers while the current
// tile computes (the one-tile-per-workgroup form paid the load latency and the 40 KB weight staging
// for every tile: 141 us at bs 32).
template <bool NCHW>
__global__ void __launch_bounds__(256) k_stem_h2(const float* __restrict__ x, int B, int H, int W, int ldx,
                                                 const unsigned short* __restrict__ w, int w_rows,
                                                 const float* __restrict__ scale, const float* __restrict__ shift,
                                                 unsigned short* __restrict__ y, int ldy, int cy0, int OH, int OW,
                                                 long psy, unsigned* rflag) {
  constexpr int NPL = 2, WC = 4, WP = 4;
  using MT = MfmaTraits<f16_t>;
  using SP = SplitF32<NPL>;
  // [IR][IC][3] words, each the element split into its two fp16 planes (hi | lo' << 16), then the
  // weights in fragment order.  Splitting (and the range check) once per staged element instead of
  // once per use: every input element feeds ~12 overlapping 7 x 7 / s2 patches.
  extern __shared__ uint32_t region[];
  const int TR = 256 / OW;           // output rows per tile
  const int IR = STEM_S * TR + STEM_K - STEM_S, IC = STEM_S * OW + STEM_K - STEM_S;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wp = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, g = lane >> 4;
  const int tiles_per_img = (OH * OW) / 256, tiles = B * tiles_per_img;
  const int npix = IR * IC;
  // the packed weights staged once per workgroup (40 KB, fragment order [ks][i][plane][lane] of
  // uint4: every K step's reads are lane-linear ds_read_b128)
  uint4* wl = (uint4*)(region + ((IR * IC * 3 + 3) & ~3));
  bool bad = false;
  auto split_word = [&](float v) -> uint32_t {
    unsigned short q[NPL];
    SP::split(v, q);
    bad |= h2_overflow(v);
    return (uint32_t)q[0] | ((uint32_t)q[1] << 16);
  };
  {
    constexpr int NU = (STEM_KP / 32) * WC * NPL * 64;  // 2560 uint4 = 10 per thread
    static_assert(NU % 256 == 0, "weight staging");
    const long wps_ = (long)w_rows * STEM_KP;
#pragma unroll
    for (int m = 0; m < NU / 256; ++m) {
      const int u = tid + 256 * m, l = u & 63, r = u >> 6;
      const int pl = r % NPL, i = (r / NPL) % WC, ks = r / (NPL * WC);
      wl[tid + 256 * m] = *(const uint4*)(w + pl * wps_ + (long)(i * 16 + (l & 15)) * STEM_KP + ks * 32 + (l >> 4) * 8);
    }
  }
  // the input region of a tile, prefetched into registers (zeros outside the image): NHWC one float4
  // per pixel (channels 0..2 used), NCHW one float per element -- all of a thread's loads issued
  // before any use
  constexpr int NRP = 10;  // NHWC: pixels per thread (IR * IC <= 2560 at OW 128: 9 x 261)
  constexpr int NRE = 3 * NRP;  // NCHW: elements per thread (3 channel planes per pixel)
  float4 rp[NCHW ? 1 : NRP];
  float re[NCHW ? NRE : 1];
  auto load_region = [&](int t) {
    const int n = t / tiles_per_img;
    const int iy0 = (t - n * tiles_per_img) * TR * STEM_S - STEM_P, ix0 = -STEM_P;
    if constexpr (NCHW) {  // region pixel e's three channel planes
      const float* xn = x + (size_t)n * 3 * H * W;
      const size_t plane = (size_t)H * W;
#pragma unroll
      for (int m = 0; m < NRP; ++m) {
        const int e = tid + 256 * m;
        const int r = e / IC, c = e - r * IC;
        const int iy = iy0 + r, ix = ix0 + c;
        const bool ok = e < npix && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
        const float* px = xn + (ok ? (size_t)iy * W + ix : 0);
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) re[m * 3 + ch] = ok ? px[ch * plane] : 0.f;
      }
    } else {
#pragma unroll
      for (int m = 0; m < NRP; ++m) {
        const int e = tid + 256 * m;
        const int r = e / IC, c = e - r * IC;
        const int iy = iy0 + r, ix = ix0 + c;
        rp[m] = (e < npix && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
                    ? *(const float4*)(x + (((size_t)n * H + iy) * W + ix) * ldx) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  };
  auto store_region = [&]() {
    if constexpr (NCHW) {
#pragma unroll
      for (int m = 0; m < NRP; ++m) {
        const int e = tid + 256 * m;
        if (e < npix) {
#pragma unroll
          for (int ch = 0; ch < 3; ++ch) region[e * 3 + ch] = split_word(re[m * 3 + ch]);
        }
      }
    } else {
#pragma unroll
      for (int m = 0; m < NRP; ++m) {
        const int e = tid + 256 * m;
        if (e < npix) {
          region[e * 3 + 0] = split_word(rp[m].x);
          region[e * 3 + 1] = split_word(rp[m].y);
          region[e * 3 + 2] = split_word(rp[m].z);
        }
      }
    }
  };
  int t = blockIdx.x;
  if (t < tiles) load_region(t);
  for (; t < tiles; t += gridDim.x) {
    __syncthreads();  // (the previous tile's fragment gathers are done with the region)
    store_region();
    __syncthreads();
    if (t + (int)gridDim.x < tiles) load_region(t + gridDim.x);  // in flight during this tile
    const int n = t / tiles_per_img;
    const int oy0 = (t - n * tiles_per_img) * TR;
    // this lane's pixels: block j -> tile pixel wp * 64 + j * 16 + lr -> (oy - oy0, ox)
    int pbase[WP];
#pragma unroll
    for (int j = 0; j < WP; ++j) {
      const int q = wp * 64 + j * 16 + lr;
      const int ty = q / OW, tx = q - ty * OW;
      pbase[j] = (ty * STEM_S * IC + tx * STEM_S) * 3;  // region offset of the patch's (0, 0, 0)
    }
    f32x4 acc[WC][WP];
#pragma unroll
    for (int i = 0; i < WC; ++i)
#pragma unroll
      for (int j = 0; j < WP; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll 1  // (fully unrolled: 256 VGPRs, 175 vs 169 us)
    for (int ks = 0; ks < STEM_KP / 32; ++ks) {
      // weight fragments (rows i * 16 + lr, k = ks * 32 + 8 g ..)
      uint4 af[WC][NPL];
#pragma unroll
      for (int i = 0; i < WC; ++i)
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) af[i][pl] = wl[((ks * WC + i) * NPL + pl) * 64 + lane];
      // the region offsets of this lane's 8 patch elements kk = ks * 32 + 8 g + e (kk >= 147: zero)
      int eo[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int kk = ks * 32 + g * 8 + e;
        const int t = kk / STEM_C, c = kk - t * STEM_C;
        const int ky = t / STEM_K, kx = t - ky * STEM_K;
        eo[e] = kk < STEM_K * STEM_K * STEM_C ? (ky * IC + kx) * 3 + c : -1;
      }
#pragma unroll
      for (int j = 0; j < WP; ++j) {
        uint32_t hw[NPL][4];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const uint32_t w0 = eo[e] >= 0 ? region[pbase[j] + eo[e]] : 0u;
          const uint32_t w1 = eo[e + 1] >= 0 ? region[pbase[j] + eo[e + 1]] : 0u;
          hw[0][e >> 1] = (w0 & 0xffffu) | (w1 << 16);           // the two hi halves
          hw[1][e >> 1] = (w0 >> 16) | (w1 & 0xffff0000u);       // the two lo' halves
        }
        const uint4 bh = make_uint4(hw[0][0], hw[0][1], hw[0][2], hw[0][3]);
        const uint4 bl = make_uint4(hw[1][0], hw[1][1], hw[1][2], hw[1][3]);
#pragma unroll
        for (int i = 0; i < WC; ++i) {
          f32x4 c2 = (f32x4){0.f, 0.f, 0.f, 0.f};
          MT::mma(c2, af[i][0], bl);
          MT::mma(c2, af[i][1], bh);
          MT::mma(acc[i][j], af[i][0], bh);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] = __builtin_fmaf(c2[r], SP::CS, acc[i][j][r]);
        }
      }
    }
    // epilogue: BN scale / shift, ReLU, split; lane groups of cout blocks (i, i + 1) paired so a lane
    // holds 8 consecutive channels of one pixel (16 B stores per plane)
#pragma unroll
    for (int i = 0; i < WC; i += 2) {
      const int cs = (i + (g & 1)) * 16 + (g >> 1) * 8;
      float sc[8], sh[8];
      const float4 s0 = *(const float4*)(scale + cs), s1 = *(const float4*)(scale + cs + 4);
      const float4 h0 = *(const float4*)(shift + cs), h1 = *(const float4*)(shift + cs + 4);
      sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w; sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
      sh[0] = h0.x; sh[1] = h0.y; sh[2] = h0.z; sh[3] = h0.w; sh[4] = h1.x; sh[5] = h1.y; sh[6] = h1.z; sh[7] = h1.w;
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
        const int q = wp * 64 + j * 16 + lr;
        const int oy = oy0 + q / OW, ox = q % OW;
        uint32_t o[NPL][4];
#pragma unroll
        for (int r = 0; r < 8; r += 2) {
          const float a = fmaxf(v[r] * sc[r] + sh[r], 0.f), b = fmaxf(v[r + 1] * sc[r + 1] + sh[r + 1], 0.f);
          unsigned short q0[NPL], q1[NPL];
          SP::split(a, q0);
          SP::split(b, q1);
          bad |= h2_overflow(a) || h2_overflow(b);
#pragma unroll
          for (int pl = 0; pl < NPL; ++pl) o[pl][r >> 1] = (uint32_t)q0[pl] | ((uint32_t)q1[pl] << 16);
        }
        unsigned short* Y = y + (((size_t)n * OH + oy) * OW + ox) * ldy + cy0 + cs;
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) *(uint4*)(Y + pl * psy) = make_uint4(o[pl][0], o[pl][1], o[pl][2], o[pl][3]);
      }
    }
  }  // tiles
  raise_range_flag(rflag, bad);
}

}  // namespace zp

using namespace zp;

// zp_conv_tuning key 20: persistent stem workgroups per CU (1 or 2; -1: ZP_STEM_WGS or 1).  Measured
// (whole fp32 forward, bs 32, hipGraph, tools/bs1_ab.py): 9.392 ms with one, 9.419 with two -- one stays
static int g_stem_wgs = -1;
namespace zp {
int stem_wgs_mode(int v) {
  const int old = g_stem_wgs;
  g_stem_wgs = v;
  return old;
}
}  // namespace zp
static int stem_wgs_per_cu() {
  static const int env = getenv("ZP_STEM_WGS") ? atoi(getenv("ZP_STEM_WGS")) : 1;
  const int v = g_stem_wgs >= 0 ? g_stem_wgs : env;
  return v == 2 ? 2 : 1;
}

extern "C" int zp_stem_split(const float* x, int B, int H, int W, int ldx, const void* w, int w_rows, int k_pad,
                             const float* scale, const float* shift, int dtype, void* y, int ldy, int cy0, int OH,
                             int OW, void* stream) {
  ZP_CHECK_ARG(dtype == ZP_F32H2, "zp_stem_split: dtype %d (the two-plane form only)", dtype);
  ZP_CHECK_ARG(x && w && scale && shift && y && B > 0 && H > 0 && W > 0, "zp_stem_split: bad args");
  ZP_CHECK_ARG(ldx == 0 || (ldx >= 4 && ldx % 4 == 0),
               "zp_stem_split: input ldx %d (0: NCHW [B][3][H][W]; else f32 NHWC, 16-byte pixels)", ldx);
  ZP_CHECK_ARG(k_pad == STEM_KP && w_rows >= 64, "zp_stem_split: weights [2][w_rows >= 64][160] (got %d / %d)", w_rows,
               k_pad);
  ZP_CHECK_ARG(OH == (H + 2 * STEM_P - STEM_K) / STEM_S + 1 && OW == (W + 2 * STEM_P - STEM_K) / STEM_S + 1,
               "zp_stem_split: OH / OW");
  ZP_CHECK_ARG(OW <= 128 && 256 % OW == 0 && (OH * OW) % 256 == 0, "zp_stem_split: OW %d must divide 256, <= 128", OW);
  ZP_CHECK_ARG(ldy % 8 == 0 && cy0 % 8 == 0 && ldy >= cy0 + 64, "zp_stem_split: ldy / cy0");
  const int TR = 256 / OW;
  const size_t npix = (size_t)(STEM_S * TR + STEM_K - STEM_S) * (STEM_S * OW + STEM_K - STEM_S);
  ZP_CHECK_ARG(npix <= 2560, "zp_stem_split: input region of %zu pixels (the prefetch holds 2560)", npix);
  const size_t lds = ((npix * 3 + 3) & ~(size_t)3) * sizeof(float) + (size_t)(STEM_KP / 32) * 4 * 2 * 64 * 16;
  ZP_CHECK_ARG(lds <= 80 * 1024, "zp_stem_split: region + weights %zu B", lds);
  // dynamic LDS beyond 64 KB: the attribute is set once per device (it may be per device;
  // a process can drive several GPUs), and a failure is reported as such
  static bool attr[64] = {};
  static int cus[64] = {};
  int dev = 0;
  ZP_CHECK_ARG(hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64, "zp_stem_split: no current device");
  if (!attr[dev]) {
    ZP_CHECK_ARG(hipFuncSetAttribute((const void*)k_stem_h2<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024) ==
                         hipSuccess &&
                     hipFuncSetAttribute((const void*)k_stem_h2<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         80 * 1024) == hipSuccess,
                 "zp_stem_split: hipFuncSetAttribute(MaxDynamicSharedMemorySize, 80 KB) failed on device %d", dev);
    ZP_CHECK_ARG(hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus[dev] > 0,
                 "zp_stem_split: CU count of device %d", dev);
    attr[dev] = true;
  }
  const long tiles = (long)B * OH * OW / 256;
  // persistent workgroups, each walking ~tiles / grid tiles with the next tile's region in flight
  // during the current one's MFMAs: stem_wgs_per_cu() per CU (zp_conv_tuning key 20; 200 VGPRs and
  // ~69 KB of LDS let two share a CU)
  const long wgs = (long)cus[dev] * stem_wgs_per_cu();
  const unsigned grid = (unsigned)(tiles < wgs ? tiles : wgs);
  const long psy = (long)B * OH * OW * ldy;
  if (ldx == 0)
    hipLaunchKernelGGL(k_stem_h2<true>, dim3(grid), dim3(256), lds, (hipStream_t)stream, x, B, H, W, ldx,
                       (const unsigned short*)w, w_rows, scale, shift, (unsigned short*)y, ldy, cy0, OH, OW, psy,
                       range_flag());
  else
    hipLaunchKernelGGL(k_stem_h2<false>, dim3(grid), dim3(256), lds, (hipStream_t)stream, x, B, H, W, ldx,
                       (const unsigned short*)w, w_rows, scale, shift, (unsigned short*)y, ldy, cy0, OH, OW, psy,
                       range_flag());
  ZP_LAUNCH_CHECK("zp_stem_split");
  return ZP_OK;
}
