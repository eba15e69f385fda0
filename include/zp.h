/*
 * zp.h -- C ABI of libzp.so, the MI355X (gfx950) implementation of ZebraPose's
 * data-parallel hot path.
 *
 * Plain C: pointers, sizes and POD structs only; no torch types.  Every pointer
 * argument named x / y / w / res / ... is a DEVICE pointer (caller-owned memory,
 * e.g. the PyTorch caching allocator); `stream` is a hipStream_t (NULL = legacy
 * default stream).  All calls are stream-ordered and never synchronise the host.
 * Return value: 0 (ZP_OK) or an error code; zp_last_error() describes the last
 * failure of the calling thread.
 *
 * Layouts.  Activations are NHWC ("channels last") with a row stride `ld*`
 * (elements per pixel) and a channel offset `c*0`, so a producer can write
 * straight into a channel slice of a concat buffer (the reference's torch.cat,
 * aspp.py:101-112).  Packed conv weights are [rows_pad][k_pad] with
 * k = tap * Cin + cin ("tap-major implicit GEMM").
 *
 * Reference interfaces replaced (file:line in lyltc1/ZebraPose):
 *   zp_conv2d          nn.Conv2d / nn.ConvTranspose2d + BatchNorm2d + ReLU (+ residual add)
 *                      as called at model/resnet.py:41-51, torchvision resnet children
 *                      (resnet.py:191-199), model/aspp.py:60-80, 89-112
 *   zp_conv2d_wgrad    their weight gradients (autograd of the same modules, train_v6.py:337)
 *   zp_bn_*            BatchNorm2d train/eval semantics (resnet.py:29, aspp.py:12..)
 *   zp_maxpool3s2      torchvision maxpool (resnet.py:197), and its backward
 *   zp_global_avgpool  aspp.py:94  AdaptiveAvgPool2d(1)   (+ zp_broadcast_hw = aspp.py:96 bilinear 1x1->HxW)
 *   zp_code_loss       BinaryCodeLoss / HammingLoss / BinaryLossWeighted (model/BinaryCodeNet.py:8-81,
 *                      96-109) as driven at train_v6.py:325-327;  zp_mask_loss  MaskLoss (:84-93)
 *   zp_threshold       common_ops.py:5-19 (sigmoid > 0.5 -> {0,1})
 *   zp_decode          binary_code_helper/CNN_output_to_pose.py:34-64, 100-130 and
 *                      class_id_encoder_decoder.py:17-28 (bits -> id -> LUT -> 2D/3D)
 *   zp_lut_coarsen     binary_code_helper/generate_new_dict.py:4-33 (ignore_bit LUT)
 *   zp_adam            torch.optim.Adam step used by train_v6.py:268-269, 338
 */
#ifndef ZP_H_
#define ZP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZP_ABI_VERSION 4

#define ZP_OK 0
#define ZP_ERR_ARG 1
#define ZP_ERR_HIP 2

/* element types of activations / packed weights */
#define ZP_F32 0
#define ZP_BF16 1
#define ZP_F16 2 /* IEEE fp16 storage + v_mfma_f32_16x16x32_f16; inference (forward) kernels only */
/* fp32 in split form (eval-mode inference): a tensor is THREE contiguous bf16 planes [3][...], the
 * pointer names plane 0, plane p starts p plane-sizes later (plane size = the tensor's element
 * count: N*H*W*ld for an activation, rows_pad*k_pad for packed weights, N*C for a pooled vector).
 * v = hi + mid + lo exactly (hi = bf16(v), mid = bf16(v - hi), lo = bf16(v - hi - mid)).  zp_conv2d
 * forms every product a*b from the six terms of magnitude >= 2^-16 |a b| (hi*hi, hi*mid, mid*hi,
 * hi*lo, mid*mid, lo*hi) on bf16 MFMAs with f32 accumulation: the dropped terms are below
 * 2^-23 |a b| (f32's own product rounding is 2^-24), i.e. f32-accurate convolutions at 6/16 of the
 * f32-MFMA cost.  Forward (eval) kernels only. */
#define ZP_F32X3 3
/* fp32 in the two-plane fp16 split form (eval-mode inference), laid out like ZP_F32X3 with TWO
 * planes [2][...] of IEEE fp16: hi = fp16(v), lo = fp16((v - hi) * 2^11), v = hi + lo * 2^-11 to
 * 22 significant bits (|error| <= 2^-23 |v| in fp16's normal range; |v| must stay below 65504).
 * zp_conv2d forms a*b from hi*hi + (hi*lo + lo*hi) * 2^-11 on fp16 MFMAs (the dropped lo*lo term is
 * below 2^-22 |a b|): 3 MFMAs and 2 staged planes per product instead of ZP_F32X3's 6 and 3.
 * Forward (eval) kernels only. */
#define ZP_F32H2 4

/* Range guard of ZP_F32H2.  A finite value at or above 65520 in magnitude has no two-plane form
 * (hi rounds to fp16 infinity); a WEIGHT at or above 32 (65504 / 2^11) has none for the wide-tile
 * conv, which forms 2^11 * hi in fp16.  Every ZP_F32H2 store -- the zp_conv2d epilogues (split-K's
 * included), zp_im2col_split, the f32 stem writing ZP_OUT_NHWC_H2 and zp_pack_weight(_multi), the
 * latter with the weight bound -- sets *flag = 1 (a device word) when it meets one; nothing clears it.  The flag is per device
 * (the calling thread's current device at registration; launches read it at enqueue time, so a
 * captured hipGraph keeps the word of its capture).  NULL unregisters.  The max / average pools and
 * broadcasts of split tensors cannot leave the range of their inputs and do not check.  The Python
 * engine registers one word, reads it once per fp32 eval forward and re-runs an overflowing forward
 * on the full-range ZP_F32X3 form (reference forward: model/BinaryCodeNet.py:161-174, plain f32). */
int zp_split_range_flag(unsigned int* flag);

/* zp_conv_args.out_mode */
#define ZP_OUT_NHWC 0       /* y[n, oy, ox, cy0 + c] (ldy elements per pixel), dtype of the call */
#define ZP_OUT_HEAD_NCHW 1  /* c == 0 -> y (f32 [N,1,OH,OW]); c >= 1 -> y2 (f32 [N,Cout-1,OH,OW]) */
#define ZP_OUT_NHWC_F32 2   /* y f32 NHWC regardless of dtype (raw conv output for train-mode BN) */
#define ZP_OUT_NHWC_X3 3    /* y = plane 0 of a ZP_F32X3 NHWC tensor (an f32 call writing split output) */
#define ZP_OUT_NHWC_H2 4    /* y = plane 0 of a ZP_F32H2 NHWC tensor (an f32 call writing split output) */

#define ZP_MAX_TAPS 64
#define ZP_MAX_SUB 4

/* One implicit-GEMM sub-problem.  Grid point (n, gy, gx), tap t reads input pixel
 * (gy*sy + ty[t], gx*sx + tx[t]) (zero outside) and writes output pixel
 * (gy*oys + oyo, gx*oxs + oxo).  This covers strided/dilated convs, the four
 * sub-pixel phases of ConvTranspose2d(3, s2, p1, op1), and the data-gradient
 * convs of both. */
typedef struct zp_conv_sub {
  const void* w;        /* packed weights [rows_pad][k_pad], dtype of the call */
  const float* scale;   /* per-output-channel multiplier (folded BN) or NULL (=1) */
  const float* shift;   /* per-output-channel addend (folded BN + bias) or NULL (=0) */
  void* y;              /* output (see out_mode) */
  void* y2;             /* second output (ZP_OUT_HEAD_NCHW) */
  int ldy, cy0, OH, OW;
  int oys, oyo, oxs, oxo;
  int ntaps;            /* taps in ty/tx (general path) */
  int kw, dil, pad;     /* arithmetic taps for the small-Cin path: t -> ((t/kw)*dil-pad, (t%kw)*dil-pad) */
  signed char ty[ZP_MAX_TAPS];
  signed char tx[ZP_MAX_TAPS];
} zp_conv_sub;

typedef struct zp_conv_args {
  int dtype;            /* ZP_F32 (exact-f32 MFMA path), ZP_BF16 or ZP_F16 (16-bit MFMA, fp32 accumulate),
                           ZP_F32X3 (split fp32: x / w / res in 3 planes, Cin a multiple of 32) */
  const void* x;        /* input NHWC */
  int ldx, cx0, IH, IW, Cin;   /* Cin: multiple of 64 (bf16) / 32 (f32), or 8 (small-Cin path) */
  int N, GH, GW, sy, sx;       /* GEMM grid (pixels) and input stride */
  int Cout, k_pad;             /* k_pad: weight row length (elements) */
  int w_rows;                  /* packed weight rows (>= Cout, multiple of the cout tile: use
                                  zp_conv_rows_pad(Cout)) */
  const void* res;             /* residual NHWC (same pixel as y) or NULL */
  int ldr, cr0;
  int relu, out_mode;
  float* stats;                /* if non-NULL (raw output only: no scale/shift/res/relu): per-channel
                                  partial statistics of the stored value, [3][parts][Cout] =
                                  (count, mean, centred M2), parts = zp_conv2d_stat_parts() */
  int nsub;
  zp_conv_sub sub[ZP_MAX_SUB];
  /* ABI 3.  Data-gradient launches (ZP_F32 / ZP_BF16, NHWC, no scale / shift / residual / ReLU / stats):
   * if bnr_part is non-NULL the launch also takes the reduce of zp_bn_bwd_reduce (relu mode 2) for the
   * train-mode BatchNorm whose OUTPUT gradient it writes -- g = the stored value, masked by
   * fma(x, save scale, save shift) > 0, xhat = (x - mean) * invstd -- per stat part:
   * partials[0][k][c] = sum g, partials[1][k][c] = sum g * xhat over stat part k, in the
   * [2][parts + 1][Cout] layout of zp_bn_bwd_reduce with parts = zp_conv2d_bnr_parts(); finish with
   * zp_bn_bwd_totals.
   * Valid only when this launch is the gradient's only writer (it overwrites every pixel).
   * Replaces the separate reduce pass of the BN backward (reference model/resnet.py:41-51, autograd
   * of nn.BatchNorm2d + ReLU) */
  const void* bnr_x;       /* that BN's raw conv output x [P][Cout] (dtype) */
  const float* bnr_save;   /* its zp_bn_train_finalize save: mean, invstd, scale, shift ([4][Cout]) */
  float* bnr_part;
} zp_conv_args;

int zp_abi_version(void);
const char* zp_last_error(void);

/* ---- convolution (forward and data-gradient) ---------------------------------------- */
int zp_conv2d(const zp_conv_args* a, void* stream);
/* packed weight row count zp_conv2d expects for Cout output channels */
int zp_conv_rows_pad(int Cout);
/* number of pixel tiles (grid_x) a zp_conv2d launch with these args uses */
int zp_conv2d_grid(const zp_conv_args* a);
/* number of partial-sum slots `stats` needs: one per pixel tile and sub-problem (round 5: the conv
 * kernels merge their wave halves in LDS first; the split-fp32 forms and k_conv_strip, ZP_CONV_FLAGS
 * without 64, keep one per wave half: (pixel tile / 64) * grid_x * nsub) */
int zp_conv2d_stat_parts(const zp_conv_args* a);
/* number of partial-sum slots a launch with bnr_part emits: zp_conv2d_stat_parts, or one per
 * 256-pixel tile where the strip kernel sums its wave halves first (ABI 3) */
int zp_conv2d_bnr_parts(const zp_conv_args* a);
/* launch configuration zp_conv2d picks: cout tile, pixel tile, LDS ring depth, kernel variant
 * (0 = k_conv, 1 = k_conv_strip: 3x3 stride-1 convs with activation-strip reuse, 2 = k_conv_strip2:
 * the same with the lean main loop, 3 = k_conv_quad: the four phases of a stride-2 transposed
 * structure in one tile, 4 = k_conv3: the split-fp32 (ZP_F32X3) kernel, 5 = k_conv3s: its 3x3
 * stride-1 form with activation-strip reuse, 6 = k_conv3w: the 256 x 256 two-plane tile, 7 = k_conv1x1n: a
 * 1x1 with 32 / 64 input channels and a wide output, the weights held in LDS) */
int zp_conv2d_config(const zp_conv_args* a, int* tc, int* tp, int* stages, int* variant);
/* Split-fp32 forms (ZP_F32X3 / ZP_F32H2) only: a launch whose grid would leave most CUs idle (an
 * NHWC conv -- one sub-problem or several: ConvT phases, merged ASPP branches -- with under 256
 * workgroups, e.g. bs = 1) is cut along K into slices whose f32
 * sums are finished (summed in slice order, then BN / residual / ReLU / split store) by a second
 * kernel, when zp_conv_args.stats points to an f32 workspace of this many bytes (0: not split;
 * stats NULL: not split).  Deterministic. */
long long zp_conv2d_split_ws(const zp_conv_args* a);
/* runtime tuning knobs (tests / sweeps): key 0 = minimum workgroup count for the 256-channel
 * tile (default 1024); key 1 = conv schedule flags (-1 = ZP_CONV_FLAGS or the default); key 2 =
 * 64-channel layers on the strip kernel (default 1); key 3 = the lean weight-gradient kernel
 * (default 1); key 4 = its workgroup rounds over the CUs (default 1); key 5 = the general
 * weight-gradient kernel's workgroup rounds (default 1; 0 = a ~1024-workgroup target); key 6 = the
 * fewest workgroups the four-phase kernel (k_conv_quad) runs with (default 256); key 7 = the
 * split-fp32 strip kernel k_conv3s (0 off, 1 64-channel tiles, 2 also 128-channel tiles; -1 =
 * ZP_CONV3_STRIP or the default 1); key 8 = the fewest workgroups a split-fp32 launch runs
 * 128-channel tiles with (fewer: 64-channel tiles); key 9 = split-K of small split-fp32 launches
 * (default 1, 0 off); keys 10-12 = the 256 x 256 two-plane tile (on / fewest workgroups / split-K);
 * key 13 = its accumulation form (0 the flushed correction accumulator, default; 1 one scaled
 * accumulator; 2 per-step partial sums; 3 flushed on the 2^11 scale); key 14 = its 256 x 128 tile
 * (default 0); key 15 = zp_bn_train_finalize's merge in one launch (1, default) or two (0); key 16 =
 * k_conv3's multi-sub launches with a tile's subs adjacent on one XCD (default 0); key 17 = k_conv3w's
 * multi-sub launches (ConvT phases) with a pixel tile's phases adjacent on one XCD (default 0); key 18
 * = the 256 x 256 two-plane tile on 32x32x16 MFMAs (default 0); key 19 = the ring depth (2, 3, 4) of
 * the register-pipelined two-plane 64-channel tile (default 2); key 20 = persistent workgroups per CU
 * of the two-plane stem (1 or 2, default 1); key 21 = the wide strip tile's next-step pixel fragments
 * read before the step's barrier (1, default) or after it (0).  Returns the previous value, -1 for an
 * unknown key. */
int zp_conv_tuning(int key, int value);

/* Fused 1x1 head (the reference's conv_1x1_4 over torch.cat([x, x_128]) and the mask / code split,
 * model/aspp.py:112 + model/BinaryCodeNet.py:172).  The conv of *a (one sub, NHWC, BN scale / shift,
 * bias, residual and ReLU applied as by zp_conv2d) is NOT stored: each output pixel's Cout channels,
 * followed by the C2 channels of x2 at the same pixel (NHWC of a's dtype, [N][OH][OW][ldx2], channels
 * cx20..), feed a 1x1 conv with hcout <= 32 outputs: weights w packed by zp_pack_weight(a's dtype,
 * rows_pad 32, k = channel, k_pad >= Cout + C2), bias (f32 [hcout] or NULL).  Output f32 NCHW:
 * channel 0 -> mask [N][1][OH][OW], channels 1.. -> code [N][hcout-1][OH][OW].
 *   ZP_F32H2: the 256 x 256 two-plane tile runs the conv and the whole head (one launch).
 *   ZP_BF16 / ZP_F16 (eval, ABI 2): the 3x3 conv runs on the strip tile (two 128-channel cout tiles);
 *   each tile's head sums over its channels (the first tile's also over x2) go to ws, f32
 *   [2][32][N*OH*OW] (zp_conv2d_head_ws bytes), and a second launch adds the two in a fixed order,
 *   plus the bias: deterministic.
 * zp_conv2d_head_ok: 1 if *a has a geometry the fused kernels take (e.g. not at bs = 1 for
 * ZP_F32H2, where the unfused path runs). */
typedef struct zp_head_args {
  const void* w;
  int k_pad;
  const float* bias;
  int cout;
  const void* x2;
  int ldx2, cx20, C2;
  float* mask;
  float* code;
  float* ws;  /* ABI 2: the 16-bit path's partial sums (zp_conv2d_head_ws bytes); ignored by ZP_F32H2 */
} zp_head_args;
int zp_conv2d_head_ok(const zp_conv_args* a);
long long zp_conv2d_head_ws(const zp_conv_args* a);
int zp_conv2d_head(const zp_conv_args* a, const zp_head_args* h, void* stream);

/* Pack an f32 weight tensor src[d0][d1][kh][kw] into dst[rows_pad][k_pad] (dtype), taps
 * (ky[t], kx[t]), t < ntaps:
 *   transposed == 0: dst[r][t*cstride + c] = src[r][c][ky[t]][kx[t]]   (conv forward: OIHW)
 *   transposed == 1: dst[r][t*cstride + c] = src[c][r][ky[t]][kx[t]]   (ConvT forward, conv dgrad)
 * ky/kx are HOST arrays (<= ZP_MAX_TAPS).  Padding rows / columns / channels are zeroed. */
int zp_pack_weight(const float* src, int d0, int d1, int kh, int kw, int transposed, int ntaps,
                   const int* ky, const int* kx, int cstride, int dtype, void* dst, int rows_pad,
                   int k_pad, void* stream);

/* Many zp_pack_weight jobs in one launch (training repacks every conv's weights once per
 * optimizer step).  `jobs` and `prefix` are DEVICE arrays: prefix[i] = sum of rows_pad*k_pad of
 * jobs before i (prefix[n] = total elements; validated, the kernel maps one grid row per job,
 * n <= 65535).  Same element mapping as zp_pack_weight. */
typedef struct zp_pack_job {
  const float* src;
  void* dst;
  int d0, d1, kh, kw, transposed, ntaps, cstride, rows_pad, k_pad, dtype;
  signed char ky[ZP_MAX_TAPS], kx[ZP_MAX_TAPS];
} zp_pack_job;
int zp_pack_weight_multi(int n, const zp_pack_job* jobs, const long long* prefix, long long total,
                         void* stream);

/* ---- weight gradient ------------------------------------------------------------------
 * dw[co][ci][ky][kx] (f32, layout of the conv's own weight; transposed_w=1 for ConvT's
 * [ci][co][kh][kw]) = sum over grid points and taps of dy[out pixel][co] * x[in pixel][ci],
 * with the same sub/tap geometry as the forward zp_conv_args (sub[].y = dy, dtype = act dtype).
 * `ws` is a device workspace of zp_conv2d_wgrad_ws_bytes() bytes. accumulate != 0 adds to dw. */
typedef struct zp_wgrad_args {
  int dtype;
  const void* x; int ldx, cx0, IH, IW, Cin;
  int N, GH, GW, sy, sx;
  int Cout;
  int Cw;                      /* input channels of the weight tensor (<= Cin; Cin may be padded) */
  int kh, kw, transposed_w;
  int nsub;
  struct {
    const void* dy; int lddy, cdy0, OH, OW, oys, oyo, oxs, oxo;
    int ntaps;
    signed char ky[ZP_MAX_TAPS], kx[ZP_MAX_TAPS];   /* weight tap of each geometric tap */
    signed char ty[ZP_MAX_TAPS], tx[ZP_MAX_TAPS];
  } sub[ZP_MAX_SUB];
  float* dw;
  int accumulate;
} zp_wgrad_args;
long long zp_conv2d_wgrad_ws_bytes(const zp_wgrad_args* a);
int zp_conv2d_wgrad(const zp_wgrad_args* a, void* ws, void* stream);

/* ---- batch norm ---------------------------------------------------------------------- */
/* eval: scale = gamma / sqrt(var + eps); shift = beta + (bias - mean) * scale (bias may be NULL) */
int zp_bn_fold(const float* gamma, const float* beta, const float* mean, const float* var,
               const float* conv_bias, float eps, int C, float* scale, float* shift, void* stream);
/* train: merge the [3][parts][C] partial statistics of zp_conv2d(stats) (count = P, checked),
 * update running stats (momentum, unbiased var; the conv bias, if any, is added to the mean)
 * and emit scale/shift for the apply pass, plus save[4][C] = (mean, invstd, scale, shift) of the
 * raw values (shift = fma(-mean, scale, beta)).
 * partials is scratch: a first merge level overwrites it in place (every 64th part).
 * ABI 4: partials holds zp_bn_finalize_floats(parts, C) floats -- the [3][parts][C] statistics and,
 * past them, the one-launch merge's per-launch hand-off counters (zeroed on `stream` by this call),
 * so concurrent finalizes on different streams or hipGraphs never share counters. */
int zp_bn_train_finalize(float* partials, int parts, int C, long long count, float eps,
                         float momentum, const float* gamma, const float* beta, const float* conv_bias,
                         float* running_mean, float* running_var, int64_t* num_batches_tracked,
                         float* scale, float* shift, float* save, void* stream);
/* size in floats of zp_bn_train_finalize's partials buffer for (parts, C) (ABI 4) */
long long zp_bn_finalize_floats(int parts, int C);
/* y[p, cy0+c] = act(fma(x[p, c], scale[c], shift[c]) (+ res[p, cr0+c])), x: raw conv output [P][C] */
int zp_bn_apply(const void* x, int P, int C, const float* scale, const float* shift,
                const void* res, int ldr, int cr0, int relu, int dtype, void* y, int ldy, int cy0,
                void* stream);
/* number of partial slots zp_bn_bwd_reduce uses for P pixels (partials needs [2][parts+1][C]) */
int zp_bn_bwd_parts(int P, int C);
/* backward of y = act(bn(x) (+res)):  g = dy * mask;  xhat = (x - mean) * invstd;
 * relu 0: no mask; 1: mask = y > 0 (y read); 2: mask = fma(x, save scale, save shift) > 0, recomputed
 * from the raw x exactly as zp_bn_apply formed y (no residual) -- y is not read and may be NULL;
 * partials[0][k][c] = sum g, partials[1][k][c] = sum g*xhat over pixel block k (x == NULL: only sum g);
 * then totals into partials[.][parts][c] and (optional) dgamma = sum g*xhat, dbeta = sum g
 * (written, or added if accumulate). */
int zp_bn_bwd_reduce(const void* dy, int lddy, int cdy0, const void* y, int ldy, int cy0,
                     const void* x, int P, int C, const float* save, int relu, int dtype,
                     float* partials, float* dgamma, float* dbeta, int accumulate, void* stream);
/* totals of partials [2][parts + 1][C] filled by a zp_conv2d launch with bnr_part (parts =
 * zp_conv2d_bnr_parts) -> partials[0][out_parts][c], partials[1][out_parts][c] of the [2][out_parts
 * + 1][C] layout zp_bn_bwd_apply reads (out_parts = zp_bn_bwd_parts(P, C); the buffer holds
 * [2][max(parts, out_parts) + 1][C]); dgamma / dbeta as zp_bn_bwd_reduce */
int zp_bn_bwd_totals(float* partials, int parts, int C, int out_parts, float* dgamma, float* dbeta,
                     int accumulate, void* stream);
/* dx[p][c] = gamma*invstd*(g - sum_g/P - xhat*sum_gx/P)  (dx dtype, [P][C]); relu as for the
 * reduce (mode 2 needs dx);
 * dres (optional) [p, cdres0+c] = g, or += g if res_accumulate */
int zp_bn_bwd_apply(const void* dy, int lddy, int cdy0, const void* y, int ldy, int cy0,
                    const void* x, int P, int C, const float* save, const float* partials,
                    const float* gamma, int relu, int dtype, void* dx, void* dres, int lddres,
                    int cdres0, int res_accumulate, void* stream);

/* ---- layout / pooling ---------------------------------------------------------------- */
/* x f32 NCHW [B][C][H][W] -> y NHWC [B][H][W][cpad] (dtype), channels C..cpad-1 zero */
int zp_nchw_to_nhwc(const float* x, int B, int C, int H, int W, int cpad, int dtype, void* y,
                    void* stream);
/* Split-fp32 stem input (ZP_F32X3 / ZP_F32H2): the im2col of an f32 NHWC image x [B][H][W][ldx]
 * (C real channels) for a k x k / stride s / padding p conv -- y [NPL][B][OH][OW][kpad] with
 * element kk = (ky * k + kx) * C + c (kk >= k*k*C and out-of-image taps zero), stored split.  The
 * stem conv (torchvision ResNet conv1 7x7/s2/p3, reference model/resnet.py:195) then runs as a 1x1
 * split-fp32 conv over kpad channels, weights packed with zp_pack_weight(..., cstride = C, ...). */
int zp_im2col_split(const float* x, int B, int H, int W, int ldx, int C, int k, int s, int p, int OH, int OW,
                    int kpad, int dtype, void* y, void* stream);
/* The stem conv of the two-plane engine in one launch (ZP_F32H2 only): torchvision conv1 (7x7,
 * stride 2, pad 3, 3 -> 64 channels; reference model/resnet.py:195) + folded BN (scale, shift) +
 * ReLU, from the f32 image x -- ldx == 0: NCHW [B][3][H][W], the reference's input tensor
 * (bop_dataset_pytorch.py:345; no zp_nchw_to_nhwc copy); else NHWC [B][H][W][ldx] (channels 0..2, ldx a
 * multiple of 4) -- to a ZP_F32H2 NHWC slice y [2][B][OH][OW][ldy] at channel cy0.  Weights:
 * zp_pack_weight of the 7x7 kernel in the zp_im2col_split order (taps row-major, cstride 3, k_pad 160,
 * dtype ZP_F32H2, w_rows >= 64).  Replaces zp_im2col_split + the 1x1 split GEMM (no patch tensor).
 * OW must divide 256 and be <= 128. */
int zp_stem_split(const float* x, int B, int H, int W, int ldx, const void* w, int w_rows, int k_pad,
                  const float* scale, const float* shift, int dtype, void* y, int ldy, int cy0, int OH, int OW,
                  void* stream);
/* 3x3 / stride 2 / pad 1 max pool, NHWC slices; C multiple of 8 */
int zp_maxpool3s2(const void* x, int B, int IH, int IW, int ldx, int cx0, int C, int dtype,
                  void* y, int OH, int OW, int ldy, int cy0, void* stream);
int zp_maxpool3s2_bwd(const void* x, int ldx, int cx0, const void* dy, int lddy, int cdy0,
                      int B, int IH, int IW, int C, int OH, int OW, int dtype,
                      void* dx, int lddx, int cdx0, int accumulate, void* stream);
/* y[b][c] = mean over H*W of x (f32 accumulate), y dtype */
int zp_global_avgpool(const void* x, int B, int H, int W, int ldx, int cx0, int C, int dtype,
                      void* y, void* stream);
/* y[b, :, :, cy0 + c] = src[b][c] */
int zp_broadcast_hw(const void* src, int B, int C, int dtype, void* y, int H, int W, int ldy, int cy0,
                    void* stream);
/* backward of zp_broadcast_hw: out[b][c] (dtype) = sum over H*W of dy[b, h, w, cdy0 + c] */
int zp_sum_hw(const void* dy, int B, int H, int W, int lddy, int cdy0, int C, int dtype, void* out,
              void* stream);
/* backward of zp_global_avgpool: y[b, h, w, cy0 + c] (+)= src[b][c] * mul  (src dtype) */
int zp_add_broadcast_hw(const void* src, float mul, int B, int C, int dtype, void* y, int H, int W,
                        int ldy, int cy0, int accumulate, void* stream);
/* generic NHWC slice copy / add / cast: y[p, cy0+c] (+)= x[p, cx0+c]  */
int zp_copy_slice(const void* x, int ldx, int cx0, int xdtype, void* y, int ldy, int cy0, int ydtype,
                  int P, int C, int accumulate, void* stream);
/* F.interpolate(mask, (OH, OW), mode="bilinear", align_corners=False) of a one-channel f32 NCHW
 * map into channel cy0 of an NHWC concat buffer (BinaryCodeNet_Deeplab_v3: aspp_v3.py:89, 96-101),
 * and its backward (gather form, deterministic) into f32 NCHW dx (accumulate: dx += ...). */
int zp_mask_interp(const float* x, int B, int H, int W, int OH, int OW, int dtype, void* y, int ldy, int cy0,
                   void* stream);
int zp_mask_interp_bwd(const void* dy, int lddy, int cdy0, int B, int OH, int OW, int H, int W, int dtype, float* dx,
                       int accumulate, void* stream);
/* head gradient f32 NCHW (dmask [B][1][H][W], dcode [B][L][H][W]) -> y NHWC [B][H][W][ldy]
 * (dtype), channel 0 = mask, 1..L = code, channels L+1..ldy-1 zeroed */
int zp_head_grad_to_nhwc(const float* dmask, const float* dcode, int B, int L, int H, int W, int ldy,
                         int dtype, void* y, void* stream);

/* ---- loss ---------------------------------------------------------------------------- */
/* loss_b of BinaryCodeLoss('BCE', mask_binary_code_loss=mask_code, 2, use_hist)
 * (model/BinaryCodeNet.py:34-81 with HammingLoss :100-109), f64 like the reference:
 *   code_logits f32 [B][L][H][W];
 *   mask: mask01 (f64 [B][1][H][W], rounded and clamped to {0,1} as HammingLoss does) or, if
 *         mask01 == NULL, mask_logits (f32 [B][1][H][W]) thresholded like train_v6.py:325-326;
 *   gt [B][L][H][W]: f64 if gt_f64 else u8 (0/1);
 *   hist_state f64[L+1]: [0..L) the histogram EMA (module state), [L] = 0 before the first call;
 *   out f64[2] = (loss_b, mean hamming loss); coef f64[L] = w_i / sum(w) / (B*H*W), kept for the
 *   backward.  ws: zp_code_loss_ws_bytes(B, L, H, W) bytes. */
long long zp_code_loss_ws_bytes(int B, int L, int H, int W);
int zp_code_loss(const float* code_logits, const double* mask01, const float* mask_logits, const void* gt,
                 int gt_f64, int B, int L, int H, int W, int use_hist, int mask_code, double* hist_state,
                 double* out, double* coef, void* ws, void* stream);
/* dcode[b][i][p] = gscale * coef[i] * (sigmoid(z) - t) * (mask_code ? m : 1), z = (mask_code ? m : 1) * code;
 * gscale = *grad_scale (f64 device scalar) or 1 if NULL */
int zp_code_loss_bwd(const float* code_logits, const double* mask01, const float* mask_logits, const void* gt,
                     int gt_f64, int B, int L, int H, int W, int mask_code, const double* coef,
                     const double* grad_scale, float* dcode, void* stream);
/* MaskLoss (BinaryCodeNet.py:89-93): out f32[1] = mean |sigmoid(x) - g| over n elements
 * (x = mask logits [B][1][H][W] viewed as [B][H][W]); ws: zp_mask_loss_ws_bytes(n) bytes */
long long zp_mask_loss_ws_bytes(long long n);
int zp_mask_loss(const float* mask_logits, const float* gt_mask, long long n, float* out, void* ws, void* stream);
/* dmask = gscale * sign(sigmoid(x) - g) * sigmoid(x) * (1 - sigmoid(x)) / n  (gscale f32 device scalar or NULL) */
int zp_mask_loss_bwd(const float* mask_logits, const float* gt_mask, long long n, const float* grad_scale,
                     float* dmask, void* stream);

/* ---- decode -------------------------------------------------------------------------- */
/* bits (u8, or f64 if out_f64) = logits > 8.940696716308594e-08f  (CPU fp32 sigmoid(x) > 0.5) */
int zp_threshold(const float* logits, long long n, int out_f64, void* bits, void* stream);
/* Per crop b (lut_index[b] selects the LUT when several objects are batched, NULL = 0):
 *   mask = threshold(mask_logits), id = sum_i bit_i << (L-1-i) over code channels 0..L-1,
 *   in row-major order of the mask pixels: xy = (int)(bbox[2]/bbox_size * x + bbox[0]),
 *   (int)(bbox[3]/bbox_size * y + bbox[1]) (truncation toward zero), xyz = lut[id] or 0 if any
 *   component is NaN; counts[b] = number of mask pixels.  ids (optional) = id image [B][H][W].
 *   mask_logits f32 [B][1][H][W], code_logits f32 [B][Lfull][H][W], lut f32 [n_lut][2^L][3],
 *   bbox int32 [B][4], xy int32 [B][H*W][2], xyz f32 [B][H*W][3].
 *   ws: zp_decode_ws_bytes(B, H, W) bytes. */
long long zp_decode_ws_bytes(int B, int H, int W);
int zp_decode(const float* mask_logits, const float* code_logits, int B, int H, int W, int Lfull,
              int L, const float* lut, const int* lut_index, const int* bbox, int bbox_size,
              int* ids, int* counts, int* xy, float* xyz, void* ws, void* stream);
/* out[n][3] (f32) = mean over the 2^(old-new) children of lut64 (f64, summed in order) */
int zp_lut_coarsen(const double* lut64, int old_bits, int new_bits, float* out, void* stream);

/* ---- pose ---------------------------------------------------------
 * Batched RANSAC-EPnP, replacing cv2.solvePnPRansac(P3D, P2D, K, None, reprojectionError,
 * iterationsCount, flags=SOLVEPNP_EPNP) at binary_code_helper/CNN_output_to_pose.py:152-156.
 * Inputs are zp_decode's outputs: counts[B], xy int32 [B][HW][2] (original-image pixels),
 * xyz f32 [B][HW][3]; K f64 [B][4] = (fx, fy, cx, cy).  Outputs R f64 [B][9] (row-major),
 * T f64 [B][3], success[B] (RANSAC found a model), inliers[B].  ws: zp_pnp_ws_bytes(B, iters). */
long long zp_pnp_ws_bytes(int B, int iters);
int zp_pnp_ransac(int B, int HW, const int* counts, const int* xy, const float* xyz, const double* K,
                  int iters, double reproj_err, double confidence, double* R, double* T, int* success,
                  int* inliers, void* ws, void* stream);

/* ---- pose error ----------------------------------------------------
 * ADD / ADI of B pose pairs over one model's points pts f32 [n][3], replacing
 * metric.py:8-18 (bop_toolkit pose_error.add / adi; lib/pysixd/pose_error.py:297-336).
 * R f64 [B][9] row-major, t f64 [B][3]; out f64 [B].  ADI is an exact nearest-neighbour search. */
#define ZP_METRIC_ADD 0
#define ZP_METRIC_ADI 1
long long zp_pose_error_ws_bytes(int B, int n, int mode);
int zp_pose_error(int B, const float* pts, int n, const double* R_est, const double* t_est,
                  const double* R_gt, const double* t_gt, int mode, double* out, void* ws, void* stream);

/* ---- device crop pipeline --------------------------------------------
 * Replaces the DataLoader worker's crop_square_resize (bop_dataset_pytorch.py:36-72) of the image
 * (cv2.INTER_LINEAR -> S px) + transform_pre (:333-347: ToTensor + ImageNet Normalize on the BGR
 * array), and of the GT code image / visible mask / entire mask (cv2.INTER_NEAREST -> S px)
 * + RGB_image_to_class_id_image / class_id_image_to_class_code_images
 * (class_id_encoder_decoder.py:6-15, 43-63).  Images stay on the device as one stack
 * u8 [n_img][H][W][3] (masks [n_img][H][W]); crop b reads image img_index[b] with the padded box
 * bbox[b] = (x, y, w, h) int32 (padding_Bbox output).  A box with w <= 0 and h <= 0 gives the
 * reference's all-zero dummy crop.
 *   zp_crop_image: out f32 [B][3][S][S] (normalised, BGR channel order as the reference feeds it)
 *   zp_crop_gt:    code u8 [B][L][S][S] (0/1, channel 0 = MSB), mask_out / entire_out f32
 *                  [B][S][S] = v / 255; any of the three outputs may be NULL */
int zp_crop_image(const uint8_t* imgs, int n_img, int H, int W, const int* img_index, const int* bbox, int B, int S,
                  float* out, void* stream);
int zp_crop_gt(const uint8_t* gts, const uint8_t* masks, const uint8_t* entire_masks, int n_img, int H, int W,
               const int* img_index, const int* bbox, int B, int S, int L, uint8_t* code, float* mask_out,
               float* entire_out, void* stream);

/* ---- optimizer ----------------------------------------------------------------------- */
/* torch.optim.Adam (no weight decay, amsgrad off) over one flat f32 buffer; step >= 1 */
int zp_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long long n,
            double lr, double beta1, double beta2, double eps, long long step, void* stream);
/* the same update for `count` tensors in ceil(count / 40) launches (host arrays of device
 * pointers; every tensor at the same step), bitwise identical to zp_adam per tensor */
int zp_adam_multi(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                  float* const* exp_avg_sq, const long long* numel, double lr, double beta1, double beta2,
                  double eps, long long step, void* stream);
/* the same with the step count read on the device (f32 scalar, already advanced to this step):
 * capturable in a hipGraph, whose replays then use the current count (GraphedTrainStep) */
int zp_adam_multi_dev(int count, float* const* params, const float* const* grads, float* const* exp_avg,
                      float* const* exp_avg_sq, const long long* numel, double lr, double beta1, double beta2,
                      double eps, const float* step_dev, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ZP_H_ */
