// Host-side checks of libzp's C-ABI entry points under AddressSanitizer (tests/test_asan_host.py;
// SURVEY §5 "race / memory checking": host code only -- the device kernels are not instrumented
// and nothing here launches one).  Argument validation, workspace sizing and launch-configuration
// queries run on the host; every call below returns before any HIP launch.
#include <stdio.h>
#include <string.h>
#include "../../include/zp.h"

static int fails = 0;
#define CHECK(c)                                             \
  do {                                                       \
    if (!(c)) {                                              \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                               \
    }                                                        \
  } while (0)

static zp_conv_args conv(int dtype, int N, int H, int W, int Cin, int Cout, int k, int d) {
  zp_conv_args a;
  memset(&a, 0, sizeof(a));
  a.dtype = dtype;
  a.N = N; a.IH = a.GH = H; a.IW = a.GW = W; a.sy = a.sx = 1;
  a.Cin = Cin; a.ldx = Cin; a.Cout = Cout;
  a.k_pad = k * k * Cin;
  a.w_rows = zp_conv_rows_pad(Cout);
  a.nsub = 1;
  a.sub[0].ntaps = k * k;
  a.sub[0].ldy = Cout; a.sub[0].OH = H; a.sub[0].OW = W; a.sub[0].oys = a.sub[0].oxs = 1;
  for (int t = 0; t < k * k; ++t) {
    a.sub[0].ty[t] = (signed char)((t / k - k / 2) * d);
    a.sub[0].tx[t] = (signed char)((t % k - k / 2) * d);
  }
  return a;
}

int main() {
  CHECK(zp_abi_version() == ZP_ABI_VERSION);
  CHECK(zp_last_error() != NULL);
  // invalid calls return ZP_ERR_ARG with a message (no launch)
  CHECK(zp_conv2d(NULL, NULL) != ZP_OK);
  zp_conv_args bad = conv(ZP_F32H2, 2, 32, 32, 48, 256, 3, 1);  // Cin not a multiple of 32
  bad.sub[0].w = (void*)16; bad.sub[0].y = (void*)16; bad.x = (void*)16;
  CHECK(zp_conv2d(&bad, NULL) == ZP_ERR_ARG);
  CHECK(strlen(zp_last_error()) > 0);
  CHECK(zp_conv2d_head(NULL, NULL, NULL) == ZP_ERR_ARG);
  CHECK(zp_pack_weight(NULL, 1, 1, 1, 1, 0, 1, NULL, NULL, 1, ZP_F32, NULL, 1, 1, NULL) == ZP_ERR_ARG);
  const int ky[1] = {0}, kx[1] = {5};  // tap outside a 3x3 kernel
  CHECK(zp_pack_weight((const float*)16, 8, 8, 3, 3, 0, 1, ky, kx, 8, ZP_F32H2, (void*)16, 128, 32, NULL) == ZP_ERR_ARG);
  CHECK(zp_pack_weight_multi(-1, NULL, NULL, 0, NULL) == ZP_ERR_ARG);
  CHECK(zp_pack_weight_multi(0, NULL, NULL, 0, NULL) == ZP_OK);  // nothing to do
  CHECK(zp_im2col_split(NULL, 1, 8, 8, 8, 3, 7, 2, 3, 4, 4, 160, ZP_F32, NULL, NULL) == ZP_ERR_ARG);
  // launch configuration and workspace queries (host logic only)
  int tc = 0, tp = 0, st = 0, var = -1;
  zp_conv_args up2 = conv(ZP_F32H2, 32, 128, 128, 256, 256, 3, 1);  // up2's 3x3 at bs 32
  CHECK(zp_conv2d_config(&up2, &tc, &tp, &st, &var) == ZP_OK);
  CHECK(tc == 256 && tp == 256 && var == 6);                          // the 256 x 256 tile
  CHECK(zp_conv2d_head_ok(&up2) == 1);
  CHECK(zp_conv2d_head_ws(&up2) == 0);                               // the two-plane head: one launch
  CHECK(zp_conv2d_split_ws(&up2) == 0);                               // big grid: no split-K
  zp_conv_args l5 = conv(ZP_F32H2, 1, 32, 32, 512, 512, 3, 4);        // layer5 at bs 1
  CHECK(zp_conv2d_config(&l5, &tc, &tp, &st, &var) == ZP_OK);
  CHECK(zp_conv2d_head_ok(&l5) == 0);
  const long long ws = zp_conv2d_split_ws(&l5);
  CHECK(ws > 0 && ws % (4LL * 512 * 32 * 32) == 0);                  // [slices][M][Cout] f32
  zp_conv_args bf = conv(ZP_BF16, 32, 64, 64, 256, 256, 3, 1);
  CHECK(zp_conv2d_config(&bf, &tc, &tp, &st, &var) == ZP_OK && tc >= 64 && tp >= 128);
  CHECK(zp_conv2d_grid(&bf) > 0 && zp_conv2d_stat_parts(&bf) > 0);
  zp_conv_args bf2 = conv(ZP_BF16, 32, 128, 128, 256, 256, 3, 1);   // up2's last 3x3 at bs 32, bf16
  CHECK(zp_conv2d_head_ok(&bf2) == 1);                               // the fused 16-bit head
  CHECK(zp_conv2d_head_ws(&bf2) == 2LL * 32 * 32 * 128 * 128 * 4);   // [2 cout tiles][32][M] f32
  zp_wgrad_args wa;
  memset(&wa, 0, sizeof(wa));
  wa.dtype = ZP_BF16; wa.N = 32; wa.IH = wa.GH = 32; wa.IW = wa.GW = 32; wa.sy = wa.sx = 1;
  wa.Cin = wa.Cw = wa.ldx = 256; wa.Cout = 256; wa.kh = wa.kw = 3; wa.nsub = 1;
  wa.sub[0].ntaps = 9; wa.sub[0].lddy = 256; wa.sub[0].OH = wa.sub[0].OW = 32; wa.sub[0].oys = wa.sub[0].oxs = 1;
  for (int t = 0; t < 9; ++t) {
    wa.sub[0].ky[t] = (signed char)(t / 3); wa.sub[0].kx[t] = (signed char)(t % 3);
    wa.sub[0].ty[t] = (signed char)(t / 3 - 1); wa.sub[0].tx[t] = (signed char)(t % 3 - 1);
  }
  CHECK(zp_conv2d_wgrad_ws_bytes(&wa) > 0);
  CHECK(zp_decode_ws_bytes(32, 128, 128) > 0);
  CHECK(zp_pnp_ws_bytes(32, 150) > 0);
  CHECK(zp_code_loss_ws_bytes(32, 16, 128, 128) > 0);
  CHECK(zp_mask_loss_ws_bytes(32LL * 128 * 128) > 0);
  CHECK(zp_pose_error_ws_bytes(32, 1000, ZP_METRIC_ADI) >= 0);
  CHECK(zp_bn_bwd_parts(32 * 64 * 64, 64) > 0);
  // the fused BN backward reduce (ABI 3): refused without its inputs, with a residual or a split dtype
  zp_conv_args bnr = conv(ZP_BF16, 32, 32, 32, 256, 256, 3, 1);
  bnr.x = (void*)16; bnr.sub[0].w = (void*)16; bnr.sub[0].y = (void*)16;
  bnr.bnr_part = (float*)16;
  CHECK(zp_conv2d(&bnr, NULL) == ZP_ERR_ARG);                        // no bnr_x / bnr_save
  bnr.bnr_x = (void*)16; bnr.bnr_save = (const float*)16; bnr.res = (void*)16; bnr.ldr = 256;
  CHECK(zp_conv2d(&bnr, NULL) == ZP_ERR_ARG);                        // residual epilogue
  zp_conv_args bnr3 = up2;
  bnr3.bnr_part = (float*)16; bnr3.bnr_x = (void*)16; bnr3.bnr_save = (const float*)16;
  CHECK(zp_conv2d(&bnr3, NULL) == ZP_ERR_ARG);                       // split-fp32 forms: eval only
  CHECK(zp_bn_bwd_totals(NULL, 4, 64, 4, NULL, NULL, 0, NULL) == ZP_ERR_ARG);
  zp_conv_args bnr2 = conv(ZP_BF16, 32, 128, 128, 256, 256, 3, 1);  // strip tile: one part per 256 pixels
  CHECK(zp_conv2d_bnr_parts(&bnr2) == 32 * 128 * 128 / 256);
  CHECK(zp_conv2d_bnr_parts(&bnr2) == zp_conv2d_stat_parts(&bnr2));       // (the statistics too, round 5)
  // tuning knobs round-trip; unknown keys answer -1
  const int old = zp_conv_tuning(10, 0);
  CHECK(zp_conv_tuning(10, old) == 0);
  CHECK(zp_conv_tuning(-7, 0) == -1);
  printf(fails ? "abi_driver: %d failure(s)\n" : "abi_driver: ok\n", fails);
  return fails ? 1 : 0;
}
