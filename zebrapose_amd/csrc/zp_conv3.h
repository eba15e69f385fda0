// Host entry points of the split-fp32 (ZP_F32X3) convolutions in zp_conv3.hip, called by zp_conv2d.
#pragma once
#include "zp_common.h"

namespace zp {
int conv3_tc(const zp_conv_args& a);             // cout tile
int conv3_tp(const zp_conv_args& a, int tc);     // pixel tile of the generic kernel
bool conv3_strip_ok(const zp_conv_args& a, int tc);  // k_conv3s eligible
int conv3_strip_mode(int v);
int conv3_min_blocks(int v);                      // zp_conv_tuning key 8; returns the previous value
int conv3_splitk_mode(int v);                     // zp_conv_tuning key 9; returns the previous value
int conv3_nsplit(const zp_conv_args& a);          // split-K slices (1: none)
int conv3_subint_mode(int v);                     // zp_conv_tuning key 16; returns the previous value
int conv3_pipe_st_mode(int v);                    // zp_conv_tuning key 19; returns the previous value
int stem_wgs_mode(int v);                         // zp_conv_tuning key 20; returns the previous value
int conv3w_pfb_mode(int v);                       // zp_conv_tuning key 21; returns the previous value
int conv3_launch(const zp_conv_args& a, hipStream_t st, int flags, const zp_head_args* head = nullptr);
// k_conv3w (zp_conv3w.hip): the 256 x 256 two-plane tile
struct conv_taps;
bool conv3w_ok(const zp_conv_args& a);            // eligible (and enabled)
int conv3w_mode(int v);                           // zp_conv_tuning key 10; returns the previous value
int conv3w_min_blocks(int v);                     // zp_conv_tuning key 11; returns the previous value
void conv3w_launch(const zp_conv_args& a, const conv_taps& tg, hipStream_t st, int flags, float* ws, int nsplit);
int conv3w_splitk(const zp_conv_args& a);         // split-K slices of the wide tile (1: none)
int conv3w_splitk_mode(int v);                    // zp_conv_tuning key 12; returns the previous value
int conv3w_tp(const zp_conv_args& a);            // pixel tile of the wide kernel (256, or 128)
int conv3w_tp_head(const zp_conv_args& a);       // pixel tile the fused head's conv would run on
int conv3w_acc_mode(int v);                       // zp_conv_tuning key 13; returns the previous value
int conv3w_tp128_mode(int v);                     // zp_conv_tuning key 14; returns the previous value
int conv3w_subint_mode(int v);                    // zp_conv_tuning key 17; returns the previous value
// k_conv3w32 (zp_conv3w32.hip): the 256 x 256 tile on 32 x 32 MFMAs
int conv3w_mf32_mode(int v);                      // zp_conv_tuning key 18; returns the previous value
bool conv3w_mf32_on();
void conv3w32_launch(const zp_conv_args& a, const conv_taps& tg, hipStream_t st, int flags, bool str);
void conv3w_head_launch(const zp_conv_args& a, const conv_taps& tg, const zp_head_args& h, hipStream_t st, int flags);
}  // namespace zp
