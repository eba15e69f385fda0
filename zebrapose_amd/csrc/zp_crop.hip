// Device-side crop pipeline: square ROI crop + resize + normalisation of the
// RGB input, nearest-neighbour crops of the GT code image and the masks, GT colour -> 16-bit
// code planes.  Replaces the CPU DataLoader worker path of bop_dataset_pytorch.py:
//   padding_Bbox (:124-139, host) -> get_roi(.., "crop_square_resize") (:36-72, :110-122)
//   with cv2.INTER_LINEAR (image, 256) / cv2.INTER_NEAREST (GT image, masks, 128) (:311-316)
//   -> RGB_image_to_class_id_image + class_id_image_to_class_code_images
//      (class_id_encoder_decoder.py:6-15, 43-63) -> transform_pre (:333-347: ToTensor +
//      Normalize with the RGB ImageNet constants on the BGR array, masks / 255.)
// cv2.resize is a third-party dependency absent from the image; the resize arithmetic follows
// OpenCV 4.x's generic (non-IPP) path, restated in oracle/crop_ref.py (parity vs OpenCV unpinned):
//   INTER_LINEAR, 8U: fx = (float)((dx + 0.5) * scale - 0.5), sx = floor(fx), clamped at both
//     borders with fx = 0; 11-bit fixed-point coefficients saturate_cast<short>(c * 2048);
//     horizontal pass exact in int32; vertical pass as the SIMD kernel computes it:
//     u8((mulhi16(h0 >> 4, b0) + mulhi16(h1 >> 4, b1) + 2) >> 2); an exact 2x downscale is
//     routed to INTER_AREA (2x2 box, (a + b + c + d + 2) >> 2) as cv::resize does.
//   INTER_NEAREST: sx = min(floor(dx * (1 / (dsize / ssize))), ssize - 1).
// One thread per output pixel; the source image stays in HBM/L2 (one crop reads at most its
// ROI once), outputs are written coalesced.
#include <math.h>
#include "zp_common.h"

namespace zp {

struct CropGeo {
  int x1, y1, xe, ye;  // ROI origin in the image, exclusive end of the copied image region
  int s;               // ROI side (max(bh, bw)); 0 = dummy crop
};

// crop_square_resize (:36-72): square-ify around the box centre, int() truncation, the ROI is
// s x s with roi(y, x) = img(y1 + y, x1 + x) inside [0, min(H, y2)) x [0, min(W, x2)), else 0
__device__ __forceinline__ CropGeo crop_geo(const int* bb, int H, int W) {
  CropGeo g;
  const int bx = bb[0], by = bb[1];
  const int bw = max(bb[2], 0), bh = max(bb[3], 0);
  double x1 = bx, x2 = (double)bx + bw, y1 = by, y2 = (double)by + bh;
  const double cx = 0.5 * (x1 + x2), cy = 0.5 * (y1 + y2);
  if (bh > bw) {
    x1 = cx - bh / 2.0;
    x2 = cx + bh / 2.0;
  } else {
    y1 = cy - bw / 2.0;
    y2 = cy + bw / 2.0;
  }
  g.x1 = (int)x1;  // Python int(): truncation toward zero
  g.y1 = (int)y1;
  g.xe = min((int)x2, W);
  g.ye = min((int)y2, H);
  g.s = max(bh, bw);
  return g;
}

__device__ __forceinline__ int roi_px(const uint8_t* img, int W, const CropGeo& g, int y, int x, int c) {
  const int iy = g.y1 + y, ix = g.x1 + x;
  if (iy < 0 || ix < 0 || iy >= g.ye || ix >= g.xe) return 0;
  return img[((size_t)iy * W + ix) * 3 + c];
}

// OpenCV cvRound on float (round half to even) then saturate to short
__device__ __forceinline__ int coef_q11(float c) { return (int)rintf(c * 2048.f); }

struct LinTap {
  int s0, s1;  // source index pair
  int a0, a1;  // Q11 coefficients
  bool edge;   // beyond xmax / clamped: only s0 * 2048 (horizontal pass)
};

__device__ __forceinline__ LinTap lin_tap(int d, double scale, int n) {
  float f = (float)((d + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f -= (float)s;
  LinTap t;
  t.edge = false;
  if (s < 0) {
    f = 0.f;
    s = 0;
  }
  if (s + 1 >= n) {
    t.edge = true;
    if (s >= n - 1) {
      f = 0.f;
      s = n - 1;
    }
  }
  t.s0 = s;
  t.s1 = min(s + 1, n - 1);
  t.a0 = coef_q11(1.f - f);
  t.a1 = coef_q11(f);
  return t;
}

__device__ __forceinline__ int mulhi16(int a, int b) {
  a = max(-32768, min(32767, a));  // v_pack saturation
  return (a * b) >> 16;
}

// image crop: out f32 NCHW [B][3][S][S], normalised ((v / 255 - mean[c]) / std[c], BGR order kept)
__global__ void __launch_bounds__(256) k_crop_image(const uint8_t* __restrict__ imgs, int H, int W,
                                                    const int* __restrict__ img_index, const int* __restrict__ bbox,
                                                    int S, float* __restrict__ out) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= S * S) return;
  const int dy = p / S, dx = p - dy * S;
  const CropGeo g = crop_geo(bbox + 4 * b, H, W);
  const float mean[3] = {0.485f, 0.456f, 0.406f}, stdv[3] = {0.229f, 0.224f, 0.225f};
  float* o = out + (size_t)b * 3 * S * S + p;
  if (g.s <= 0) {  // the reference's dummy input for a missing detection (:285-298): zeros
    for (int c = 0; c < 3; ++c) o[(size_t)c * S * S] = 0.f;
    return;
  }
  const uint8_t* img = imgs + (size_t)img_index[b] * H * W * 3;
  int v[3];
  const double inv = (double)S / g.s;  // cv::resize: inv_scale = dsize / ssize, scale = 1 / inv_scale
  const double scale = 1.0 / inv;
  const int iscale = (int)rint(scale);
  if (g.s == S) {
    for (int c = 0; c < 3; ++c) v[c] = roi_px(img, W, g, dy, dx, c);
  } else if (iscale == 2 && fabs(scale - iscale) < 2.220446049250313e-16) {
    // INTER_LINEAR at an exact 2x downscale -> INTER_AREA fast path (2 x 2 box)
    for (int c = 0; c < 3; ++c)
      v[c] = (roi_px(img, W, g, 2 * dy, 2 * dx, c) + roi_px(img, W, g, 2 * dy, 2 * dx + 1, c) +
              roi_px(img, W, g, 2 * dy + 1, 2 * dx, c) + roi_px(img, W, g, 2 * dy + 1, 2 * dx + 1, c) + 2) >> 2;
  } else {
    const LinTap tx = lin_tap(dx, scale, g.s), ty = lin_tap(dy, scale, g.s);
    for (int c = 0; c < 3; ++c) {
      int h[2];
      for (int k = 0; k < 2; ++k) {
        const int sy = k == 0 ? ty.s0 : ty.s1;
        const int p0 = roi_px(img, W, g, sy, tx.s0, c);
        h[k] = tx.edge ? p0 * 2048 : p0 * tx.a0 + roi_px(img, W, g, sy, tx.s1, c) * tx.a1;
      }
      const int r = (mulhi16(h[0] >> 4, ty.a0) + mulhi16(h[1] >> 4, ty.a1) + 2) >> 2;
      v[c] = max(0, min(255, r));
    }
  }
  for (int c = 0; c < 3; ++c) {
    const float x = (float)v[c] / 255.f;  // ToTensor: byte -> float / 255
    o[(size_t)c * S * S] = (x - mean[c]) / stdv[c];
  }
}

// GT crop (nearest, S_gt): code planes u8 [B][L][S][S] (bit i = (id >> (L - 1 - i)) & 1 with
// id = B << 16 | G << 8 | R of the BGR GT image), visible / entire masks f32 [B][S][S] = v / 255.
__global__ void __launch_bounds__(256) k_crop_gt(const uint8_t* __restrict__ gts, const uint8_t* __restrict__ masks,
                                                 const uint8_t* __restrict__ entire, int H, int W,
                                                 const int* __restrict__ img_index, const int* __restrict__ bbox, int S,
                                                 int L, uint8_t* __restrict__ code, float* __restrict__ mask_out,
                                                 float* __restrict__ entire_out) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= S * S) return;
  const int dy = p / S, dx = p - dy * S;
  const CropGeo g = crop_geo(bbox + 4 * b, H, W);
  int id = 0, mv = 0, ev = 0;
  if (g.s > 0) {
    const double ifx = 1.0 / ((double)S / g.s);
    const int sx = min((int)floor(dx * ifx), g.s - 1), sy = min((int)floor(dy * ifx), g.s - 1);
    const int iy = g.y1 + sy, ix = g.x1 + sx;
    if (iy >= 0 && ix >= 0 && iy < g.ye && ix < g.xe) {
      const size_t im = (size_t)img_index[b] * H * W;
      const size_t q = im + (size_t)iy * W + ix;
      if (gts) id = (gts[q * 3] << 16) | (gts[q * 3 + 1] << 8) | gts[q * 3 + 2];
      if (masks) mv = masks[q];
      if (entire) ev = entire[q];
    }
  }
  if (code) {
    uint8_t* cp = code + (size_t)b * L * S * S + p;
    for (int i = 0; i < L; ++i) cp[(size_t)i * S * S] = (uint8_t)((id >> (L - 1 - i)) & 1);
  }
  if (mask_out) mask_out[(size_t)b * S * S + p] = (float)((double)mv / 255.0);
  if (entire_out) entire_out[(size_t)b * S * S + p] = (float)((double)ev / 255.0);
}

}  // namespace zp

using namespace zp;

extern "C" int zp_crop_image(const uint8_t* imgs, int n_img, int H, int W, const int* img_index, const int* bbox,
                             int B, int S, float* out, void* stream) {
  ZP_CHECK_ARG(imgs && img_index && bbox && out && n_img > 0 && H > 0 && W > 0 && B > 0 && S > 0,
               "zp_crop_image: bad args");
  ZP_CHECK_ARG((long long)n_img * H * W * 3 < (1ll << 40), "zp_crop_image: image stack too large");
  hipLaunchKernelGGL(k_crop_image, dim3((S * S + 255) / 256, B), dim3(256), 0, (hipStream_t)stream, imgs, H, W,
                     img_index, bbox, S, out);
  ZP_LAUNCH_CHECK("zp_crop_image");
  return ZP_OK;
}

extern "C" int zp_crop_gt(const uint8_t* gts, const uint8_t* masks, const uint8_t* entire_masks, int n_img, int H,
                          int W, const int* img_index, const int* bbox, int B, int S, int L, uint8_t* code,
                          float* mask_out, float* entire_out, void* stream) {
  ZP_CHECK_ARG(img_index && bbox && n_img > 0 && H > 0 && W > 0 && B > 0 && S > 0, "zp_crop_gt: bad args");
  ZP_CHECK_ARG(!code || (gts && L >= 1 && L <= 24), "zp_crop_gt: code planes need the GT image and 1 <= L <= 24");
  ZP_CHECK_ARG(!mask_out || masks, "zp_crop_gt: mask_out needs masks");
  ZP_CHECK_ARG(!entire_out || entire_masks, "zp_crop_gt: entire_out needs entire_masks");
  hipLaunchKernelGGL(k_crop_gt, dim3((S * S + 255) / 256, B), dim3(256), 0, (hipStream_t)stream, gts, masks,
                     entire_masks, H, W, img_index, bbox, S, L, code, mask_out, entire_out);
  ZP_LAUNCH_CHECK("zp_crop_gt");
  return ZP_OK;
}
