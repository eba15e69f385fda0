// Code -> vertex decode on gfx950: logits -> mask / code bits -> 16-bit class id -> LUT
// gather -> row-major compaction of the mask pixels -> original-image coordinates.
//
// Reference (lyltc1/ZebraPose):
//   common_ops.py:5-19                               sigmoid(x) > 0.5 (CPU fp32) == x > 8.940696716308594e-08f
//   class_id_encoder_decoder.py:17-28                id = sum_i bit_i * 2^(L-1-i)  (channel 0 = MSB)
//   CNN_output_to_pose.py:53-64                      P2D = (x, y) of mask.nonzero() (row-major),
//                                                    P3D = LUT[id], NaN rows -> [0,0,0] (kept)
//   CNN_output_to_pose.py:34-50                      x' = int(Bbox[2]/Bbox_Size * x + Bbox[0]) (f64, trunc)
//   CNN_output_to_pose.py:128-129                    P2D/P3D cast to float32 for PnP
//   generate_new_dict.py:4-33                        ignore_bit LUT = f64 mean of the 2^k children
//
// Two passes over tiles of 1024 pixels: (1) ids + per-tile mask counts, (2) per-tile
// offsets (prefix over the crop's earlier tiles) + block scan + ordered writes.
#include "zp_common.h"

namespace zp {

constexpr int DEC_TILE = 1024;  // pixels per tile (256 threads x 4)
constexpr float kHalfLogit = 8.940696716308594e-08f;

__global__ void __launch_bounds__(256) k_decode_ids(const float* __restrict__ mlog, const float* __restrict__ clog, int HW,
                                                    int Lfull, int L, int* __restrict__ packed, int* __restrict__ ids,
                                                    int* __restrict__ tile_cnt, int tiles) {
  const int b = blockIdx.y, tile = blockIdx.x;
  const int p0 = tile * DEC_TILE + threadIdx.x * 4;
  __shared__ int wsum[4];
  int cnt = 0;
  const float* mrow = mlog + (size_t)b * HW;
  const float* crow = clog + (size_t)b * Lfull * HW;
  if (p0 + 3 < HW && (HW & 3) == 0) {
    float4 m = *(const float4*)(mrow + p0);
    int id[4] = {0, 0, 0, 0};
    for (int i = 0; i < L; ++i) {
      float4 c = *(const float4*)(crow + (size_t)i * HW + p0);
      id[0] = (id[0] << 1) | (c.x > kHalfLogit);
      id[1] = (id[1] << 1) | (c.y > kHalfLogit);
      id[2] = (id[2] << 1) | (c.z > kHalfLogit);
      id[3] = (id[3] << 1) | (c.w > kHalfLogit);
    }
    int mb[4] = {m.x > kHalfLogit, m.y > kHalfLogit, m.z > kHalfLogit, m.w > kHalfLogit};
    int4 pk = make_int4(mb[0] ? id[0] : -1, mb[1] ? id[1] : -1, mb[2] ? id[2] : -1, mb[3] ? id[3] : -1);
    *(int4*)(packed + (size_t)b * HW + p0) = pk;
    if (ids) *(int4*)(ids + (size_t)b * HW + p0) = make_int4(id[0], id[1], id[2], id[3]);
    cnt = mb[0] + mb[1] + mb[2] + mb[3];
  } else {
    for (int k = 0; k < 4; ++k) {
      int p = p0 + k;
      if (p >= HW) break;
      int id = 0;
      for (int i = 0; i < L; ++i) id = (id << 1) | (crow[(size_t)i * HW + p] > kHalfLogit);
      int mb = mrow[p] > kHalfLogit;
      packed[(size_t)b * HW + p] = mb ? id : -1;
      if (ids) ids[(size_t)b * HW + p] = id;
      cnt += mb;
    }
  }
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) tile_cnt[b * tiles + tile] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

__global__ void __launch_bounds__(256) k_decode_emit(const int* __restrict__ packed, const int* __restrict__ tile_cnt,
                                                     int tiles, int H, int W, int L, const float* __restrict__ lut,
                                                     const int* __restrict__ lut_index, const int* __restrict__ bbox,
                                                     int bbox_size, int* __restrict__ counts, int* __restrict__ xy,
                                                     float* __restrict__ xyz) {
  const int b = blockIdx.y, tile = blockIdx.x;
  const int HW = H * W;
  __shared__ int scan[256];
  __shared__ int base_s;
  if (threadIdx.x == 0) {
    int base = 0, total = 0;
    for (int t = 0; t < tiles; ++t) {
      int c = tile_cnt[b * tiles + t];
      if (t < tile) base += c;
      total += c;
    }
    base_s = base;
    if (tile == 0) counts[b] = total;
  }
  const int p0 = tile * DEC_TILE + threadIdx.x * 4;
  int v[4];
  int mine = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int p = p0 + k;
    v[k] = p < HW ? packed[(size_t)b * HW + p] : -1;
    mine += v[k] >= 0;
  }
  scan[threadIdx.x] = mine;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    int t = threadIdx.x >= off ? scan[threadIdx.x - off] : 0;
    __syncthreads();
    scan[threadIdx.x] += t;
    __syncthreads();
  }
  int pos = base_s + scan[threadIdx.x] - mine;
  const double bx = bbox[b * 4 + 0], by = bbox[b * 4 + 1];
  const double rx = (double)bbox[b * 4 + 2] / (double)bbox_size;
  const double ry = (double)bbox[b * 4 + 3] / (double)bbox_size;
  const float* L3 = lut + (size_t)(lut_index ? lut_index[b] : 0) * ((size_t)3 << L);
  int* oxy = xy + (size_t)b * HW * 2;
  float* oxyz = xyz + (size_t)b * HW * 3;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (v[k] < 0) continue;
    int p = p0 + k;
    int py = p / W, px = p - py * W;
    // f64 multiply then add, no FMA contraction (numpy order); astype('int') truncates toward zero
    oxy[2 * pos] = (int)__dadd_rn(__dmul_rn(rx, (double)px), bx);
    oxy[2 * pos + 1] = (int)__dadd_rn(__dmul_rn(ry, (double)py), by);
    float a = L3[(size_t)v[k] * 3], c = L3[(size_t)v[k] * 3 + 1], d = L3[(size_t)v[k] * 3 + 2];
    if (isnan(a) || isnan(c) || isnan(d)) a = c = d = 0.f;
    oxyz[3 * pos] = a;
    oxyz[3 * pos + 1] = c;
    oxyz[3 * pos + 2] = d;
    ++pos;
  }
}

__global__ void k_lut_coarsen(const double* __restrict__ lut, int k, int n_new, float* __restrict__ out) {
  int nid = blockIdx.x * blockDim.x + threadIdx.x;
  if (nid >= n_new) return;
  double s0 = 0, s1 = 0, s2 = 0;
  const int nch = 1 << k;
  for (int c = 0; c < nch; ++c) {
    const double* r = lut + ((size_t)nid * nch + c) * 3;
    s0 = s0 + r[0];
    s1 = s1 + r[1];
    s2 = s2 + r[2];
  }
  out[(size_t)nid * 3] = (float)(s0 / nch);
  out[(size_t)nid * 3 + 1] = (float)(s1 / nch);
  out[(size_t)nid * 3 + 2] = (float)(s2 / nch);
}

}  // namespace zp

using namespace zp;

extern "C" long long zp_decode_ws_bytes(int B, int H, int W) {
  long long HW = (long long)H * W;
  long long tiles = (HW + DEC_TILE - 1) / DEC_TILE;
  return (long long)B * HW * 4 + (long long)B * tiles * 4 + 256;
}

extern "C" int zp_decode(const float* mask_logits, const float* code_logits, int B, int H, int W, int Lfull, int L,
                         const float* lut, const int* lut_index, const int* bbox, int bbox_size, int* ids, int* counts,
                         int* xy, float* xyz, void* ws, void* stream) {
  ZP_CHECK_ARG(mask_logits && code_logits && lut && bbox && counts && xy && xyz && ws, "zp_decode: null pointer");
  ZP_CHECK_ARG(B > 0 && H > 0 && W > 0 && L >= 1 && L <= 24 && L <= Lfull && bbox_size > 0, "zp_decode: bad sizes");
  const int HW = H * W;
  const int tiles = (HW + DEC_TILE - 1) / DEC_TILE;
  int* packed = (int*)ws;
  int* tile_cnt = packed + (size_t)B * HW;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_decode_ids, dim3(tiles, B), dim3(256), 0, st, mask_logits, code_logits, HW, Lfull, L, packed,
                     ids, tile_cnt, tiles);
  ZP_LAUNCH_CHECK("zp_decode ids");
  hipLaunchKernelGGL(k_decode_emit, dim3(tiles, B), dim3(256), 0, st, packed, tile_cnt, tiles, H, W, L, lut, lut_index,
                     bbox, bbox_size, counts, xy, xyz);
  ZP_LAUNCH_CHECK("zp_decode emit");
  return ZP_OK;
}

extern "C" int zp_lut_coarsen(const double* lut64, int old_bits, int new_bits, float* out, void* stream) {
  ZP_CHECK_ARG(lut64 && out && new_bits >= 1 && new_bits <= old_bits && old_bits <= 24, "zp_lut_coarsen: bad args");
  const int n_new = 1 << new_bits;
  hipLaunchKernelGGL(k_lut_coarsen, dim3((n_new + 255) / 256), dim3(256), 0, (hipStream_t)stream, lut64,
                     old_bits - new_bits, n_new, out);
  ZP_LAUNCH_CHECK("zp_lut_coarsen");
  return ZP_OK;
}
