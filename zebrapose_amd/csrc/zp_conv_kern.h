// Device helpers shared by the conv kernels of zp_conv.hip and zp_conv3.hip (MFMA operand traits,
// counted vmcnt waits, LDS addressing, immediate-offset ds_read_b128, compile-time loops, DPP row
// sums, the per-launch tap grid).
#pragma once
#include <type_traits>
#include "zp_common.h"

namespace zp {

template <typename T> struct MfmaTraits;
template <> struct MfmaTraits<bf16_t> {
  static constexpr int E = 8;  // elements per 16 B chunk
  static __device__ __forceinline__ void mma(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                  acc, 0, 0, 0);
  }
};
template <> struct MfmaTraits<f16_t> {
  static constexpr int E = 8;
  static __device__ __forceinline__ void mma(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b),
                                                 acc, 0, 0, 0);
  }
};
template <> struct MfmaTraits<float> {
  static constexpr int E = 4;
  // 16 B chunk = 4 consecutive k of one row; element e is k-substep e for every lane
  // group, so the four 16x16x4 MFMAs together cover all 16 k of the 4 lane groups.
  static __device__ __forceinline__ void mma(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
  }
};

__device__ __forceinline__ int swz(int row, int chunk) { return row * 8 + (chunk ^ (row & 7)); }


// s_waitcnt vmcnt(N) only (LDS-DMA loads count on vmcnt); "memory" keeps LDS accesses in place
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Per-launch tap grids, derived on the host from the subs' tap lists (every plan of
// geometry.py enumerates taps as a (tap row) x (tap column) grid, rows outer:
// ty = ty0 + q * dty, tx = tx0 + r * dtx for tap q * nx + r), plus the byte extents of the
// activation / weight buffers for the buffer-load range check.
struct conv_taps {
  int ny[ZP_MAX_SUB], nx[ZP_MAX_SUB], ty0[ZP_MAX_SUB], dty[ZP_MAX_SUB], tx0[ZP_MAX_SUB], dtx[ZP_MAX_SUB];
  unsigned x_bytes, w_bytes[ZP_MAX_SUB];
  unsigned* rflag;  // two-plane split stores: the range flag (range_flag()), or NULL
};

// LDS byte address of a __shared__ pointer
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// ds_read_b128 with an immediate offset; the caller waits lgkmcnt itself
template <int OFF>
__device__ __forceinline__ uint4 ds_read16(unsigned addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset range");
  uint4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF) : "memory");
  return r;
}

// 2^11 * x for the 8 fp16 values of a fragment (v_pk_mul_f16; exact: fp16 exponent shift, no
// overflow for |x| < 32 -- the two-plane weight packs flag larger weights, zp_misc.hip)
__device__ __forceinline__ uint4 scale_hi(const uint4 a) {
  typedef _Float16 h2v __attribute__((ext_vector_type(2)));
  const h2v k = {(_Float16)2048.f, (_Float16)2048.f};
  uint4 r;
  r.x = __builtin_bit_cast(unsigned, __builtin_bit_cast(h2v, a.x) * k);
  r.y = __builtin_bit_cast(unsigned, __builtin_bit_cast(h2v, a.y) * k);
  r.z = __builtin_bit_cast(unsigned, __builtin_bit_cast(h2v, a.z) * k);
  r.w = __builtin_bit_cast(unsigned, __builtin_bit_cast(h2v, a.w) * k);
  return r;
}

template <int N, typename F, int I = 0>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, F, I + 1>(static_cast<F&&>(f));
  }
}

// Sum over the 16 lanes of each DPP row (lanes 16k .. 16k + 15), the total in every lane of the row:
// quad_perm xor 1, xor 2, then row_half_mirror and row_mirror -- the same pairing tree as
// __shfl_xor over 1, 2, 4, 8 (bit-identical sums) as four DPP adds instead of four ds_bpermute
// round trips through the LDS crossbar.
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));  // row_half_mirror
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));  // row_mirror
  return v;
}

}  // namespace zp
