// Shared definitions for the ZebraPose MI355X (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include "../../include/zp.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef unsigned short bf16_t;  // bf16 storage
typedef _Float16 f16_t;         // IEEE fp16 (inference-only compute dtype ZP_F16)

namespace zp {

void set_error(const char* fmt, ...);

#define ZP_CHECK_ARG(cond, ...)                 \
  do {                                          \
    if (!(cond)) {                              \
      ::zp::set_error(__VA_ARGS__);             \
      return ZP_ERR_ARG;                        \
    }                                           \
  } while (0)

#define ZP_LAUNCH_CHECK(what)                                                   \
  do {                                                                          \
    hipError_t e_ = hipGetLastError();                                          \
    if (e_ != hipSuccess) {                                                     \
      ::zp::set_error("%s: launch failed: %s", what, hipGetErrorString(e_));    \
      return ZP_ERR_HIP;                                                        \
    }                                                                           \
  } while (0)

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // RNE, NaN-preserving (v_cvt_pk_bf16_f32)
  return __builtin_bit_cast(bf16_t, b);
}

// ZP_F32X3 (split fp32, zp.h): v -> (hi, mid, lo) bf16 with v == hi + mid + lo exactly for finite
// v (each round-to-nearest step leaves a remainder exactly representable in f32 with at most 16 /
// 8 significant bits, so lo is exact); infinities / NaN keep mid = lo = 0.
__device__ __forceinline__ void split3(float v, bf16_t& h, bf16_t& m, bf16_t& l) {
  h = f2bf(v);
  const float r1 = v - bf2f(h);
  m = f2bf(r1);
  l = f2bf(r1 - bf2f(m));
  if (!__builtin_isfinite(v)) {
    m = 0;
    l = 0;
  }
}
// (hi + mid) is exact, and the exact total is an f32, so the second add rounds to it
__device__ __forceinline__ float join3(bf16_t h, bf16_t m, bf16_t l) { return (bf2f(h) + bf2f(m)) + bf2f(l); }

// The two split-fp32 storage forms as NPL planes of 16-bit words (zp.h ZP_F32X3 / ZP_F32H2):
//   SplitF32<3>: bf16 hi + mid + lo, exact (split3 / join3);
//   SplitF32<2>: IEEE fp16 hi + lo' with v ~ hi + lo' * 2^-11: hi = RNE(v), lo' = RNE((v - hi) * 2^11)
//     (the residual is scaled into fp16's normal range; 22 significant bits, |v - join| <= 2^-23 |v|
//     for |v| in fp16's normal range, 2^-36 absolute below it).  Finite |v| >= 65520 rounds hi to
//     infinity: every store site raises the range flag for it (h2_overflow below) and the engine
//     re-runs the forward on the full-range SplitF32<3>; non-finite values keep lo' = 0.
// CS: the factor the lo-plane products carry (k_conv3 scales its correction accumulator by it).
template <int NPL> struct SplitF32;
template <> struct SplitF32<3> {
  static constexpr float CS = 1.f;
  static __device__ __forceinline__ void split(float v, unsigned short (&p)[3]) { split3(v, p[0], p[1], p[2]); }
  static __device__ __forceinline__ float join(const unsigned short (&p)[3]) { return join3(p[0], p[1], p[2]); }
};
template <> struct SplitF32<2> {
  static constexpr float CS = 1.f / 2048.f;
  static __device__ __forceinline__ void split(float v, unsigned short (&p)[2]) {
    const f16_t h = (f16_t)v;
    const float r = v - (float)h;
    f16_t l = (f16_t)(r * 2048.f);
    if (!__builtin_isfinite((float)h)) l = (f16_t)0.f;
    p[0] = __builtin_bit_cast(unsigned short, h);
    p[1] = __builtin_bit_cast(unsigned short, l);
  }
  static __device__ __forceinline__ float join(const unsigned short (&p)[2]) {
    return __builtin_fmaf((float)__builtin_bit_cast(f16_t, p[1]), CS, (float)__builtin_bit_cast(f16_t, p[0]));
  }
};

// Range guard of the two-plane form (zp_split_range_flag): a finite value at or above 65520 in
// magnitude rounds hi to fp16 infinity.  Every ZP_F32H2 store site ORs this per lane and, at the
// end, raises the registered device word with a plain vector store (any lane, value 1).
__device__ __forceinline__ bool h2_overflow(float v) {
  const float a = __builtin_fabsf(v);
  return a >= 65520.f && a < __builtin_inff();
}
// Weights of the two-plane form carry a tighter bound: k_conv3w forms 2^11 * hi in fp16 (its single
// scaled accumulator), which overflows for |w| >= 65504 / 2048 = 31.984375.  The weight packs flag
// it (the engine falls back to SplitF32<3> as for activations; trained conv weights sit far below).
__device__ __forceinline__ bool h2w_overflow(float v) {
  const float a = __builtin_fabsf(v);
  return a >= 31.984375f && a < __builtin_inff();
}
__device__ __forceinline__ void raise_range_flag(unsigned* flag, bool bad) {
  if (bad && flag) *flag = 1u;
}
// the word registered for the calling thread's current device (NULL: no guard); read by the host
// launch code of every split store (a captured hipGraph keeps the pointer of its capture)
unsigned* range_flag();
// zp_conv_tuning key 15 (zp_misc.hip): the train-mode BN statistics merge in one launch (1) or two (0)
int bn_fused_mode(int v);

template <typename T> struct Elem;
template <> struct Elem<float> {
  static __device__ __forceinline__ float ld(const float* p) { return *p; }
  static __device__ __forceinline__ float cvt(float v) { return v; }
};
template <> struct Elem<bf16_t> {
  static __device__ __forceinline__ float ld(const bf16_t* p) { return bf2f(*p); }
  static __device__ __forceinline__ bf16_t cvt(float v) { return f2bf(v); }
};

template <> struct Elem<f16_t> {
  static __device__ __forceinline__ float ld(const f16_t* p) { return (float)*p; }
  static __device__ __forceinline__ f16_t cvt(float v) { return (f16_t)v; }  // RNE
};

// 16-bit storage formats as raw bits: from(bits) -> f32, to(f32) -> bits.  H16<float> exists only
// so that runtime-dead 16-bit branches of f32 instantiations compile.
template <typename T> struct H16 {
  static __device__ __forceinline__ float from(uint32_t u) { return bf2f((bf16_t)u); }
  static __device__ __forceinline__ uint32_t to(float v) { return f2bf(v); }
};
template <> struct H16<f16_t> {
  static __device__ __forceinline__ float from(uint32_t u) {
    return (float)__builtin_bit_cast(f16_t, (unsigned short)u);
  }
  static __device__ __forceinline__ uint32_t to(float v) { return __builtin_bit_cast(unsigned short, (f16_t)v); }
};

inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

}  // namespace zp
