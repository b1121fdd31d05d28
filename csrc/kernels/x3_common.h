// Helpers of the fp32-accurate split-bf16 GEMM kernels (conv_x3.hip, wgrad.hip).
//
//   x = h0 + h1 + h2 exactly (barring underflow), h0 = rn_bf16(x), h1 = rn_bf16(x - h0),
//   h2 = rn_bf16(x - h0 - h1); both subtractions are exact (Sterbenz).
//
// Pairs are split together: v_cvt_pk_bf16_f32 for the rounding, a shift and a mask to widen the two
// bf16 back to f32, scalar subtractions for the residuals: 11 VALU per pair of elements.
#pragma once
#include "common.h"

namespace cdp {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned pack_bf16x2(f32x2 v) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2_v));
}

__device__ __forceinline__ f32x2 widen_bf16x2(unsigned h) {
  return f32x2{__uint_as_float(h << 16), __uint_as_float(h & 0xffff0000u)};
}

// (scalar f32 subtractions: see split_pair_h on packed-f32 VALU beside MFMAs)
__device__ __forceinline__ void split_pair(float x, float y, unsigned& h0, unsigned& h1, unsigned& h2) {
  h0 = pack_bf16x2(f32x2{x, y});
  const f32x2 w0 = widen_bf16x2(h0);
  const float r1x = x - w0.x, r1y = y - w0.y;
  h1 = pack_bf16x2(f32x2{r1x, r1y});
  const f32x2 w1 = widen_bf16x2(h1);
  h2 = pack_bf16x2(f32x2{r1x - w1.x, r1y - w1.y});
}

// ---- f16x2 engine: two fp16 terms of a power-of-two-scaled operand ------------------------
//
//   s*x = h0 + h1 + r,  h0 = rn_f16(s*x), h1 = rn_f16(s*x - h0),  |r| <= 2^-22 |s*x|
//
// fp16 keeps 11 significant bits, so two terms carry 22 -- against 24 for fp32 and 3 x 8 for
// the bf16 split -- and the product needs three MFMA terms (h0g0 + h0g1 + h1g0, dropped
// h1g1 <= 2^-22 |ab|) instead of six. fp16's 5-bit exponent is what the scale s = 2^e is for: it
// maps a group's |max| to [2^14, 2^15), so nothing overflows and everything within 2^17 of the
// group max keeps all 22 bits (smaller values degrade to an absolute error of ~2^-39 of the group
// max).
//
// The groups are GEMM rows, one scale per row of each operand (per image for the gathered
// activation, per output / input channel for the weights, per channel for both weight-gradient
// operands): an output y[m][n] = sum_k a[m][k] b[n][k] sees one scale s_m of A and one s_n of B,
// so y = (sum_k (s_m a)(s_n b)) / (s_m s_n) -- the scales factor out of every dot product and the
// epilogue's division is exact. The only values that lose bits are those more than 2^17 below the
// max of their own row, i.e. dynamic range WITHIN one image (or one channel) along the reduction,
// whose contribution to that output is then < 2^-39 max_k |a[m][k]| sum_k |b[n][k]|
// (tests/test_accuracy_gpu.py documents that limit).
typedef _Float16 f16x2_v __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ unsigned pack_f16x2(f32x2 v) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, f16x2_v));
}
__device__ __forceinline__ f32x2 widen_f16x2(unsigned h) {
  return __builtin_convertvector(__builtin_bit_cast(f16x2_v, h), f32x2);
}
// 2 x v_mul_f32, v_cvt_pk_f16_f32, 2 x v_cvt_f32_f16, 2 x v_fma_f32, v_cvt_pk_f16_f32 per pair.
// Scalar f32 on purpose: packed-f32 VALU (v_pk_mul/v_pk_fma) issued between MFMAs costs ~22 extra
// cycles per MFMA gap (MI355X_MICROARCH.md, per-instruction constants), scalar FMAs ~0; the
// kernels are built with -fno-slp-vectorize so the compiler does not re-pack these.
__device__ __forceinline__ void split_pair_h(float x, float y, float s, unsigned& h0, unsigned& h1) {
  const float vx = x * s, vy = y * s;
  h0 = pack_f16x2(f32x2{vx, vy});
  const f32x2 w = widen_f16x2(h0);
  h1 = pack_f16x2(f32x2{__builtin_fmaf(x, s, -w.x), __builtin_fmaf(y, s, -w.y)});
}

// Power-of-two operand scale of a group whose |max| is m: maps m to [2^14, 2^15). A zero, inf or
// NaN max gives 1 (zeros stay zeros; non-finite inputs propagate as in fp32). The exponent is
// clamped to +-100 so both the scale and its reciprocal stay normal fp32 numbers.
__device__ __forceinline__ float pow2_scale(float m) {
  if (!(m > 0.f) || !(m < 3.0e38f)) return 1.f;
  int e;
  (void)frexpf(m, &e);  // m < 2^e
  return ldexpf(1.f, max(-100, min(100, 15 - e)));
}

// Raw buffer resource over [base, base + bytes): loads past `bytes` return 0 (hardware range
// check), which implements the implicit-GEMM zero padding without branches or selects.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

constexpr unsigned kOOB = 0x80000000u;  // a byte offset past every buffer (host keeps buffers < 2 GiB)

__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

// full-rate 24-bit multiplies (v_mul_u32_u24 / v_mul_i32_i24) for index math; every operand is < 2^23
__device__ __forceinline__ int mul24(int a, int b) { return __mul24(a, b); }

}  // namespace cdp
