// x3.h — the three-way bf16 split of fp32 operands shared by the split-bf16 ("x3") MFMA kernels
// (gemm.hip's tiled GEMM).
//
// Every fp32 value is a = a0 + a1 + a2 with each term the round-to-nearest bf16 of the remainder
// (|a - a0| <= 2^-8 |a|, |a - a0 - a1| <= 2^-16 |a|, the rest <= 2^-24 |a|: fp32 input precision),
// so a.b is recovered to fp32 accuracy from six bf16 x bf16 products (each exact in fp32) summed in
// fp32: a2b0 + a1b1 + a0b2 + a1b0 + a0b1 + a0b0 (increasing magnitude).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mpr {
namespace x3 {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// RNE bf16 of (a, b) packed in one word (one v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
}
// fp32 value of the low / high bf16 of a packed word
__device__ __forceinline__ float lo_f(uint32_t p) { return __builtin_bit_cast(float, p << 16); }
__device__ __forceinline__ float hi_f(uint32_t p) {
  return __builtin_bit_cast(float, p & 0xffff0000u);
}

// v = h0 + h1 + h2 exactly (each an RNE bf16 of the remainder), on packed words: the plain
// vector form (convert, convert back, subtract) compiled to a convert per element and a second
// convert + shift for the way back, 32 VALU per float4 in place of these 18.
__device__ __forceinline__ void split3(const f32x4& v, bf16x4& h0, bf16x4& h1, bf16x4& h2) {
  u32x2 p0, p1, p2;
  f32x4 r1, r2;
  p0[0] = pk_bf16(v[0], v[1]);
  p0[1] = pk_bf16(v[2], v[3]);
  r1[0] = v[0] - lo_f(p0[0]);
  r1[1] = v[1] - hi_f(p0[0]);
  r1[2] = v[2] - lo_f(p0[1]);
  r1[3] = v[3] - hi_f(p0[1]);
  p1[0] = pk_bf16(r1[0], r1[1]);
  p1[1] = pk_bf16(r1[2], r1[3]);
  r2[0] = r1[0] - lo_f(p1[0]);
  r2[1] = r1[1] - hi_f(p1[0]);
  r2[2] = r1[2] - lo_f(p1[1]);
  r2[3] = r1[3] - hi_f(p1[1]);
  p2[0] = pk_bf16(r2[0], r2[1]);
  p2[1] = pk_bf16(r2[2], r2[3]);
  h0 = __builtin_bit_cast(bf16x4, p0);
  h1 = __builtin_bit_cast(bf16x4, p1);
  h2 = __builtin_bit_cast(bf16x4, p2);
}

// Eight consecutive values (two float4) into three bf16x8 planes: one MFMA operand fragment of a
// 16x16x32 step (lane (i, g) holds row i, k = 8g .. 8g + 7).
__device__ __forceinline__ void split8(const f32x4& lo, const f32x4& hi, bf16x8& h0, bf16x8& h1,
                                       bf16x8& h2) {
  bf16x4 a0, a1, a2, b0, b1, b2;
  split3(lo, a0, a1, a2);
  split3(hi, b0, b1, b2);
  h0 = __builtin_shufflevector(a0, b0, 0, 1, 2, 3, 4, 5, 6, 7);
  h1 = __builtin_shufflevector(a1, b1, 0, 1, 2, 3, 4, 5, 6, 7);
  h2 = __builtin_shufflevector(a2, b2, 0, 1, 2, 3, 4, 5, 6, 7);
}

}  // namespace x3
}  // namespace mpr
