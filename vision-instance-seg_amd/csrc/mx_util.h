// Block-scaled MX (OCP e4m3 + e8m0) helpers shared by the fp8 kernels (window attention,
// token GEMM): the v_mfma_scale_f32_32x32x64_f8f6f4 wrapper and the scaled conversions
// from / to bf16 pairs (gfx950).  Operand layout of the MX MFMA as measured on the box
// (tools/micro/mfma_scale_probe.hip, profiles/r3_mfma_scale_probe.txt): lane l (row or
// column l & 31, half hh = l >> 5) holds in bytes 0..15 sixteen elements of K-block 0 and
// in bytes 16..31 sixteen of K-block 1 (the two lanes of a row together cover each
// 32-element block); its scale byte is that of block hh of its row / column.
#pragma once
#include "mfma_util.h"

namespace vs {

typedef int i32x8_t __attribute__((ext_vector_type(8)));

// The MX MFMA builtin is not marked convergent by this compiler (ROCm 7.2): when its result
// only feeds a divergent store (the forward's `if (q < N)` epilogue) LLVM sinks it, with the
// VALU that builds its operands, into that branch, and the operand lanes of inactive
// queries are then never written (tools/fp8_debug.py: channels of the last query tile came
// out garbage).  The empty volatile asm consuming the result pins the instruction -- and so
// its operands -- where it is written, with every lane active.
__device__ __forceinline__ f32x16_t mfma_mx(i32x8_t a, int sa, i32x8_t b, int sb, f32x16_t c) {
  f32x16_t d = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
  __asm__ volatile("" : "+v"(d));
  return d;
}

// Conversions use gfx950's scaled instructions straight from / to bf16 pairs (one
// instruction per pair and direction): v_cvt_scalef32_pk_fp8_bf16 with scale 2^-k makes
// e4m3(x 2^k), and v_cvt_scalef32_pk_bf16_fp8 with the same scale gives back e4m3 2^-k, both
// bit-identical to the unscaled conversion of the rescaled value
// (tools/micro/cvt_scale_probe.hip, profiles/r3_cvt_scale_probe.txt).
typedef short s16x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v_t __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint4 bits128(bf16x8_t c) { return __builtin_bit_cast(uint4, c); }

// e4m3 bytes of two bf16 pairs, x 2^k (inv = 2^-k)
__device__ __forceinline__ int e4m3x4(unsigned lo, unsigned hi, float inv) {
  s16x2_t r = {0, 0};
  r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, __builtin_bit_cast(bf16x2v_t, lo), inv, false);
  r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, __builtin_bit_cast(bf16x2v_t, hi), inv, true);
  return __builtin_bit_cast(int, r);
}

// largest |x| of 8 bf16 values as bf16 bits (for non-negative bf16, integer order is value
// order): packed 16-bit max over the sign-cleared dwords
__device__ __forceinline__ unsigned amax8_bits(bf16x8_t c) {
  const uint4 u = bits128(c);
  u16x2_t m = __builtin_bit_cast(u16x2_t, u.x & 0x7fff7fffu);
  m = __builtin_elementwise_max(m, __builtin_bit_cast(u16x2_t, u.y & 0x7fff7fffu));
  m = __builtin_elementwise_max(m, __builtin_bit_cast(u16x2_t, u.z & 0x7fff7fffu));
  m = __builtin_elementwise_max(m, __builtin_bit_cast(u16x2_t, u.w & 0x7fff7fffu));
  return m[0] > m[1] ? m[0] : m[1];
}

__device__ __forceinline__ unsigned umax_xor(unsigned v, int sft) {
  const unsigned o = (unsigned)__shfl_xor((int)v, sft, 64);
  return o > v ? o : v;
}

// block scale exponent: the largest k with amax 2^k <= 448 (e4m3 max); 0 for an empty block
__device__ __forceinline__ int mx_exp(float amax) {
  const int k = amax > 0.f ? (int)floorf(log2f(448.f / amax)) : 0;
  return min(max(k, -126), 126);
}

// the same from the amax's bf16 bits: amax = 1.m 2^(e-127) and 448 = 1.75 2^8, so
// k = 135 - e, one less when the mantissa exceeds 1.75 (0x60); subnormals take the float path
__device__ __forceinline__ int mx_exp_bits(unsigned b) {
  if (b < 0x80u) return mx_exp(__uint_as_float(b << 16));
  const int k = 135 - (int)(b >> 7) - ((b & 0x7fu) > 0x60u ? 1 : 0);
  return min(max(k, -126), 126);
}

__device__ __forceinline__ unsigned xhalf_max_bits(unsigned v) { return umax_xor(v, 32); }


}  // namespace vs
