// Shared helpers for the bf16 v_mfma_f32_32x32x16_bf16 kernels (window and masked
// attention).  Fragment layout (lane l: r = l & 31, hh = l >> 5):
//   A: row r, k = 8hh + j;   B: col r, k = 8hh + j;   C/D: col r, row (i&3) + 8(i>>2) + 4hh.
// "Permuted k": when an operand is taken straight from a C tile, the MFMA k index of a
// 16-step t is mapped to C rows 16t + (j&3) + 8(j>>2) + 4hh (i = 8t + j), and the other
// operand is read from LDS in that same order (ld_perm), so no register transpose.
#pragma once
#include "common.h"

namespace vs {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short bf16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ short bf16_bits(float x) {
  const bf16 b = __float2bfloat16(x);
  return *reinterpret_cast<const short*>(&b);
}

__device__ __forceinline__ bf16x8_t ld8(const bf16* p) { return *reinterpret_cast<const bf16x8_t*>(p); }

__device__ __forceinline__ bf16x8_t zero8() {
  const bf16x8_t z = {0, 0, 0, 0, 0, 0, 0, 0};
  return z;
}

__device__ __forceinline__ void zero16(f32x16_t& a) {
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = 0.f;
}

// 8 consecutive C-tile registers (base = 0 or 8) -> bf16 B/A operand (permuted k)
__device__ __forceinline__ bf16x8_t pack8(const f32x16_t& a, int base) {
  bf16x8_t v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = bf16_bits(a[base + j]);
  return v;
}

// operand in the permuted k order from an LDS row: elements base+0..3 and base+8..11
__device__ __forceinline__ bf16x8_t ld_perm(const short* row, int base) {
  const bf16x4_t lo = *reinterpret_cast<const bf16x4_t*>(row + base);
  const bf16x4_t hi = *reinterpret_cast<const bf16x4_t*>(row + base + 8);
  bf16x8_t v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return v;
}

__device__ __forceinline__ f32x16_t mfma16(bf16x8_t a, bf16x8_t b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Workgroup barrier for LDS ordering only: waits for this wave's LDS traffic
// (lgkmcnt), NOT for its outstanding global loads / stores / atomics -- __syncthreads'
// release fence drains vmcnt, so a kernel that issues fire-and-forget atomics before a
// barrier whose only job is LDS reuse would stall on their round trip to L2.  Use only
// where no other wave reads global memory this wave wrote before the barrier.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");   // LDS-only release: lgkmcnt, no vmcnt
  __builtin_amdgcn_s_barrier();                                      // (a builtin: convergent, never duplicated)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// C-tile row of register i for lane half hh
__device__ __forceinline__ constexpr int crow(int i, int hh) { return (i & 3) + 8 * (i >> 2) + 4 * hh; }

}  // namespace vs
