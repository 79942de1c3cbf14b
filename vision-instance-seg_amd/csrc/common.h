// Shared helpers for the visionseg HIP kernels (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include <string>

#include "../../include/visionseg.h"

namespace vs {

// --- error plumbing: every C entry point returns VS_OK or an error code and leaves a
// message retrievable with vs_last_error() (thread-local, like errno).
void set_error(const std::string& msg);

#define VS_CHECK(cond, msg)                                                     \
  do {                                                                          \
    if (!(cond)) {                                                              \
      ::vs::set_error(std::string(__func__) + ": " + (msg));                    \
      return VS_ERR_INVALID;                                                    \
    }                                                                           \
  } while (0)

#define VS_HIP(expr)                                                            \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess) {                                                     \
      ::vs::set_error(std::string(__func__) + ": " #expr ": " +                 \
                      hipGetErrorString(_e));                                   \
      return VS_ERR_HIP;                                                        \
    }                                                                           \
  } while (0)

#define VS_LAUNCH_CHECK() VS_HIP(hipGetLastError())

using bf16 = __hip_bfloat16;

// d/dx of torch's exact GELU 0.5 x (1 + erf(x / sqrt2)): 0.5 (1 + erf(x / sqrt2)) + x
// exp(-x^2 / 2) / sqrt(2 pi), with erf(|x| / sqrt2) = 1 - t poly(t) e^{-x^2/2}, t = 1 / (1 +
// p |x| / sqrt2) (Abramowitz-Stegun 7.1.26, |error| <= 1.5e-7): the exponential is the one
// the density term needs anyway, so one exp + one reciprocal per element.  Shared by the
// activation backward (norm.hip) and the dX GEMM's fused GELU-backward epilogue
// (token_gemm.hip), so both produce the same bits.
__device__ __forceinline__ float gelu_grad_erf(float xv) {
  const float e = __expf(-0.5f * xv * xv);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, fabsf(xv), 1.f));
  const float poly =
      t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f), 0.254829592f);
  const float erf_abs = fmaf(-poly, e, 1.f);
  const float erf_v = xv < 0.f ? -erf_abs : erf_abs;
  return fmaf(0.5f, erf_v, 0.5f) + xv * 0.39894228040143268f * e;
}

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return __bfloat162float(x); }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return __float2bfloat16(x); }

// bf16 bit pattern <-> f32 without a library call (exact widening).
__device__ __forceinline__ float bf16_bits_to_f32(uint32_t u16) { return __uint_as_float(u16 << 16); }

// XCD-aware workgroup remap (cdna_hip_programming.md T1, bijective form): the dispatcher
// round-robins consecutive workgroups over the 8 XCDs, each with its own L2; this gives
// every XCD a contiguous range of logical workgroup ids instead.  Speed only.
__device__ __forceinline__ int xcd_swizzle(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// 16-byte vector of T (8 bf16 or 4 f32) loaded/stored in one instruction.
template <typename T> struct Vec16;
template <> struct Vec16<float> {
  static constexpr int N = 4;
  __device__ __forceinline__ static void load(const float* p, float* out) {
    float4 v = *reinterpret_cast<const float4*>(p);
    out[0] = v.x; out[1] = v.y; out[2] = v.z; out[3] = v.w;
  }
  __device__ __forceinline__ static void store(float* p, const float* in) {
    *reinterpret_cast<float4*>(p) = make_float4(in[0], in[1], in[2], in[3]);
  }
};
template <> struct Vec16<bf16> {
  static constexpr int N = 8;
  __device__ __forceinline__ static void load(const bf16* p, float* out) {
    uint4 v = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      out[2 * i] = __uint_as_float(w[i] << 16);
      out[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ __forceinline__ static void store(bf16* p, const float* in) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bf16 lo = __float2bfloat16(in[2 * i]);
      bf16 hi = __float2bfloat16(in[2 * i + 1]);
      w[i] = (uint32_t)(*reinterpret_cast<uint16_t*>(&lo)) |
             ((uint32_t)(*reinterpret_cast<uint16_t*>(&hi)) << 16);
    }
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};

inline int grid_for(long long work, int block, int cap = 256 * 16) {
  long long g = (work + block - 1) / block;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace vs
