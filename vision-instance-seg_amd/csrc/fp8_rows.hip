// Row-wise e4m3 quantisation for the vendor fp8 GEMM (config C5's fp8 Linears).
//
// hipBLASLt's fp8 GEMM with one f32 scale per row of each operand (torch._scaled_mm,
// "rowwise": out[m, n] = sa[m] sb[n] sum_k qa[m, k] qb[n, k]) ran the K-deep Swin-L
// Linears 1.5-1.7x faster than the bf16 GEMM on the box (tools/r5/scaled_mm_probe.py,
// profiles/r5_scaled_mm_probe.txt), where the hand-written MX token GEMM reached 1.0-1.4
// PF/s.  Its operands are e4m3 rows with a per-row scale: here x bf16 [M, K] -> q e4m3
// [M, K] and scale f32 [M] with x ~= q * scale, scale a power of two (2^-k, k the largest
// exponent with amax 2^k <= 448, the MX rule of mx_util.h per row instead of per 32), so
// q * scale is the e4m3 rounding of x exactly.
//
// GELU variant: y = gelu(h) (exact erf, HF:swin:511-536) stored in bf16 (the next
// Linear's weight gradient reads it) and quantised in the same pass -- the fc1 -> fc2 hand-off
// of the Swin MLP reads the pre-activation once.
//
// Layout: G lanes per row (a power of two, <= 64), 64 / G rows per wave, each lane owns
// 8-element (16 B) chunks c = lane, lane + G, ...; the row amax is a G-lane shuffle max of
// the chunks' bf16 bit patterns (sign cleared: integer order = value order).
#include "common.h"
#include "mfma_util.h"
#include "mx_util.h"

namespace vs {
namespace {

constexpr int kMaxCpl = 16;       // chunks per lane: K <= 64 x 16 x 8 = 8192

// gelu(x) = 0.5 x (1 + erf(x / sqrt2)) with erf from one exponential (Abramowitz-Stegun
// 7.1.26, |error| <= 1.5e-7, the rule of norm.hip's GELU backward): erff's branches made this
// pass VALU-bound at 2.6 TB/s (0.217 ms per C5 stage-3 launch against the ATen GELU's 0.10)
__device__ __forceinline__ bf16x8_t gelu8(bf16x8_t h) {
  bf16x8_t y;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = bf16_bits_to_f32((unsigned short)h[j]);
    const float e = __expf(-0.5f * x * x);
    const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, fabsf(x), 1.f));
    const float poly =
        t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f), 0.254829592f);
    const float ea = fmaf(-poly, e, 1.f);
    y[j] = bf16_bits(0.5f * x * (1.f + (x < 0.f ? -ea : ea)));
  }
  return y;
}

template <int CPL, bool GELU>
__global__ void __launch_bounds__(256) row_quant_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                        unsigned char* __restrict__ q, float* __restrict__ scale,
                                                        int M, int K, int G) {
  const int lane = threadIdx.x & 63;
  const int rpw = 64 / G;                                        // rows per wave
  const int row = (blockIdx.x * 4 + (threadIdx.x >> 6)) * rpw + lane / G;
  const int g = lane % G;
  const int nch = K >> 3;
  const bool live = row < M;
  const bf16* xr = x + (size_t)row * K;
  bf16x8_t c[CPL];
  unsigned amax = 0;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int ch = g + i * G;
    c[i] = (live && ch < nch) ? ld8(xr + 8 * ch) : zero8();
    if (GELU) c[i] = gelu8(c[i]);
    const unsigned m = amax8_bits(c[i]);
    amax = m > amax ? m : amax;
  }
  for (int s = 1; s < G; s <<= 1) amax = umax_xor(amax, s);
  const int k = mx_exp_bits(amax);                               // amax 2^k <= 448
  const float inv = __uint_as_float((unsigned)(127 - k) << 23);  // 2^-k: e4m3(x 2^k)
  if (!live) return;
  if (g == 0) scale[row] = inv;                                  // x ~= q 2^-k
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int ch = g + i * G;
    if (ch < nch) {
      const uint4 u = bits128(c[i]);
      const int lo = e4m3x4(u.x, u.y, inv), hi = e4m3x4(u.z, u.w, inv);
      *reinterpret_cast<int2*>(q + (size_t)row * K + 8 * ch) = make_int2(lo, hi);
      if (GELU) *reinterpret_cast<bf16x8_t*>(y + (size_t)row * K + 8 * ch) = c[i];
    }
  }
}

}  // namespace
}  // namespace vs

using namespace vs;

static int row_quant_impl(const void* x, void* y, void* q, float* scale, int M, int K, bool gelu, void* stream) {
  VS_CHECK(M >= 0 && K > 0 && K % 8 == 0 && K <= 64 * kMaxCpl * 8, "K must be a multiple of 8, <= 8192");
  if (M == 0) return VS_OK;
  VS_CHECK(x && q && scale && (!gelu || y), "null pointer");
  VS_CHECK(((uintptr_t)x & 15) == 0 && ((uintptr_t)q & 7) == 0 && (!gelu || ((uintptr_t)y & 15) == 0),
           "x / y must be 16-B aligned, q 8-B aligned");
  const int nch = K / 8;
  int G = 1;
  while (G < nch && G < 64) G <<= 1;
  const int cpl = (nch + G - 1) / G;
  const int rows_per_block = 4 * (64 / G);
  const dim3 grid((unsigned)((M + rows_per_block - 1) / rows_per_block));
  hipStream_t st = (hipStream_t)stream;
#define VS_RQ(C)                                                                                                    \
  if (gelu)                                                                                                         \
    hipLaunchKernelGGL((row_quant_kernel<C, true>), grid, dim3(256), 0, st, (const bf16*)x, (bf16*)y,              \
                       (unsigned char*)q, scale, M, K, G);                                                          \
  else                                                                                                              \
    hipLaunchKernelGGL((row_quant_kernel<C, false>), grid, dim3(256), 0, st, (const bf16*)x, (bf16*)nullptr,       \
                       (unsigned char*)q, scale, M, K, G)
  if (cpl <= 1) {
    VS_RQ(1);
  } else if (cpl <= 2) {
    VS_RQ(2);
  } else if (cpl <= 3) {
    VS_RQ(3);
  } else if (cpl <= 4) {
    VS_RQ(4);
  } else if (cpl <= 6) {
    VS_RQ(6);
  } else if (cpl <= 8) {
    VS_RQ(8);
  } else if (cpl <= 12) {
    VS_RQ(12);
  } else {
    VS_RQ(16);
  }
#undef VS_RQ
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_row_quantize_fp8(const void* x, void* q, float* scale, int M, int K, void* stream) {
  return row_quant_impl(x, nullptr, q, scale, M, K, false, stream);
}

extern "C" int vs_gelu_row_quantize_fp8(const void* h, void* y, void* q, float* scale, int M, int K, void* stream) {
  return row_quant_impl(h, y, q, scale, M, K, true, stream);
}
