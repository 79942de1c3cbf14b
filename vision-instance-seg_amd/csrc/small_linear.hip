// Weight and bias gradients of a Linear over a few hundred tokens (bf16).
//
// The masked-attention decoder (HF:m2f Mask2FormerMaskedAttentionDecoderLayer: q / k / v /
// out projections, FFN; Mask2FormerMLPPredictionHead) runs its Linears on B x Q = 400
// tokens with 256..2048 features.  Autograd's backward is dW = gY^T X as one library GEMM
// whose 256 x 256 output is a single macro-tile (one CU, ~23 us) plus a separate bias
// reduction (~12 us).  Here one launch computes both:
//   dW[o, i] = sum_t gY[t, o] X[t, i],   db[o] = sum_t gY[t, o]
// A 256-thread workgroup owns a 64 (o) x 64 (i) block of dW and streams the tokens in
// chunks of 64: the gY and X chunks are staged in LDS in their natural [t][feature]
// layout and read as MFMA operands with ds_read_b64_tr_b16 (k = t runs down the rows);
// the next chunk's 16-B loads are in flight while the current chunk's MFMAs run.  The
// product is formed transposed (dW^T tile: a lane holds 4 consecutive i of one o) so the
// output is written with 8-B stores.  Workgroups of the first i-block also sum gY's
// columns for db (f32, fixed order).
#include "common.h"
#include "mfma_util.h"

namespace vs {
namespace {

constexpr int kTC = 64;          // tokens per chunk
constexpr int kBlk = 64;         // output block edge
constexpr int kPitch = 96;       // LDS row pitch (elements): 192 B, 4 consecutive rows -> distinct banks

typedef short bf16x4v_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8_t tr_frag(const bf16* img, int k0, int cbase, int lane) {
  const int hh = lane >> 5;
  const int row = k0 + 8 * hh + ((lane & 15) >> 2);
  const int col = cbase + (lane & 16) + 4 * (lane & 3);
  typedef __attribute__((address_space(3))) bf16x4v_t lds_v4;
  const bf16x4v_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(img + row * kPitch + col));
  const bf16x4v_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(img + (row + 4) * kPitch + col));
  bf16x8_t v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return v;
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const bf16 x = __float2bfloat16(a), y = __float2bfloat16(b);
  return (uint32_t)(*reinterpret_cast<const uint16_t*>(&x)) | ((uint32_t)(*reinterpret_cast<const uint16_t*>(&y)) << 16);
}

// grid: (I / 64, O / 64); gy [T, O], x [T, I], dw [O, I], db [O] (bf16)
__global__ void __launch_bounds__(256) small_wgrad_kernel(const bf16* __restrict__ gy, const bf16* __restrict__ x,
                                                          bf16* __restrict__ dw, bf16* __restrict__ db, int T, int O,
                                                          int I) {
  __shared__ __attribute__((aligned(16))) bf16 sG[kTC * kPitch];
  __shared__ __attribute__((aligned(16))) bf16 sX[kTC * kPitch];
  __shared__ float sB[4][kBlk];
  const int i0 = blockIdx.x * kBlk, o0 = blockIdx.y * kBlk;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int wo = (wave >> 1) * 32, wi = (wave & 1) * 32;   // this wave's 32 x 32 sub-block
  const bool do_bias = db != nullptr && blockIdx.x == 0;
  // staging: chunk = 64 rows x 64 features = 512 16-B pieces per operand, 2 per thread
  uint4 rg[2], rx[2];
  auto load = [&](int t0) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int p = tid + 256 * k;
      const int row = p >> 3, c = (p & 7) * 8;
      const int t = t0 + row;
      rg[k] = t < T ? *reinterpret_cast<const uint4*>(gy + (size_t)t * O + o0 + c) : make_uint4(0, 0, 0, 0);
      rx[k] = t < T ? *reinterpret_cast<const uint4*>(x + (size_t)t * I + i0 + c) : make_uint4(0, 0, 0, 0);
    }
  };
  f32x16_t acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  float bsum = 0.f;
  const int nchunk = (T + kTC - 1) / kTC;
  load(0);
  for (int ch = 0; ch < nchunk; ++ch) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int p = tid + 256 * k;
      const int row = p >> 3, c = (p & 7) * 8;
      *reinterpret_cast<uint4*>(sG + row * kPitch + c) = rg[k];
      *reinterpret_cast<uint4*>(sX + row * kPitch + c) = rx[k];
    }
    __syncthreads();
    if (ch + 1 < nchunk) load((ch + 1) * kTC);
    if (do_bias) {      // column o = tid & 63, rows (tid >> 6) + 4 j
      const int o = tid & 63;
#pragma unroll
      for (int j = 0; j < kTC / 4; ++j) bsum += __bfloat162float(sG[(wave + 4 * j) * kPitch + o]);
    }
#pragma unroll
    for (int s = 0; s < kTC / 16; ++s) {
      // dW^T tile [i][o]: A = X^T (rows i, k = t), B = gY (k = t, cols o)
      const bf16x8_t a = tr_frag(sX, 16 * s, wi, lane);
      const bf16x8_t b = tr_frag(sG, 16 * s, wo, lane);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    }
  }
  // lane column = o (wo + r), rows = i (wi + (k & 3) + 8 (k >> 2) + 4 hh): 4 consecutive i
  bf16* dst = dw + (size_t)(o0 + wo + r) * I + i0 + wi + 4 * hh;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    uint2 w;
    w.x = pack2(acc[4 * g], acc[4 * g + 1]);
    w.y = pack2(acc[4 * g + 2], acc[4 * g + 3]);
    *reinterpret_cast<uint2*>(dst + 8 * g) = w;
  }
  if (do_bias) {
    sB[wave][tid & 63] = bsum;
    __syncthreads();
    if (tid < kBlk) db[o0 + tid] = __float2bfloat16((sB[0][tid] + sB[1][tid]) + (sB[2][tid] + sB[3][tid]));
  }
}

// The same product with the TOKENS split over the four waves: wave w takes the 64-token
// chunks w, w + 4, ... and accumulates the whole 64 x 64 dW^T block (four 32 x 32 MFMA
// tiles) from its own LDS staging, so the chunks' loads are in flight at once instead of
// one after another (400 tokens: two rounds instead of seven); the four partial blocks are
// then summed in LDS in wave order (fixed order: deterministic).  Same operand layout and
// output mapping as small_wgrad_kernel.
__global__ void __launch_bounds__(256) small_wgrad_split_kernel(const bf16* __restrict__ gy,
                                                                const bf16* __restrict__ x, bf16* __restrict__ dw,
                                                                bf16* __restrict__ db, int T, int O, int I) {
  constexpr int kStage = kTC * kPitch;                 // one operand chunk (elements)
  __shared__ __attribute__((aligned(16))) bf16 sbuf[4 * 2 * kStage];   // per wave: gY, X chunks (96 KB)
  __shared__ float sB[4][kBlk];
  const int i0 = blockIdx.x * kBlk, o0 = blockIdx.y * kBlk;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  bf16* sG = sbuf + wave * 2 * kStage;
  bf16* sX = sG + kStage;
  const bool do_bias = db != nullptr && blockIdx.x == 0;
  uint4 rg[8], rx[8];
  auto load = [&](int t0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int p = lane + 64 * k;
      const int row = p >> 3, c = (p & 7) * 8;
      const int t = t0 + row;
      rg[k] = t < T ? *reinterpret_cast<const uint4*>(gy + (size_t)t * O + o0 + c) : make_uint4(0, 0, 0, 0);
      rx[k] = t < T ? *reinterpret_cast<const uint4*>(x + (size_t)t * I + i0 + c) : make_uint4(0, 0, 0, 0);
    }
  };
  f32x16_t acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) zero16(acc[a][b]);
  float bsum = 0.f;
  const int nchunk = (T + kTC - 1) / kTC;
  if (wave < nchunk) load(wave * kTC);
  for (int ch = wave; ch < nchunk; ch += 4) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int p = lane + 64 * k;
      const int row = p >> 3, c = (p & 7) * 8;
      *reinterpret_cast<uint4*>(sG + row * kPitch + c) = rg[k];
      *reinterpret_cast<uint4*>(sX + row * kPitch + c) = rx[k];
    }
    wave_sync();
    if (ch + 4 < nchunk) load((ch + 4) * kTC);
    if (do_bias) {      // column o = lane, this chunk's 64 rows
#pragma unroll 8
      for (int j = 0; j < kTC; ++j) bsum += __bfloat162float(sG[j * kPitch + lane]);
    }
#pragma unroll
    for (int st = 0; st < kTC / 16; ++st)
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const bf16x8_t fa = tr_frag(sX, 16 * st, 32 * a, lane);
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, tr_frag(sG, 16 * st, 32 * b, lane), acc[a][b], 0, 0, 0);
      }
    wave_sync();                              // this wave's staging is rewritten next round
  }
  __syncthreads();
  // partial dW^T blocks [wave][i][o] (f32, over the staging) summed in wave order
  float* red = reinterpret_cast<float*>(sbuf);
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int k = 0; k < 16; ++k)
        red[(wave * kBlk + 32 * a + crow(k, hh)) * kBlk + 32 * b + r] = acc[a][b][k];
  if (do_bias) sB[wave][lane] = bsum;
  __syncthreads();
  // thread -> o = tid & 63, i quad 4 (tid >> 6) + 16 q: 8-B stores of 4 consecutive i
#pragma unroll
  for (int qd = 0; qd < 4; ++qd) {
    const int o = tid & 63, i = 4 * ((tid >> 6) + 4 * qd);
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) t += red[(w * kBlk + i + e) * kBlk + o];
      v[e] = t;
    }
    uint2 wv;
    wv.x = pack2(v[0], v[1]);
    wv.y = pack2(v[2], v[3]);
    *reinterpret_cast<uint2*>(dw + (size_t)(o0 + o) * I + i0 + i) = wv;
  }
  if (do_bias && tid < kBlk) db[o0 + tid] = __float2bfloat16((sB[0][tid] + sB[1][tid]) + (sB[2][tid] + sB[3][tid]));
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" int vs_small_linear_wgrad(int dtype, const void* grad_y, const void* x, void* grad_w, void* grad_b,
                                     int tokens, int out_features, int in_features, void* stream) {
  VS_CHECK(dtype == VS_BF16, "the small-token weight gradient is the bf16 path");
  VS_CHECK(grad_w, "null pointer");
  VS_CHECK(tokens >= 0 && out_features > 0 && in_features > 0, "bad sizes");
  VS_CHECK(out_features % kBlk == 0 && in_features % kBlk == 0, "features must be multiples of 64");
  if (tokens == 0) {
    VS_HIP(hipMemsetAsync(grad_w, 0, (size_t)out_features * in_features * 2, (hipStream_t)stream));
    if (grad_b) VS_HIP(hipMemsetAsync(grad_b, 0, (size_t)out_features * 2, (hipStream_t)stream));
    return VS_OK;
  }
  VS_CHECK(grad_y && x, "null pointer");
  // token split over the waves from 2 chunks up (VS_SMALL_WGRAD_SPLIT=0: the chunk-serial kernel, A/B)
  static const int split = [] {
    const char* e = getenv("VS_SMALL_WGRAD_SPLIT");
    return e ? atoi(e) : 1;
  }();
  if (split && tokens > kTC)
    hipLaunchKernelGGL(small_wgrad_split_kernel, dim3(in_features / kBlk, out_features / kBlk), dim3(256), 0,
                       (hipStream_t)stream, (const bf16*)grad_y, (const bf16*)x, (bf16*)grad_w, (bf16*)grad_b, tokens,
                       out_features, in_features);
  else
    hipLaunchKernelGGL(small_wgrad_kernel, dim3(in_features / kBlk, out_features / kBlk), dim3(256), 0,
                       (hipStream_t)stream, (const bf16*)grad_y, (const bf16*)x, (bf16*)grad_w, (bf16*)grad_b, tokens,
                       out_features, in_features);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
