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
constexpr int kStage = kTC * kPitch;                   // one operand chunk (elements)
constexpr int kSplitLds = 4 * 2 * kStage;               // per wave: gY, X chunks (96 KB)

__device__ __forceinline__ void wgrad_split_block(bf16* sbuf, float (*sB)[kBlk], int bx, int by,
                                                  const bf16* __restrict__ gy, const bf16* __restrict__ x,
                                                  bf16* __restrict__ dw, bf16* __restrict__ db, int T, int O, int I) {
  const int i0 = bx * kBlk, o0 = by * kBlk;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  bf16* sG = sbuf + wave * 2 * kStage;
  bf16* sX = sG + kStage;
  const bool do_bias = db != nullptr && bx == 0;
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

__global__ void __launch_bounds__(256) small_wgrad_split_kernel(const bf16* __restrict__ gy,
                                                                const bf16* __restrict__ x, bf16* __restrict__ dw,
                                                                bf16* __restrict__ db, int T, int O, int I) {
  __shared__ __attribute__((aligned(16))) bf16 sbuf[kSplitLds];
  __shared__ float sB[4][kBlk];
  wgrad_split_block(sbuf, sB, blockIdx.x, blockIdx.y, gy, x, dw, db, T, O, I);
}

// ---- forward and input gradient --------------------------------------------------------
// Y = X W^T + b and dX = dY W over a few hundred tokens, formed transposed so a lane's
// accumulator column is one token and its rows 4 consecutive features (8-B stores):
//   Y^T[o][t]  = sum_i W[o][i] X[t][i]     A = W rows (16-B loads), B = X rows (16-B loads)
//   dX^T[i][t] = sum_o W[o][i] dY[t][o]    A = W^T (W chunk staged in LDS, transposed
//                                          reads), B = dY rows (16-B loads)
// A workgroup owns a 32 (feature) x 32 (token) output tile; its four waves split the
// reduction (K) into quarters, and the quarter sums are added in wave order in LDS (f32,
// fixed order: deterministic), the bias added last.  A launch is a few microseconds of
// latency at these sizes: the split puts four waves' loads in flight per tile.
constexpr int kRT = 32;          // output tile edge
constexpr int kWC = 64;          // W rows per LDS chunk (input-gradient path)

template <bool TRANS_A>
__device__ __forceinline__ void reduce_tile(bf16* sbuf, int tt, int ft, const bf16* __restrict__ w,
                                            const bf16* __restrict__ bmat, const bf16* __restrict__ bias,
                                            bf16* __restrict__ out, int T, int K, int ldw, int F) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int t0 = tt * kRT, f0 = ft * kRT;
  const int kq = K / 4, kb = wave * kq;                       // this wave's K quarter (multiple of 16)
  const int t = t0 + r;
  const bf16* brow = bmat + (size_t)min(t, T - 1) * K + kb + 8 * hh;   // B: token row t, k contiguous
  const bool tv = t < T;
  f32x16_t acc;
  zero16(acc);
  if (!TRANS_A) {
    const bf16* arow = w + (size_t)(f0 + r) * ldw + kb + 8 * hh;       // A: W row o = f0 + r
    for (int k = 0; k < kq; k += 64) {
      bf16x8_t a[4], b[4];
      const int ns = min(4, (kq - k) >> 4);
#pragma unroll
      for (int s = 0; s < 4; ++s)
        if (s < ns) {
          a[s] = ld8(arow + k + 16 * s);
          b[s] = tv ? ld8(brow + k + 16 * s) : zero8();
        }
#pragma unroll
      for (int s = 0; s < 4; ++s)
        if (s < ns) acc = mfma16(a[s], b[s], acc);
    }
  } else {
    bf16* sW = sbuf + wave * kWC * kPitch;                    // this wave's W chunk [o][32 i]
    for (int k = 0; k < kq; k += kWC) {
      const int rows = min(kWC, kq - k);
      uint4 wv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {                           // 64 rows x 64 B: lane -> (row, 16-B piece)
        const int p = lane + 64 * q, row = p >> 2, c = (p & 3) * 8;
        wv[q] = row < rows ? *reinterpret_cast<const uint4*>(w + (size_t)(kb + k + row) * ldw + f0 + c)
                           : make_uint4(0, 0, 0, 0);
      }
      bf16x8_t b[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) b[s] = (tv && 16 * s < rows) ? ld8(brow + k + 16 * s) : zero8();
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int p = lane + 64 * q, row = p >> 2, c = (p & 3) * 8;
        *reinterpret_cast<uint4*>(sW + row * kPitch + c) = wv[q];
      }
      wave_sync();
#pragma unroll
      for (int s = 0; s < 4; ++s)
        if (16 * s < rows) acc = mfma16(tr_frag(sW, 16 * s, 0, lane), b[s], acc);
      wave_sync();                                            // the chunk is rewritten next round
    }
  }
  __syncthreads();
  float* red = reinterpret_cast<float*>(sbuf);                // [wave][feature 32][token 32]
#pragma unroll
  for (int i = 0; i < 16; ++i) red[(wave * kRT + crow(i, hh)) * kRT + r] = acc[i];
  __syncthreads();
  {  // thread -> token tid & 31, features 4 (tid >> 5) .. + 3
    const int tk = tid & 31, fq = 4 * (tid >> 5), tg = t0 + tk;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float s_ = red[(0 * kRT + fq + e) * kRT + tk];
#pragma unroll
      for (int wv_ = 1; wv_ < 4; ++wv_) s_ += red[(wv_ * kRT + fq + e) * kRT + tk];
      v[e] = bias ? s_ + __bfloat162float(bias[f0 + fq + e]) : s_;
    }
    if (tg < T) {
      uint2 o;
      o.x = pack2(v[0], v[1]);
      o.y = pack2(v[2], v[3]);
      *reinterpret_cast<uint2*>(out + (size_t)tg * F + f0 + fq) = o;
    }
  }
}

// grid (ceil(T / 32), O / 32): y [T, O] = x [T, I] w[O, I]^T + b
__global__ void __launch_bounds__(256) small_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                        const bf16* __restrict__ b, bf16* __restrict__ y, int T,
                                                        int O, int I) {
  __shared__ __attribute__((aligned(16))) bf16 sbuf[4 * kRT * kRT * 2];   // the f32 reduction (16 KB)
  reduce_tile<false>(sbuf, blockIdx.x, blockIdx.y, w, x, b, y, T, I, I, O);
}

// One launch for the whole backward: blocks [0, nx) are dX tiles (ceil(T / 32) x I / 32,
// when dx is requested), the rest the token-split dW / db blocks (I / 64 x O / 64).
__global__ void __launch_bounds__(256) small_bwd_kernel(const bf16* __restrict__ gy, const bf16* __restrict__ x,
                                                        const bf16* __restrict__ w, bf16* __restrict__ dx,
                                                        bf16* __restrict__ dw, bf16* __restrict__ db, int T, int O,
                                                        int I, int nx) {
  __shared__ __attribute__((aligned(16))) bf16 sbuf[kSplitLds];
  __shared__ float sB[4][kBlk];
  const int blk = blockIdx.x;
  const int ntt = (T + kRT - 1) / kRT;
  if (blk < nx) {
    reduce_tile<true>(sbuf, blk % ntt, blk / ntt, w, gy, nullptr, dx, T, O, I, I);
  } else {
    const int wb = blk - nx, nbx = I / kBlk;
    wgrad_split_block(sbuf, sB, wb % nbx, wb / nbx, gy, x, dw, db, T, O, I);
  }
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

extern "C" int vs_small_linear_forward(int dtype, const void* x, const void* weight, const void* bias, void* y,
                                       int tokens, int out_features, int in_features, void* stream) {
  VS_CHECK(dtype == VS_BF16, "the small-token Linear is the bf16 path");
  VS_CHECK(tokens >= 0 && out_features > 0 && in_features > 0, "bad sizes");
  VS_CHECK(out_features % kBlk == 0 && in_features % kBlk == 0, "features must be multiples of 64");
  if (tokens == 0) return VS_OK;
  VS_CHECK(x && weight && y, "null pointer");
  hipLaunchKernelGGL(small_fwd_kernel, dim3((tokens + kRT - 1) / kRT, out_features / kRT), dim3(256), 0,
                     (hipStream_t)stream, (const bf16*)x, (const bf16*)weight, (const bf16*)bias, (bf16*)y, tokens,
                     out_features, in_features);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_small_linear_backward(int dtype, const void* grad_y, const void* x, const void* weight,
                                        void* grad_x, void* grad_w, void* grad_b, int tokens, int out_features,
                                        int in_features, void* stream) {
  VS_CHECK(dtype == VS_BF16, "the small-token Linear is the bf16 path");
  VS_CHECK(tokens >= 0 && out_features > 0 && in_features > 0, "bad sizes");
  VS_CHECK(out_features % kBlk == 0 && in_features % kBlk == 0, "features must be multiples of 64");
  VS_CHECK(grad_w || grad_x, "nothing to compute");
  hipStream_t st = (hipStream_t)stream;
  if (tokens == 0) {
    if (grad_w) VS_HIP(hipMemsetAsync(grad_w, 0, (size_t)out_features * in_features * 2, st));
    if (grad_b) VS_HIP(hipMemsetAsync(grad_b, 0, (size_t)out_features * 2, st));
    return VS_OK;
  }
  VS_CHECK(grad_y && (!grad_x || weight) && (!grad_w || x), "null pointer");
  if (!grad_w) VS_CHECK(!grad_b, "grad_b needs grad_w");
  const int nx = grad_x ? ((tokens + kRT - 1) / kRT) * (in_features / kRT) : 0;
  const int nw = grad_w ? (in_features / kBlk) * (out_features / kBlk) : 0;
  hipLaunchKernelGGL(small_bwd_kernel, dim3(nx + nw), dim3(256), 0, st, (const bf16*)grad_y, (const bf16*)x,
                     (const bf16*)weight, (bf16*)grad_x, (bf16*)grad_w, (bf16*)grad_b, tokens, out_features,
                     in_features, nx);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
