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

// x + pos rounded to bf16 (torch's bf16 add: f32 sum, one rounding), 8 elements
__device__ __forceinline__ uint4 add_bf16x8(uint4 a, uint4 b) {
  const uint32_t* pa = reinterpret_cast<const uint32_t*>(&a);
  const uint32_t* pb = reinterpret_cast<const uint32_t*>(&b);
  uint4 o;
  uint32_t* po = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    po[j] = pack2(bf16_bits_to_f32(pa[j] & 0xffffu) + bf16_bits_to_f32(pb[j] & 0xffffu),
                  bf16_bits_to_f32(pa[j] >> 16) + bf16_bits_to_f32(pb[j] >> 16));
  return o;
}

// g where the ReLU output y > 0, else 0 (relu'(x) as torch's threshold_backward on the
// result), 8 bf16 elements
__device__ __forceinline__ uint4 mask_bf16x8(uint4 g, uint4 y) {
  const uint32_t* pg = reinterpret_cast<const uint32_t*>(&g);
  const uint32_t* py = reinterpret_cast<const uint32_t*>(&y);
  uint4 o;
  uint32_t* po = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t lo = py[j] & 0xffffu, hi = py[j] >> 16;
    const uint32_t keep = ((lo != 0u && !(lo & 0x8000u)) ? 0x0000ffffu : 0u) |
                          ((hi != 0u && !(hi & 0x8000u)) ? 0xffff0000u : 0u);
    po[j] = pg[j] & keep;
  }
  return o;
}

__device__ __forceinline__ bf16x8_t mask8(bf16x8_t g, bf16x8_t y) {
  const uint4 o = mask_bf16x8(*reinterpret_cast<const uint4*>(&g), *reinterpret_cast<const uint4*>(&y));
  return *reinterpret_cast<const bf16x8_t*>(&o);
}

__device__ __forceinline__ bf16x8_t add8(bf16x8_t a, bf16x8_t b) {
  const uint4 o = add_bf16x8(*reinterpret_cast<const uint4*>(&a), *reinterpret_cast<const uint4*>(&b));
  return *reinterpret_cast<const bf16x8_t*>(&o);
}

// pos (may be NULL): the x operand is x + pos (the decoder's query + query-position input),
// pos row t % prows (prows = Q: one query-position table broadcast over the batch);
// gmask (may be NULL): gY is masked by a ReLU output of gY's shape (fused ReLU backward)
__device__ __forceinline__ void wgrad_split_block(bf16* sbuf, float (*sB)[kBlk], int bx, int by,
                                                  const bf16* __restrict__ gy, const bf16* __restrict__ x,
                                                  bf16* __restrict__ dw, bf16* __restrict__ db, int T, int O, int I,
                                                  const bf16* __restrict__ pos = nullptr, int prows = 1,
                                                  const bf16* __restrict__ gmask = nullptr) {
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
      if (gmask && t < T)
        rg[k] = mask_bf16x8(rg[k], *reinterpret_cast<const uint4*>(gmask + (size_t)t * O + o0 + c));
      rx[k] = t < T ? *reinterpret_cast<const uint4*>(x + (size_t)t * I + i0 + c) : make_uint4(0, 0, 0, 0);
      if (pos && t < T)
        rx[k] = add_bf16x8(rx[k], *reinterpret_cast<const uint4*>(pos + (size_t)(t % prows) * I + i0 + c));
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

// One wave's partial product over k in [kb, kb + klen) (klen a multiple of 16) for the
// tile (features f0.., tokens t0..): !TRANS_A: A = W rows [f][k]; TRANS_A: A = W^T, W rows
// k, columns f (staged through this wave's LDS chunk sW).  B = token rows of bmat (ldb
// elements per row) + pos row t % prows (pos may be NULL), masked where bmask (a ReLU
// output of bmat's shape, may be NULL) is not positive.
template <bool TRANS_A>
__device__ __forceinline__ f32x16_t tile_partial(bf16* sW, const bf16* __restrict__ w, int ldw,
                                                 const bf16* __restrict__ bmat, const bf16* __restrict__ pos, int ldb,
                                                 int kb, int klen, int T, int t0, int f0, int prows = 1,
                                                 const bf16* __restrict__ bmask = nullptr) {
  const int lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int t = t0 + r;
  const bool tv = t < T;
  const int tc = min(t, T - 1);
  const size_t boff = (size_t)tc * ldb + kb + 8 * hh;             // B: token row t, k contiguous
  const size_t poff = (size_t)(tc % prows) * ldb + kb + 8 * hh;
  auto ldb8 = [&](int k) {
    if (!tv) return zero8();
    bf16x8_t v = ld8(bmat + boff + k);
    if (bmask) v = mask8(v, ld8(bmask + boff + k));
    return pos ? add8(v, ld8(pos + poff + k)) : v;
  };
  f32x16_t acc;
  zero16(acc);
  if (!TRANS_A) {
    const bf16* arow = w + (size_t)(f0 + r) * ldw + kb + 8 * hh;     // A: W row f0 + r
    for (int k = 0; k < klen; k += 64) {
      bf16x8_t a[4], b[4];
      const int ns = min(4, (klen - k) >> 4);
#pragma unroll
      for (int s = 0; s < 4; ++s)
        if (s < ns) {
          a[s] = ld8(arow + k + 16 * s);
          b[s] = ldb8(k + 16 * s);
        }
#pragma unroll
      for (int s = 0; s < 4; ++s)
        if (s < ns) acc = mfma16(a[s], b[s], acc);
    }
  } else {
    for (int k = 0; k < klen; k += kWC) {
      const int rows = min(kWC, klen - k);
      uint4 wv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {                           // 64 rows x 64 B: lane -> (row, 16-B piece)
        const int p = lane + 64 * q, row = p >> 2, c = (p & 3) * 8;
        wv[q] = row < rows ? *reinterpret_cast<const uint4*>(w + (size_t)(kb + k + row) * ldw + f0 + c)
                           : make_uint4(0, 0, 0, 0);
      }
      bf16x8_t b[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) b[s] = 16 * s < rows ? ldb8(k + 16 * s) : zero8();
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
  return acc;
}

// The four waves' partials -> LDS [wave][feature 32][token 32] (f32), after a barrier
__device__ __forceinline__ float* stash_partials(bf16* sbuf, const f32x16_t& acc) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, hh = lane >> 5;
  __syncthreads();
  float* red = reinterpret_cast<float*>(sbuf);
#pragma unroll
  for (int i = 0; i < 16; ++i) red[(wave * kRT + crow(i, hh)) * kRT + r] = acc[i];
  __syncthreads();
  return red;
}

// thread -> token tid & 31, features 4 (tid >> 5) .. + 3: 8-B store of 4 values
__device__ __forceinline__ void store_quad(bf16* __restrict__ out, int ld, int T, int t0, int f0, const float* v) {
  const int tid = threadIdx.x, tg = t0 + (tid & 31), fq = 4 * (tid >> 5);
  if (tg < T) {
    uint2 o;
    o.x = pack2(v[0], v[1]);
    o.y = pack2(v[2], v[3]);
    *reinterpret_cast<uint2*>(out + (size_t)tg * ld + f0 + fq) = o;
  }
}

// v[0..3] += src[token tg][features f .. f + 3] (bf16), when src is non-NULL and tg < T
__device__ __forceinline__ void add_quad(const bf16* __restrict__ src, int ld, int T, int tg, int f, float* v) {
  if (!src || tg >= T) return;
  const uint2 q = *reinterpret_cast<const uint2*>(src + (size_t)tg * ld + f);
  v[0] += bf16_bits_to_f32(q.x & 0xffffu);
  v[1] += bf16_bits_to_f32(q.x >> 16);
  v[2] += bf16_bits_to_f32(q.y & 0xffffu);
  v[3] += bf16_bits_to_f32(q.y >> 16);
}

template <bool TRANS_A>
__device__ __forceinline__ void reduce_tile(bf16* sbuf, int tt, int ft, const bf16* __restrict__ w,
                                            const bf16* __restrict__ bmat, const bf16* __restrict__ pos,
                                            const bf16* __restrict__ bias, bf16* __restrict__ out, int T, int K,
                                            int ldw, int F, int prows = 1, const bf16* __restrict__ bmask = nullptr,
                                            bool relu = false, bf16* __restrict__ out2 = nullptr,
                                            bool acc2 = false, const bf16* __restrict__ add_in = nullptr) {
  const int wave = threadIdx.x >> 6;
  const int t0 = tt * kRT, f0 = ft * kRT, kq = K / 4;        // this wave's K quarter (multiple of 16)
  const f32x16_t acc = tile_partial<TRANS_A>(sbuf + wave * kWC * kPitch, w, ldw, bmat, pos, K, wave * kq, kq, T,
                                             t0, f0, prows, bmask);
  const float* red = stash_partials(sbuf, acc);
  const int tk = threadIdx.x & 31, fq = 4 * (threadIdx.x >> 5);
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float s_ = red[(0 * kRT + fq + e) * kRT + tk];
#pragma unroll
    for (int w_ = 1; w_ < 4; ++w_) s_ += red[(w_ * kRT + fq + e) * kRT + tk];
    v[e] = bias ? s_ + __bfloat162float(bias[f0 + fq + e]) : s_;
    if (relu) v[e] = fmaxf(v[e], 0.f);
  }
  const int tg = t0 + tk;
  if (out2) {                                 // the position rows' gradient (+= when accumulating)
    float v2[4] = {v[0], v[1], v[2], v[3]};
    if (acc2) add_quad(out2, F, T, tg, f0 + fq, v2);
    store_quad(out2, F, T, t0, f0, v2);
  }
  add_quad(add_in, F, T, tg, f0 + fq, v);     // the residual gradient (ops.ResidualSink)
  store_quad(out, F, T, t0, f0, v);
}

// grid (ceil(T / 32), O / 32): y [T, O] = [relu](x (+ pos) [T, I] w[O, I]^T + b)
__global__ void __launch_bounds__(256) small_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ pos,
                                                        int prows, const bf16* __restrict__ w,
                                                        const bf16* __restrict__ b, int relu, bf16* __restrict__ y,
                                                        int T, int O, int I) {
  __shared__ __attribute__((aligned(16))) bf16 sbuf[4 * kRT * kRT * 2];   // the f32 reduction (16 KB)
  reduce_tile<false>(sbuf, blockIdx.x, blockIdx.y, w, x, pos, b, y, T, I, I, O, prows, nullptr, relu != 0);
}

// One launch for the whole backward: blocks [0, nx) are dX tiles (ceil(T / 32) x I / 32,
// when dx is requested), the rest the token-split dW / db blocks (I / 64 x O / 64).  pos:
// the forward's x + pos operand (dW); ymask: the forward's ReLU output (gY masked by it).
__global__ void __launch_bounds__(256) small_bwd_kernel(const bf16* __restrict__ gy, const bf16* __restrict__ x,
                                                        const bf16* __restrict__ pos, int prows,
                                                        const bf16* __restrict__ w, const bf16* __restrict__ ymask,
                                                        bf16* __restrict__ dx, bf16* __restrict__ dpos,
                                                        bf16* __restrict__ dw, bf16* __restrict__ db, int T, int O,
                                                        int I, int nx, const bf16* __restrict__ gres, int acc_pos) {
  __shared__ __attribute__((aligned(16))) bf16 sbuf[kSplitLds];
  __shared__ float sB[4][kBlk];
  const int blk = blockIdx.x;
  const int ntt = (T + kRT - 1) / kRT;
  if (blk < nx) {
    reduce_tile<true>(sbuf, blk % ntt, blk / ntt, w, gy, nullptr, nullptr, dx, T, O, I, I, 1, ymask, false, dpos,
                      acc_pos != 0, gres);
  } else {
    const int wb = blk - nx, nbx = I / kBlk;
    wgrad_split_block(sbuf, sB, wb % nbx, wb / nbx, gy, x, dw, db, T, O, I, pos, prows, ymask);
  }
}

// ---- the self-attention input projections of a decoder layer ------------------------------
// q = (h + pos) Wq^T + bq, k = (h + pos) Wk^T + bk, v = h Wv^T + bv (HF:m2f
// Mask2FormerAttention: queries and keys carry the query position embedding, values do
// not), all [T, D] with D x D weights.  Forward: one launch, the tile's group picked by its
// feature block, h + pos formed in the operand loads (bf16-rounded like torch's add).
// Backward: one launch --
//   dpos = dq Wq + dk Wk             (the position embedding's gradient)
//   dh   = dpos + dv Wv              (h's, every use summed in-kernel: no autograd adds)
// per dX tile wave 0 takes the q term, wave 1 the k term, waves 2 / 3 the two halves of the
// v term, summed in that order; plus the three groups' token-split dW / db blocks.
struct QkvPtrs {
  const bf16* w[3];
  const bf16* b[3];
  bf16* y[3];
  const bf16* dy[3];
  bf16* dw[3];
  bf16* db[3];
};

__global__ void __launch_bounds__(256) qkv_fwd_kernel(const bf16* __restrict__ h, const bf16* __restrict__ pos,
                                                      QkvPtrs p, int T, int D, int prows) {
  __shared__ __attribute__((aligned(16))) bf16 sbuf[4 * kRT * kRT * 2];
  const int fpg = D / kRT, g = blockIdx.y / fpg, ft = blockIdx.y % fpg;
  reduce_tile<false>(sbuf, blockIdx.x, ft, p.w[g], h, g < 2 ? pos : nullptr, p.b[g], p.y[g], T, D, D, D, prows);
}

__global__ void __launch_bounds__(256) qkv_bwd_kernel(const bf16* __restrict__ h, const bf16* __restrict__ pos,
                                                      QkvPtrs p, bf16* __restrict__ dh, bf16* __restrict__ dpos,
                                                      int T, int D, int nx, int prows, const bf16* __restrict__ gres,
                                                      int acc_pos) {
  __shared__ __attribute__((aligned(16))) bf16 sbuf[kSplitLds];
  __shared__ float sB[4][kBlk];
  const int blk = blockIdx.x;
  const int ntt = (T + kRT - 1) / kRT;
  if (blk < nx) {
    const int wave = threadIdx.x >> 6;
    const int t0 = (blk % ntt) * kRT, f0 = (blk / ntt) * kRT;
    const int g = wave < 2 ? wave : 2;
    const int kb = wave < 2 ? 0 : (wave - 2) * (D / 2), klen = wave < 2 ? D : D / 2;
    const f32x16_t acc = tile_partial<true>(sbuf + wave * kWC * kPitch, p.w[g], D, p.dy[g], nullptr, D, kb, klen,
                                            T, t0, f0);
    const float* red = stash_partials(sbuf, acc);
    const int tk = threadIdx.x & 31, fq = 4 * (threadIdx.x >> 5);
    float vp[4], vh[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int o = (fq + e) * kRT + tk;
      vp[e] = red[0 * kRT * kRT + o] + red[1 * kRT * kRT + o];
      vh[e] = vp[e] + (red[2 * kRT * kRT + o] + red[3 * kRT * kRT + o]);
    }
    if (dpos) {
      if (acc_pos) add_quad(dpos, D, T, t0 + tk, f0 + fq, vp);
      store_quad(dpos, D, T, t0, f0, vp);
    }
    add_quad(gres, D, T, t0 + tk, f0 + fq, vh);
    store_quad(dh, D, T, t0, f0, vh);
  } else {
    const int nb = (D / kBlk) * (D / kBlk);
    const int wb = blk - nx, g = wb / nb, r_ = wb % nb;
    wgrad_split_block(sbuf, sB, r_ % (D / kBlk), r_ / (D / kBlk), p.dy[g], h, p.dw[g], p.db[g], T, D, D,
                      g < 2 ? pos : nullptr, prows);
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
  // token split over the waves from 2 chunks up (the chunk-serial kernel for one chunk)
  if (tokens > kTC)
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

extern "C" int vs_small_linear_forward(int dtype, const void* x, const void* pos, int pos_rows, const void* weight,
                                       const void* bias, int relu, void* y, int tokens, int out_features,
                                       int in_features, void* stream) {
  VS_CHECK(dtype == VS_BF16, "the small-token Linear is the bf16 path");
  VS_CHECK(tokens >= 0 && out_features > 0 && in_features > 0, "bad sizes");
  VS_CHECK(!pos || (pos_rows > 0 && tokens % pos_rows == 0), "pos_rows must divide tokens");
  VS_CHECK(out_features % kBlk == 0 && in_features % kBlk == 0, "features must be multiples of 64");
  if (tokens == 0) return VS_OK;
  VS_CHECK(x && weight && y, "null pointer");
  hipLaunchKernelGGL(small_fwd_kernel, dim3((tokens + kRT - 1) / kRT, out_features / kRT), dim3(256), 0,
                     (hipStream_t)stream, (const bf16*)x, (const bf16*)pos, pos ? pos_rows : 1, (const bf16*)weight,
                     (const bf16*)bias, relu, (bf16*)y, tokens, out_features, in_features);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_small_linear_backward(int dtype, const void* grad_y, const void* x, const void* pos, int pos_rows,
                                        const void* weight, const void* relu_out, const void* grad_res,
                                        void* grad_x, void* grad_pos, int accumulate_pos, void* grad_w,
                                        void* grad_b, int tokens, int out_features, int in_features, void* stream) {
  VS_CHECK(dtype == VS_BF16, "the small-token Linear is the bf16 path");
  VS_CHECK(tokens >= 0 && out_features > 0 && in_features > 0, "bad sizes");
  VS_CHECK(!pos || (pos_rows > 0 && tokens % pos_rows == 0), "pos_rows must divide tokens");
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
  VS_CHECK(!grad_pos || grad_x, "grad_pos needs grad_x");
  const int nx = grad_x ? ((tokens + kRT - 1) / kRT) * (in_features / kRT) : 0;
  const int nw = grad_w ? (in_features / kBlk) * (out_features / kBlk) : 0;
  hipLaunchKernelGGL(small_bwd_kernel, dim3(nx + nw), dim3(256), 0, st, (const bf16*)grad_y, (const bf16*)x,
                     (const bf16*)pos, pos ? pos_rows : 1, (const bf16*)weight, (const bf16*)relu_out,
                     (bf16*)grad_x, (bf16*)grad_pos, (bf16*)grad_w, (bf16*)grad_b, tokens, out_features,
                     in_features, nx, (const bf16*)grad_res, accumulate_pos);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_self_attn_in_proj_forward(int dtype, const void* h, const void* pos, int pos_rows,
                                            const void* const* weights, const void* const* biases, void* const* outs,
                                            int tokens, int dim, void* stream) {
  VS_CHECK(dtype == VS_BF16, "the small-token Linear is the bf16 path");
  VS_CHECK(tokens >= 0 && dim > 0 && dim % kBlk == 0, "dim must be a positive multiple of 64");
  VS_CHECK(pos_rows > 0 && tokens % pos_rows == 0, "pos_rows must divide tokens");
  if (tokens == 0) return VS_OK;
  VS_CHECK(h && pos && weights && biases && outs, "null pointer");
  QkvPtrs p{};
  for (int g = 0; g < 3; ++g) {
    VS_CHECK(weights[g] && biases[g] && outs[g], "null pointer");
    p.w[g] = (const bf16*)weights[g];
    p.b[g] = (const bf16*)biases[g];
    p.y[g] = (bf16*)outs[g];
  }
  hipLaunchKernelGGL(qkv_fwd_kernel, dim3((tokens + kRT - 1) / kRT, 3 * dim / kRT), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)h, (const bf16*)pos, p, tokens, dim, pos_rows);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_self_attn_in_proj_backward(int dtype, const void* h, const void* pos, int pos_rows,
                                             const void* const* weights, const void* const* grad_outs,
                                             const void* grad_res, void* grad_h, void* grad_pos, int accumulate_pos,
                                             void* const* grad_weights, void* const* grad_biases, int tokens,
                                             int dim, void* stream) {
  VS_CHECK(dtype == VS_BF16, "the small-token Linear is the bf16 path");
  VS_CHECK(tokens >= 0 && dim > 0 && dim % kBlk == 0, "dim must be a positive multiple of 64");
  VS_CHECK(pos_rows > 0 && tokens % pos_rows == 0, "pos_rows must divide tokens");
  VS_CHECK(grad_h && grad_weights && grad_biases, "null pointer");
  hipStream_t st = (hipStream_t)stream;
  if (tokens == 0) {
    for (int g = 0; g < 3; ++g) {
      VS_CHECK(grad_weights[g] && grad_biases[g], "null pointer");
      VS_HIP(hipMemsetAsync(grad_weights[g], 0, (size_t)dim * dim * 2, st));
      VS_HIP(hipMemsetAsync(grad_biases[g], 0, (size_t)dim * 2, st));
    }
    return VS_OK;
  }
  VS_CHECK(h && pos && weights && grad_outs, "null pointer");
  QkvPtrs p{};
  for (int g = 0; g < 3; ++g) {
    VS_CHECK(weights[g] && grad_outs[g] && grad_weights[g] && grad_biases[g], "null pointer");
    p.w[g] = (const bf16*)weights[g];
    p.dy[g] = (const bf16*)grad_outs[g];
    p.dw[g] = (bf16*)grad_weights[g];
    p.db[g] = (bf16*)grad_biases[g];
  }
  const int nx = ((tokens + kRT - 1) / kRT) * (dim / kRT);
  const int nw = 3 * (dim / kBlk) * (dim / kBlk);
  hipLaunchKernelGGL(qkv_bwd_kernel, dim3(nx + nw), dim3(256), 0, st, (const bf16*)h, (const bf16*)pos, p,
                     (bf16*)grad_h, (bf16*)grad_pos, tokens, dim, nx, pos_rows, (const bf16*)grad_res,
                     accumulate_pos);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
