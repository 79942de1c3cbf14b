// Token-major LayerNorm (forward + backward) and column sums (Linear bias gradients).
//
// Swin and the pixel-decoder encoder normalise [M, C] activations with M = 16k..270k
// tokens and short rows (C = 96..768 for Swin-T).  PyTorch's kernels spend a workgroup
// per row and run these far below the HBM roofline (10.8 ms of LayerNorm per C2 step for
// < 1 GB of traffic).  Here a row belongs to a GROUP of G lanes (G = 4..64, a power of
// two) and each lane owns K 16-byte chunks of the row, so a wave normalises 64/G rows
// with 16-B loads/stores; statistics in f32 (two-pass in registers), one read and one
// write per element.  Semantics: torch.nn.functional.layer_norm (biased variance,
// y = (x - mean) * rsqrt(var + eps) * w + b).
//
// Backward: dx per row from the saved mean / rstd (xhat recomputed); dw / db are
// accumulated per lane in registers over a grid-stride sweep of rows, reduced across the
// workgroup's groups in LDS and written as one f32 partial row per workgroup, then
// summed over workgroups by `colsum_partials_kernel` (deterministic, no atomics).
//
// Column sum (bias gradient of a token-major Linear, sum over M of dY [M, N]): same
// partial-row scheme.
#include "common.h"
#include "mx_util.h"

#include <algorithm>
#include <cstdlib>

namespace vs {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxPartials = 512;    // workgroups of a backward / column-sum sweep

// lanes of one group: shuffle-reduce within G lanes (G a power of two, <= 64)
__device__ __forceinline__ float group_sum(float x, int G) {
  for (int s = G >> 1; s >= 1; s >>= 1) x += __shfl_xor(x, s, G);
  return x;
}

template <typename T>
__device__ __forceinline__ void load_chunk(const T* p, float* out) {
  Vec16<T>::load(p, out);
  if constexpr (Vec16<T>::N == 4) Vec16<T>::load(p + 4, out + 4);
}

template <typename T>
__device__ __forceinline__ void store_chunk(T* p, const float* v) {
  Vec16<T>::store(p, v);
  if constexpr (Vec16<T>::N == 4) Vec16<T>::store(p + 4, v + 4);
}

// A chunk as loaded (16 B of bf16 / 32 B of f32), unpacked to f32 only where it is used:
// a row's operands stay in flight in half the registers for bf16.
template <typename T> struct RawChunk;
template <> struct RawChunk<bf16> {
  uint4 a;
  __device__ __forceinline__ void load(const bf16* p) { a = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void zero() { a = make_uint4(0u, 0u, 0u, 0u); }
  __device__ __forceinline__ void unpack(float* out) const {
    const uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      out[2 * i] = __uint_as_float(w[i] << 16);
      out[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
};
template <> struct RawChunk<float> {
  float4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = *reinterpret_cast<const float4*>(p);
    b = *reinterpret_cast<const float4*>(p + 4);
  }
  __device__ __forceinline__ void zero() { a = b = make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ __forceinline__ void unpack(float* out) const {
    out[0] = a.x; out[1] = a.y; out[2] = a.z; out[3] = a.w;
    out[4] = b.x; out[5] = b.y; out[6] = b.z; out[7] = b.w;
  }
};

// chunk = 8 elements (one 16-B load for bf16, two for f32); C % 8 == 0
// RES: y = LN(s) with s = x + r rounded to T (the residual add of a pre-/post-norm block,
// written to s_out): one pass instead of an add kernel plus a LayerNorm.
// Q (bf16, C % 32 == 0): y also as MX fp8 -- e4m3 yq [rows, C] + e8m0 yqs [rows, C/32] at
// the same (window-layout) rows, the bytes vs_mx_quantize would make of y: the operand of
// the fp8 token GEMM that consumes y (config C5) without a quantisation pass.  A 32-element
// block is the 4 chunks of lanes 4t..4t+3 (G is a multiple of 4): amax by two exchanges.
// Q == 2 (bf16): y also as ROW-scaled e4m3 (yq [rows, C] + f32 scale [rows] in yqs, x ~= q
// * scale, the power-of-two rule of csrc/fp8_rows.hip): the operand of the vendor rowwise fp8
// GEMM (config C5's fp8 Linears); the row amax is a group max over the G lanes of the row.
template <typename T, int K, bool RES = false, int Q = 0>
__global__ void __launch_bounds__(kThreads) ln_fwd_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                          const T* __restrict__ b, T* __restrict__ y,
                                                          float* __restrict__ mean, float* __restrict__ rstd,
                                                          int M, int C, float eps, int G,
                                                          const T* __restrict__ r = nullptr,
                                                          T* __restrict__ s_out = nullptr,
                                                          const int* __restrict__ yrows = nullptr,
                                                          unsigned char* __restrict__ yq = nullptr,
                                                          unsigned char* __restrict__ yqs = nullptr) {
  const int nch = C >> 3;
  const int lane = threadIdx.x & (G - 1);
  const int rows_per_block = kThreads / G;
  const float invC = 1.f / (float)C;
  // weight / bias loaded once (they were a dependent round trip at every row's store), U
  // rows per iteration with every load (x, and r for the residual form) issued up front
  float wv[K][8], bv[K][8];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int j = lane + k * G;
#pragma unroll
    for (int i = 0; i < 8; ++i) wv[k][i] = bv[k][i] = 0.f;
    if (j < nch) {
      load_chunk(w + j * 8, wv[k]);
      load_chunk(b + j * 8, bv[k]);
    }
  }
  constexpr int U = K <= 2 ? 2 : 1;
  const long long stride = (long long)gridDim.x * rows_per_block;
  for (long long row0 = (long long)blockIdx.x * rows_per_block + threadIdx.x / G; row0 < M; row0 += U * stride) {
    RawChunk<T> xr[U][K], rr[RES ? U : 1][RES ? K : 1];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long row = row0 + u * stride;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int j = lane + k * G;
        if (row < M && j < nch) {
          xr[u][k].load(x + row * C + j * 8);
          if constexpr (RES) rr[u][k].load(r + row * C + j * 8);
        } else {
          xr[u][k].zero();
          if constexpr (RES) rr[u][k].zero();
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long row = row0 + u * stride;
      float v[K][8];
      float sm = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int j = lane + k * G;
        xr[u][k].unpack(v[k]);
        if constexpr (RES) {
          float rv[8];
          rr[u][k].unpack(rv);
#pragma unroll
          for (int i = 0; i < 8; ++i) v[k][i] = to_f32(from_f32<T>(v[k][i] + rv[i]));
          if (row < M && j < nch) store_chunk(s_out + row * C + j * 8, v[k]);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) sm += v[k][i];          // masked chunks are zero
      }
      const float mu = group_sum(sm, G) * invC;
      float q = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int j = lane + k * G;
        if (j < nch) {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float d = v[k][i] - mu;
            q += d * d;
          }
        }
      }
      const float rs = rsqrtf(group_sum(q, G) * invC + eps);
      if (Q == 2 && row < M) {                // row-scaled fp8 copy: all chunks, then one scale
        const long long yr = yrows ? (long long)yrows[row] : row;
        bf16x8_t c[K];
        unsigned am = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const int j = lane + k * G;
          c[k] = zero8();
          if (j < nch) {
            float o[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] = (v[k][i] - mu) * rs * wv[k][i] + bv[k][i];
            store_chunk(y + yr * C + j * 8, o);
#pragma unroll
            for (int i = 0; i < 8; ++i) c[k][i] = bf16_bits(o[i]);      // the stored bf16 values
            const unsigned m = amax8_bits(c[k]);
            am = m > am ? m : am;
          }
        }
        for (int sft = 1; sft < G; sft <<= 1) am = umax_xor(am, sft);
        const int kq = mx_exp_bits(am);
        const float inv = __uint_as_float((unsigned)(127 - kq) << 23);   // 2^-kq
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const int j = lane + k * G;
          if (j < nch) {
            const uint4 u = bits128(c[k]);
            *reinterpret_cast<uint2*>(yq + yr * C + j * 8) =
                make_uint2((unsigned)e4m3x4(u.x, u.y, inv), (unsigned)e4m3x4(u.z, u.w, inv));
          }
        }
        if (lane == 0) {
          reinterpret_cast<float*>(yqs)[yr] = inv;
          mean[row] = mu;
          rstd[row] = rs;
        }
      } else if (row < M) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const int j = lane + k * G;
          if (j < nch) {
            float o[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] = (v[k][i] - mu) * rs * wv[k][i] + bv[k][i];
            const long long yr = yrows ? (long long)yrows[row] : row;
            store_chunk(y + yr * C + j * 8, o);
            if constexpr (Q == 1) {
              bf16x8_t c;
#pragma unroll
              for (int i = 0; i < 8; ++i) c[i] = bf16_bits(o[i]);      // the stored bf16 values
              const unsigned am = umax_xor(umax_xor(amax8_bits(c), 1), 2);
              const int kq = mx_exp_bits(am);
              const float inv = __builtin_ldexpf(1.f, -kq);
              const uint4 u = bits128(c);
              *reinterpret_cast<uint2*>(yq + yr * C + j * 8) =
                  make_uint2((unsigned)e4m3x4(u.x, u.y, inv), (unsigned)e4m3x4(u.z, u.w, inv));
              if ((j & 3) == 0) yqs[yr * (C / 32) + (j >> 2)] = (unsigned char)(127 - kq);
            }
          }
        }
        if (lane == 0) {
          mean[row] = mu;
          rstd[row] = rs;
        }
      }
    }
  }
}

// dx, plus per-workgroup partial dw / db rows (f32) in part[blockIdx][NR][C]
// ADD: dx += dres (the gradient reaching the LayerNorm input through the residual path),
// accumulated in f32 and rounded once.
// CS: a third partial row, the column sums of dx as stored (rounded to T): the bias
// gradient of the Linear whose output fed the LayerNorm input (a Swin block's attention
// projection / MLP fc2, an encoder layer's output projection / fc2), so that Linear's
// backward reads no dY for it (visionseg.linear, ops.AddLayerNormFunction).
template <typename T, int K, bool ADD = false, bool CS = false>
__global__ void __launch_bounds__(kThreads) ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                          const T* __restrict__ w, const float* __restrict__ mean,
                                                          const float* __restrict__ rstd, T* __restrict__ dx,
                                                          float* __restrict__ part, int M, int C, int G,
                                                          const T* __restrict__ dres = nullptr,
                                                          const int* __restrict__ dyrows = nullptr) {
  extern __shared__ float red[];             // [4 waves][NR][C]
  constexpr int NR = CS ? 3 : 2;
  const int nch = C >> 3;
  const int lane = threadIdx.x & (G - 1);
  const int grp = threadIdx.x / G;
  const int rows_per_block = kThreads / G;
  const float invC = 1.f / (float)C;
  float dw[K][8], db[K][8], wv[K][8], ds[CS ? K : 1][8];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int j = lane + k * G;
#pragma unroll
    for (int i = 0; i < 8; ++i) dw[k][i] = db[k][i] = wv[k][i] = 0.f;   // masked chunks must hold 0, not garbage
    if constexpr (CS) {
#pragma unroll
      for (int i = 0; i < 8; ++i) ds[k][i] = 0.f;
    }
    if (j < nch) load_chunk(w + j * 8, wv[k]);
  }
  // U rows per iteration, every load of them (x, dy and the residual gradient) issued before
  // the math and held packed (memory-level parallelism: the residual gradient used to be a
  // second round trip, loaded only when its row was stored)
  constexpr int U = K <= 2 ? 2 : 1;
  const long long stride = (long long)gridDim.x * rows_per_block;
  for (long long row0 = (long long)blockIdx.x * rows_per_block + grp; row0 < M; row0 += U * stride) {
    RawChunk<T> xr[U][K], dr[U][K], rr[ADD ? U : 1][ADD ? K : 1];
    float mu[U], rs[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long row = row0 + u * stride;
      const bool ok = row < M;
      mu[u] = ok ? mean[row] : 0.f;
      rs[u] = ok ? rstd[row] : 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int j = lane + k * G;
        if (ok && j < nch) {
          xr[u][k].load(x + row * C + j * 8);
          dr[u][k].load(dy + (dyrows ? (long long)dyrows[row] : row) * C + j * 8);
          if constexpr (ADD) rr[u][k].load(dres + row * C + j * 8);
        } else {
          xr[u][k].zero();
          dr[u][k].zero();
          if constexpr (ADD) rr[u][k].zero();
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long row = row0 + u * stride;
      float xv[K][8], dv[K][8];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        xr[u][k].unpack(xv[k]);
        dr[u][k].unpack(dv[k]);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float xh = (xv[k][i] - mu[u]) * rs[u];   // masked chunks / rows have dv = 0: no effect
          const float g = dv[k][i] * wv[k][i];
          s1 += g;
          s2 += g * xh;
          dw[k][i] += dv[k][i] * xh;
          db[k][i] += dv[k][i];
          xv[k][i] = xh;                                  // keep xhat, reuse dv for g
          dv[k][i] = g;
        }
      }
      s1 = group_sum(s1, G) * invC;
      s2 = group_sum(s2, G) * invC;
      if (row < M) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const int j = lane + k * G;
          if (j < nch) {
            float o[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] = rs[u] * (dv[k][i] - s1 - xv[k][i] * s2);
            if constexpr (ADD) {
              float rv[8];
              rr[u][k].unpack(rv);
#pragma unroll
              for (int i = 0; i < 8; ++i) o[i] += rv[i];
            }
            store_chunk(dx + row * C + j * 8, o);
            if constexpr (CS) {
#pragma unroll
              for (int i = 0; i < 8; ++i) ds[k][i] += to_f32(from_f32<T>(o[i]));
            }
          }
        }
      }
    }
  }
  // reduce the wave's groups with shuffles (lanes holding the same chunks), then the 4
  // waves in LDS -> one partial row pair per workgroup
  for (int o = G; o < 64; o <<= 1) {
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        dw[k][i] += __shfl_xor(dw[k][i], o, 64);
        db[k][i] += __shfl_xor(db[k][i], o, 64);
        if constexpr (CS) ds[k][i] += __shfl_xor(ds[k][i], o, 64);
      }
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) < G) {
    float* mine = red + (size_t)wave * NR * C;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int j = lane + k * G;
      if (j < nch) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          mine[j * 8 + i] = dw[k][i];
          mine[C + j * 8 + i] = db[k][i];
          if constexpr (CS) mine[2 * C + j * 8 + i] = ds[k][i];
        }
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < NR * C; c += kThreads) {
    const float acc = (red[c] + red[NR * C + c]) + (red[2 * NR * C + c] + red[3 * NR * C + c]);
    part[(size_t)blockIdx.x * NR * C + c] = acc;
  }
}

// column sums of x [M, N] -> part[blockIdx][N] (f32); a thread owns one 8-column chunk
// and a subset of rows
// Row segments of a [B, S, N] tensor (the levels of a multi-scale token sequence):
// segment k = rows [start[k], start[k + 1]) of every image.
struct RowSegments {
  int start[9];
  int nseg;
};

template <typename T>
__device__ __forceinline__ void colsum_rows(const T* __restrict__ x, float* __restrict__ part, long long M, int N,
                                            int nblk, int blk, float* red, int c0, int Nb);

// Column blocks: a workgroup covers at most kColBlock columns (one 8-column chunk per
// thread); wider rows (Swin-L MLP hidden: 3072, 6144) take grid.y = ceil(N / kColBlock).
constexpr int kColBlock = 8 * kThreads;

template <typename T>
__global__ void __launch_bounds__(kThreads) colsum_kernel(const T* __restrict__ x, float* __restrict__ part, int M,
                                                          int N) {
  extern __shared__ float red[];
  const int c0 = blockIdx.y * kColBlock;
  colsum_rows(x, part + (size_t)blockIdx.x * N, M, N, gridDim.x, blockIdx.x, red, c0, min(kColBlock, N - c0));
}

// per-segment column sums of x [B, S, N]: grid (nblk, nseg * B); workgroup (x, k*B + b)
// sums its share of image b's rows of segment k -> part[(k*B + b)*nblk + x][N]
template <typename T>
__global__ void __launch_bounds__(kThreads) colsum_seg_kernel(const T* __restrict__ x, float* __restrict__ part,
                                                              int B, int S, int N, RowSegments seg) {
  extern __shared__ float red[];
  const int k = blockIdx.y / B, b = blockIdx.y % B;
  const int r0 = seg.start[k];
  colsum_rows(x + ((size_t)b * S + r0) * N, part + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * N,
              seg.start[k + 1] - r0, N, gridDim.x, blockIdx.x, red, 0, N);
}

// column sums of rows [0, M) of x [M, N], columns [c0, c0 + Nb) -> part[c0 ..] (f32) for
// workgroup blk of nblk; a thread owns one 8-column chunk and a subset of rows
template <typename T>
__device__ __forceinline__ void colsum_rows(const T* __restrict__ x, float* __restrict__ part, long long M, int N,
                                            int nblk, int blk, float* red, int c0, int Nb) {   // red: [rowsets][Nb]
  x += c0;
  part += c0;
  const int nch = Nb >> 3;
  const int rowsets = kThreads / nch;        // nch <= 256
  const int ch = threadIdx.x % nch;
  const int rs = threadIdx.x / nch;
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
  if (rs < rowsets) {
    const long long stride = (long long)nblk * rowsets;
    for (long long row = (long long)blk * rowsets + rs; row < M; row += 4 * stride) {
      float v[4][8];                            // 4 rows' loads in flight
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (row + u * stride < M) {
          load_chunk(x + (row + u * stride) * N + ch * 8, v[u]);
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) v[u][i] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += v[u][i];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) red[(size_t)rs * Nb + ch * 8 + i] = acc[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < Nb; c += kThreads) {
    float a = 0.f;
    for (int r = 0; r < rowsets; ++r) a += red[(size_t)r * Nb + c];
    part[c] = a;
  }
}

// Activation backward fused with the column sums of its output (the bias gradient of the
// Linear that produced the activation's input: fc1 of a Swin MLP (GELU) or of an encoder
// FFN (ReLU)): dx = dy * act'(x), stored, and per-workgroup partial column sums of dx as
// stored -> part[blockIdx][N]; same thread layout as colsum_kernel (a thread owns one
// 8-column chunk, rows strided).  GELU is torch's exact form: 0.5 x (1 + erf(x / sqrt2)),
// derivative 0.5 (1 + erf(x / sqrt2)) + x exp(-x^2 / 2) / sqrt(2 pi).
template <typename T, int ACT>   // ACT 0: ReLU, 1: GELU (erf)
__global__ void __launch_bounds__(kThreads) act_bwd_colsum_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                                  T* __restrict__ dx, float* __restrict__ part, int M,
                                                                  int N) {
  extern __shared__ float red[];             // [rowsets][Nb]
  const int c0 = blockIdx.y * kColBlock, Nb = min(kColBlock, N - c0);   // this workgroup's columns
  dy += c0;
  x += c0;
  dx += c0;
  part += c0;
  const int nch = Nb >> 3;
  const int rowsets = kThreads / nch;
  const int ch = threadIdx.x % nch;
  const int rs = threadIdx.x / nch;
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
  if (rs < rowsets) {
    const long long stride = (long long)gridDim.x * rowsets;
    for (long long row = (long long)blockIdx.x * rowsets + rs; row < M; row += 2 * stride) {
      float g[2][8], v[2][8];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const long long rr = row + u * stride;
        if (rr < M) {
          load_chunk(dy + rr * N + ch * 8, g[u]);
          load_chunk(x + rr * N + ch * 8, v[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const long long rr = row + u * stride;
        if (rr < M) {
          float o[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float xv = v[u][i];
            float d;
            if (ACT == 0) {
              d = xv > 0.f ? 1.f : 0.f;
            } else {
              // (common.h: one exp + one reciprocal per element instead of erff's branches +
              // an exp -- the kernel was VALU-bound at GELU, 4.5 vs 5.9 TB/s at ReLU)
              d = gelu_grad_erf(xv);
            }
            o[i] = g[u][i] * d;
          }
          store_chunk(dx + rr * N + ch * 8, o);
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[i] += to_f32(from_f32<T>(o[i]));
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) red[(size_t)rs * Nb + ch * 8 + i] = acc[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < Nb; c += kThreads) {
    float a = 0.f;
    for (int r = 0; r < rowsets; ++r) a += red[(size_t)r * Nb + c];
    part[(size_t)blockIdx.x * N + c] = a;
  }
}

// out[c] = sum_b part[b][c] (b < nb) in a fixed order; columns [0, split) go to out0,
// [split, split2) to out1, [split2, N) to out2.  A block = 32 columns x 32 row slices (1024
// threads), 4 independent accumulators per thread, slices combined in LDS: 512 partial rows
// are one batch of 16 loads per thread.  (32 x 8 slices took four dependent batches: ~4.9
// us per launch, 90 launches per C2 step, for < 2 MB read.)
constexpr int kCsThreads = 1024, kCsSlices = kCsThreads / 32;
template <typename T>
__global__ void __launch_bounds__(kCsThreads) colsum_partials_kernel(const float* __restrict__ part, T* __restrict__ out0,
                                                                     T* __restrict__ out1, int nb, int N, int split,
                                                                     T* __restrict__ out2 = nullptr, int split2 = 1 << 30) {
  constexpr int S = kCsSlices;
  __shared__ float red[S][33];
  const int lane = threadIdx.x & 31;
  const int sl = threadIdx.x >> 5;
  const int col = blockIdx.x * 32 + lane;
  part += (size_t)blockIdx.y * nb * N;         // grid.y > 1: one output row per segment
  out0 += (size_t)blockIdx.y * N;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (col < N) {
    int r = sl;
#pragma unroll 4
    for (; r + 3 * S < nb; r += 4 * S) {
      a0 += part[(size_t)r * N + col];
      a1 += part[(size_t)(r + S) * N + col];
      a2 += part[(size_t)(r + 2 * S) * N + col];
      a3 += part[(size_t)(r + 3 * S) * N + col];
    }
    for (; r < nb; r += S) a0 += part[(size_t)r * N + col];
  }
  red[sl][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (sl == 0 && col < N) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < S; ++i) t += red[i][lane];
    if (col < split) out0[col] = from_f32<T>(t);
    else if (col < split2) out1[col - split] = from_f32<T>(t);
    else out2[col - split2] = from_f32<T>(t);
  }
}

// Relative-position-table gradient from per-window partials: the partial rows [P, H*T]
// were column-summed as [P/F, F*H*T] (F folds rows so the width is a multiple of 8: H*T is
// odd * heads for the (2ws-1)^2 tables) into part[nb][F*H*T]; out[t][h] = sum over b, f of
// part[b][f*H*T + h*T + t] in a fixed order, written transposed ([T, H]: the table's own
// layout) in the table's dtype.  Same block shape as colsum_partials_kernel.
template <typename T>
__global__ void __launch_bounds__(kCsThreads) table_fold_kernel(const float* __restrict__ part, T* __restrict__ out,
                                                                int nb, int F, int H, int TT) {
  constexpr int S = kCsSlices;
  __shared__ float red[S][33];
  const int lane = threadIdx.x & 31;
  const int sl = threadIdx.x >> 5;
  const int R = H * TT, W = F * R;
  const int col = blockIdx.x * 32 + lane;      // h * TT + t
  float a0 = 0.f, a1 = 0.f;
  if (col < R) {
    for (int r = sl; r < nb; r += S)
      for (int f = 0; f < F; ++f) {
        if (f & 1) a1 += part[(size_t)r * W + f * R + col];
        else a0 += part[(size_t)r * W + f * R + col];
      }
  }
  red[sl][lane] = a0 + a1;
  __syncthreads();
  if (sl == 0 && col < R) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < S; ++i) t += red[i][lane];
    const int h = col / TT, tt = col - h * TT;
    out[(size_t)tt * H + h] = from_f32<T>(t);
  }
}

// split-K epilogue: out[i] = sum_{s < S} part[s][i] (+ extra[i]), f32 accumulation in a
// fixed order, written in the output dtype; 4 elements per thread (float4), 4 partial
// rows in flight
template <typename T>
__global__ void __launch_bounds__(kThreads) splitk_sum_kernel(const float* __restrict__ part,
                                                              const float* __restrict__ extra, T* __restrict__ out,
                                                              int S, long long n4) {
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (long long)gridDim.x * kThreads) {
    float4 a = extra ? reinterpret_cast<const float4*>(extra)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 b = make_float4(0.f, 0.f, 0.f, 0.f), c = b, d = b;
    const float4* p = reinterpret_cast<const float4*>(part) + i;
    int s = 0;
    for (; s + 3 < S; s += 4) {
      const float4 v0 = p[(size_t)s * n4], v1 = p[(size_t)(s + 1) * n4], v2 = p[(size_t)(s + 2) * n4],
                   v3 = p[(size_t)(s + 3) * n4];
      a.x += v0.x; a.y += v0.y; a.z += v0.z; a.w += v0.w;
      b.x += v1.x; b.y += v1.y; b.z += v1.z; b.w += v1.w;
      c.x += v2.x; c.y += v2.y; c.z += v2.z; c.w += v2.w;
      d.x += v3.x; d.y += v3.y; d.z += v3.z; d.w += v3.w;
    }
    for (; s < S; ++s) {
      const float4 v = p[(size_t)s * n4];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    const float r[4] = {(a.x + b.x) + (c.x + d.x), (a.y + b.y) + (c.y + d.y), (a.z + b.z) + (c.z + d.z),
                        (a.w + b.w) + (c.w + d.w)};
    T* o = out + i * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = from_f32<T>(r[k]);
  }
}

// Many partials (S >= 16, the split-K weight gradients of the token-heavy Linears: up to
// 256 chunks): the S loop is the latency.  A workgroup takes 256 / PH element quads and
// PH phases; phase p sums partials p, p + PH, ... (two rows in flight), and the phases
// are combined in LDS in phase order (fixed order: deterministic).  PH = 8 gives 8x the
// workgroups of splitk_sum_kernel for the same output.
template <typename T, int PH>
__global__ void __launch_bounds__(kThreads) splitk_sum_phased_kernel(const float* __restrict__ part,
                                                                     const float* __restrict__ extra,
                                                                     T* __restrict__ out, int S, long long n4) {
  constexpr int QPB = kThreads / PH;         // element quads per workgroup
  __shared__ float4 red[PH][QPB];
  const int qi = threadIdx.x % QPB, ph = threadIdx.x / QPB;
  const long long i = (long long)blockIdx.x * QPB + qi;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
  if (i < n4) {
    const float4* p = reinterpret_cast<const float4*>(part) + i;
    int s = ph;
    for (; s + PH < S; s += 2 * PH) {
      const float4 v0 = p[(size_t)s * n4], v1 = p[(size_t)(s + PH) * n4];
      a.x += v0.x; a.y += v0.y; a.z += v0.z; a.w += v0.w;
      b.x += v1.x; b.y += v1.y; b.z += v1.z; b.w += v1.w;
    }
    if (s < S) {
      const float4 v = p[(size_t)s * n4];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  red[ph][qi] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  __syncthreads();
  if (ph == 0 && i < n4) {
    float4 r = extra ? reinterpret_cast<const float4*>(extra)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < PH; ++k) {
      const float4 v = red[k][qi];
      r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
    }
    T* o = out + i * 4;
    o[0] = from_f32<T>(r.x);
    o[1] = from_f32<T>(r.y);
    o[2] = from_f32<T>(r.z);
    o[3] = from_f32<T>(r.w);
  }
}

// pick (G, K): a power-of-two group of G <= 16 lanes (else <= 64) with K chunks per lane,
// fewest idle chunk slots G*K - nch first, then the smaller K (registers).  C = 96
// (nch 12): G = 4, K = 3 -- no idle lanes -- where the smallest-K rule gave G = 16, K = 1
// with a quarter of the lanes idle (Swin-T stage 1, the largest LayerNorm of the step).
bool pick_gk(int nch, int kmax, int* G, int* K) {
  for (int lim : {16, 64}) {
    int best_g = 0, best_k = 0, best_w = 1 << 30;
    for (int k = 1; k <= kmax && k <= 4; ++k) {
      int g = 4;
      while (g * k < nch) g <<= 1;
      if (g > lim) continue;
      const int w = g * k - nch;
      if (w < best_w) {
        best_w = w;
        best_g = g;
        best_k = k;
      }
    }
    if (best_g) {
      *G = best_g;
      *K = best_k;
      return true;
    }
  }
  return false;
}

int blocks_for(long long M, int rows_per_block, int cap) {
  long long nb = (M + rows_per_block - 1) / rows_per_block;
  return (int)std::max<long long>(1, std::min<long long>(nb, cap));
}

}  // namespace
}  // namespace vs

using namespace vs;

#define VS_LN_K(KK, ...)           \
  switch (KK) {                    \
    case 1: __VA_ARGS__(1); break; \
    case 2: __VA_ARGS__(2); break; \
    case 3: __VA_ARGS__(3); break; \
    default: __VA_ARGS__(4); break; \
  }

// at most 4 chunks of 8 per lane (register budget of the backward): C <= 64 * 32 = 2048
static int ln_kmax(int) { return 4; }

static int layer_norm_forward_impl(int dtype, const void* x, const void* w, const void* b, void* y, float* mean,
                                   float* rstd, int M, int C, float eps, const int* yrows, void* stream,
                                   void* q = nullptr, void* qs = nullptr, int qmode = 0);

extern "C" int vs_layer_norm_forward(int dtype, const void* x, const void* w, const void* b, void* y, float* mean,
                                     float* rstd, int M, int C, float eps, void* stream) {
  return layer_norm_forward_impl(dtype, x, w, b, y, mean, rstd, M, C, eps, nullptr, stream);
}

extern "C" int vs_layer_norm_forward_rows(int dtype, const void* x, const void* w, const void* b, void* y,
                                          float* mean, float* rstd, int M, int C, float eps, const int* y_rows,
                                          void* stream) {
  VS_CHECK(M == 0 || y_rows, "null pointer");
  return layer_norm_forward_impl(dtype, x, w, b, y, mean, rstd, M, C, eps, y_rows, stream);
}

extern "C" int vs_layer_norm_forward_rows_q(const void* x, const void* w, const void* b, void* y, void* y_q,
                                            void* y_qscales, float* mean, float* rstd, int M, int C, float eps,
                                            const int* y_rows, void* stream) {
  VS_CHECK(M == 0 || (y_rows && y_q && y_qscales), "null pointer");
  VS_CHECK(C % 32 == 0, "C must be a multiple of 32 for the MX fp8 copy");
  return layer_norm_forward_impl(VS_BF16, x, w, b, y, mean, rstd, M, C, eps, y_rows, stream, y_q, y_qscales, 1);
}

extern "C" int vs_layer_norm_forward_qr(const void* x, const void* w, const void* b, void* y, void* y_q,
                                        float* y_scale, float* mean, float* rstd, int M, int C, float eps,
                                        const int* y_rows, void* stream) {
  VS_CHECK(M == 0 || (y_q && y_scale), "null pointer");
  return layer_norm_forward_impl(VS_BF16, x, w, b, y, mean, rstd, M, C, eps, y_rows, stream, y_q, y_scale, 2);
}

static int layer_norm_forward_impl(int dtype, const void* x, const void* w, const void* b, void* y, float* mean,
                                   float* rstd, int M, int C, float eps, const int* yrows, void* stream, void* q,
                                   void* qs, int qmode) {
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");
  VS_CHECK(M >= 0 && C > 0 && C % 8 == 0, "C must be a positive multiple of 8");
  VS_CHECK(w && b && (M == 0 || (x && y && mean && rstd)), "null pointer");
  int G, K;
  VS_CHECK(pick_gk(C / 8, ln_kmax(dtype), &G, &K), "row too long for the LayerNorm kernel (C <= 2048)");
  if (M == 0) return VS_OK;
  hipStream_t st = (hipStream_t)stream;
  const int grid = blocks_for(M, kThreads / G, 256 * 32);
#define VS_LNF(KK)                                                                                          \
  if (q && qmode == 2)                                                                                      \
    hipLaunchKernelGGL((ln_fwd_kernel<bf16, KK, false, 2>), dim3(grid), dim3(kThreads), 0, st,              \
                       (const bf16*)x, (const bf16*)w, (const bf16*)b, (bf16*)y, mean, rstd, M, C, eps, G,  \
                       nullptr, nullptr, yrows, (unsigned char*)q, (unsigned char*)qs);                     \
  else if (q)                                                                                               \
    hipLaunchKernelGGL((ln_fwd_kernel<bf16, KK, false, 1>), dim3(grid), dim3(kThreads), 0, st,              \
                       (const bf16*)x, (const bf16*)w, (const bf16*)b, (bf16*)y, mean, rstd, M, C, eps, G,  \
                       nullptr, nullptr, yrows, (unsigned char*)q, (unsigned char*)qs);                     \
  else if (dtype == VS_BF16)                                                                                \
    hipLaunchKernelGGL((ln_fwd_kernel<bf16, KK>), dim3(grid), dim3(kThreads), 0, st, (const bf16*)x,        \
                       (const bf16*)w, (const bf16*)b, (bf16*)y, mean, rstd, M, C, eps, G, nullptr, nullptr, \
                       yrows);                                                                              \
  else                                                                                                      \
    hipLaunchKernelGGL((ln_fwd_kernel<float, KK>), dim3(grid), dim3(kThreads), 0, st, (const float*)x,      \
                       (const float*)w, (const float*)b, (float*)y, mean, rstd, M, C, eps, G, nullptr,      \
                       nullptr, yrows)
  VS_LN_K(K, VS_LNF)
#undef VS_LNF
  VS_LAUNCH_CHECK();
  return VS_OK;
}

static int add_layer_norm_forward_impl(int dtype, const void* x, const void* r, const void* w, const void* b,
                                       void* s, void* y, float* mean, float* rstd, int M, int C, float eps,
                                       const int* yrows, void* stream, void* q = nullptr, void* qs = nullptr,
                                       int qmode = 0);

extern "C" int vs_add_layer_norm_forward(int dtype, const void* x, const void* r, const void* w, const void* b,
                                         void* s, void* y, float* mean, float* rstd, int M, int C, float eps,
                                         void* stream) {
  return add_layer_norm_forward_impl(dtype, x, r, w, b, s, y, mean, rstd, M, C, eps, nullptr, stream);
}

extern "C" int vs_add_layer_norm_forward_rows(int dtype, const void* x, const void* r, const void* w, const void* b,
                                              void* s, void* y, float* mean, float* rstd, int M, int C, float eps,
                                              const int* y_rows, void* stream) {
  VS_CHECK(M == 0 || y_rows, "null pointer");
  return add_layer_norm_forward_impl(dtype, x, r, w, b, s, y, mean, rstd, M, C, eps, y_rows, stream);
}

extern "C" int vs_add_layer_norm_forward_q(const void* x, const void* r, const void* w, const void* b, void* s,
                                           void* y, void* y_q, void* y_qscales, float* mean, float* rstd, int M,
                                           int C, float eps, const int* y_rows, void* stream) {
  VS_CHECK(M == 0 || (y_q && y_qscales), "null pointer");
  VS_CHECK(C % 32 == 0, "C must be a multiple of 32 for the MX fp8 copy");
  return add_layer_norm_forward_impl(VS_BF16, x, r, w, b, s, y, mean, rstd, M, C, eps, y_rows, stream, y_q,
                                     y_qscales, 1);
}

extern "C" int vs_add_layer_norm_forward_qr(const void* x, const void* r, const void* w, const void* b, void* s,
                                            void* y, void* y_q, float* y_scale, float* mean, float* rstd, int M,
                                            int C, float eps, const int* y_rows, void* stream) {
  VS_CHECK(M == 0 || (y_q && y_scale), "null pointer");
  return add_layer_norm_forward_impl(VS_BF16, x, r, w, b, s, y, mean, rstd, M, C, eps, y_rows, stream, y_q,
                                     y_scale, 2);
}

static int add_layer_norm_forward_impl(int dtype, const void* x, const void* r, const void* w, const void* b,
                                       void* s, void* y, float* mean, float* rstd, int M, int C, float eps,
                                       const int* yrows, void* stream, void* q, void* qs, int qmode) {
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");
  VS_CHECK(M >= 0 && C > 0 && C % 8 == 0, "C must be a positive multiple of 8");
  VS_CHECK(w && b && (M == 0 || (x && r && s && y && mean && rstd)), "null pointer");
  int G, K;
  VS_CHECK(pick_gk(C / 8, ln_kmax(dtype), &G, &K), "row too long for the LayerNorm kernel (C <= 2048)");
  if (M == 0) return VS_OK;
  hipStream_t st = (hipStream_t)stream;
  const int grid = blocks_for(M, kThreads / G, 256 * 32);
#define VS_ALNF(KK)                                                                                           \
  if (q && qmode == 2)                                                                                        \
    hipLaunchKernelGGL((ln_fwd_kernel<bf16, KK, true, 2>), dim3(grid), dim3(kThreads), 0, st,                 \
                       (const bf16*)x, (const bf16*)w, (const bf16*)b, (bf16*)y, mean, rstd, M, C, eps, G,    \
                       (const bf16*)r, (bf16*)s, yrows, (unsigned char*)q, (unsigned char*)qs);               \
  else if (q)                                                                                                 \
    hipLaunchKernelGGL((ln_fwd_kernel<bf16, KK, true, 1>), dim3(grid), dim3(kThreads), 0, st,                 \
                       (const bf16*)x, (const bf16*)w, (const bf16*)b, (bf16*)y, mean, rstd, M, C, eps, G,    \
                       (const bf16*)r, (bf16*)s, yrows, (unsigned char*)q, (unsigned char*)qs);               \
  else if (dtype == VS_BF16)                                                                                  \
    hipLaunchKernelGGL((ln_fwd_kernel<bf16, KK, true>), dim3(grid), dim3(kThreads), 0, st, (const bf16*)x,    \
                       (const bf16*)w, (const bf16*)b, (bf16*)y, mean, rstd, M, C, eps, G, (const bf16*)r,    \
                       (bf16*)s, yrows);                                                                      \
  else                                                                                                        \
    hipLaunchKernelGGL((ln_fwd_kernel<float, KK, true>), dim3(grid), dim3(kThreads), 0, st, (const float*)x,  \
                       (const float*)w, (const float*)b, (float*)y, mean, rstd, M, C, eps, G, (const float*)r, \
                       (float*)s, yrows)
  VS_LN_K(K, VS_ALNF)
#undef VS_ALNF
  VS_LAUNCH_CHECK();
  return VS_OK;
}

// workgroups of the LayerNorm backward sweep (512 vs 256 / 1024 at the C2 shapes:
// profiles/r6_ln_bwd_ab.txt)
constexpr int kMaxPartialsLN = 512;
static int ln_bwd_parts() { return kMaxPartialsLN; }

extern "C" long long vs_layer_norm_backward_workspace_bytes(int M, int C) {
  return (long long)kMaxPartialsLN * 3 * C * sizeof(float);   // dw, db (+ dx column sums)
}

static int layer_norm_backward_impl(int dtype, const void* dy, const void* x, const void* w, const float* mean,
                                    const float* rstd, const void* dres, void* dx, void* dw, void* db, void* dsum,
                                    void* ws, int M, int C, void* stream, const int* dyrows = nullptr);

extern "C" int vs_layer_norm_backward(int dtype, const void* dy, const void* x, const void* w, const float* mean,
                                      const float* rstd, void* dx, void* dw, void* db, void* ws, int M, int C,
                                      void* stream) {
  return layer_norm_backward_impl(dtype, dy, x, w, mean, rstd, nullptr, dx, dw, db, nullptr, ws, M, C, stream);
}

extern "C" int vs_layer_norm_backward_add(int dtype, const void* dy, const void* x, const void* w, const float* mean,
                                          const float* rstd, const void* dres, void* dx, void* dw, void* db, void* ws,
                                          int M, int C, void* stream) {
  VS_CHECK(M == 0 || dres, "null pointer");
  return layer_norm_backward_impl(dtype, dy, x, w, mean, rstd, dres, dx, dw, db, nullptr, ws, M, C, stream);
}

extern "C" int vs_layer_norm_backward_ex(int dtype, const void* dy, const void* x, const void* w, const float* mean,
                                         const float* rstd, const void* dres, void* dx, void* dw, void* db,
                                         void* dx_colsum, void* ws, int M, int C, void* stream) {
  return layer_norm_backward_impl(dtype, dy, x, w, mean, rstd, dres, dx, dw, db, dx_colsum, ws, M, C, stream);
}

extern "C" int vs_layer_norm_backward_rows(int dtype, const void* dy, const void* x, const void* w, const float* mean,
                                           const float* rstd, const void* dres, void* dx, void* dw, void* db,
                                           void* dx_colsum, void* ws, int M, int C, const int* dy_rows,
                                           void* stream) {
  VS_CHECK(M == 0 || dy_rows, "null pointer");
  return layer_norm_backward_impl(dtype, dy, x, w, mean, rstd, dres, dx, dw, db, dx_colsum, ws, M, C, stream,
                                  dy_rows);
}

static int layer_norm_backward_impl(int dtype, const void* dy, const void* x, const void* w, const float* mean,
                                    const float* rstd, const void* dres, void* dx, void* dw, void* db, void* dsum,
                                    void* ws, int M, int C, void* stream, const int* dyrows) {
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");
  VS_CHECK(M >= 0 && C > 0 && C % 8 == 0, "C must be a positive multiple of 8");
  VS_CHECK(w && dw && db && ws && (M == 0 || (dy && x && mean && rstd && dx)), "null pointer");
  int G, K;
  VS_CHECK(pick_gk(C / 8, ln_kmax(dtype), &G, &K), "row too long for the LayerNorm kernel (C <= 2048)");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  const int grid = blocks_for(M, kThreads / G, ln_bwd_parts());
  const int NR = dsum ? 3 : 2;
  const size_t lds = (size_t)(kThreads / 64) * NR * C * sizeof(float);
  VS_CHECK(lds <= 64 * 1024, "LayerNorm backward LDS budget exceeded");
#define VS_LNB_T(TT, KK, AD, CS_)                                                                            \
  hipLaunchKernelGGL((ln_bwd_kernel<TT, KK, AD, CS_>), dim3(grid), dim3(kThreads), lds, st, (const TT*)dy,    \
                     (const TT*)x, (const TT*)w, mean, rstd, (TT*)dx, part, M, C, G, (const TT*)dres, dyrows)
#define VS_LNB_D(TT, KK)                                        \
  if (dres && dsum) {                                            \
    VS_LNB_T(TT, KK, true, true);                               \
  } else if (dres) {                                            \
    VS_LNB_T(TT, KK, true, false);                              \
  } else if (dsum) {                                            \
    VS_LNB_T(TT, KK, false, true);                              \
  } else {                                                      \
    VS_LNB_T(TT, KK, false, false);                             \
  }
#define VS_LNB(KK)                   \
  if (dtype == VS_BF16) {            \
    VS_LNB_D(bf16, KK);              \
  } else {                           \
    VS_LNB_D(float, KK);             \
  }
  VS_LN_K(K, VS_LNB)
#undef VS_LNB
#undef VS_LNB_D
#undef VS_LNB_T
  // dw / db (/ dx column sums) = column sums of the partial rows' thirds
  const int rgrid = (NR * C + 31) / 32;
  if (dtype == VS_BF16)
    hipLaunchKernelGGL(colsum_partials_kernel<bf16>, dim3(rgrid), dim3(kCsThreads), 0, st, part, (bf16*)dw, (bf16*)db,
                       grid, NR * C, C, (bf16*)dsum, 2 * C);
  else
    hipLaunchKernelGGL(colsum_partials_kernel<float>, dim3(rgrid), dim3(kCsThreads), 0, st, part, (float*)dw,
                       (float*)db, grid, NR * C, C, (float*)dsum, 2 * C);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" long long vs_column_sum_workspace_bytes(int M, int N) {
  return (long long)kMaxPartials * N * sizeof(float);
}

extern "C" int vs_column_sum(int dtype, const void* x, void* out, void* ws, int M, int N, void* stream) {
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");
  VS_CHECK(M >= 0 && N > 0 && N % 8 == 0 && N <= 8 * kColBlock, "N must be a multiple of 8, <= 16384");
  VS_CHECK(out && ws && (M == 0 || x), "null pointer");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  const int Nb = std::min(N, kColBlock), rowsets = kThreads / (Nb / 8);
  const int grid = blocks_for(M, rowsets * 16, kMaxPartials);
  const dim3 g2(grid, (N + kColBlock - 1) / kColBlock);
  const size_t lds = (size_t)rowsets * Nb * sizeof(float);   // >= every column block's rowsets x Nb
  if (dtype == VS_BF16) {
    hipLaunchKernelGGL(colsum_kernel<bf16>, g2, dim3(kThreads), lds, st, (const bf16*)x, part, M, N);
    hipLaunchKernelGGL(colsum_partials_kernel<bf16>, dim3((N + 31) / 32), dim3(kCsThreads), 0, st, part, (bf16*)out,
                       (bf16*)nullptr, grid, N, N);
  } else {
    hipLaunchKernelGGL(colsum_kernel<float>, g2, dim3(kThreads), lds, st, (const float*)x, part, M, N);
    hipLaunchKernelGGL(colsum_partials_kernel<float>, dim3((N + 31) / 32), dim3(kCsThreads), 0, st, part,
                       (float*)out, (float*)nullptr, grid, N, N);
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}

static int table_fold_factor(int R) {
  for (int f : {1, 2, 4, 8})
    if ((f * R) % 8 == 0) return f;
  return 8;
}

extern "C" long long vs_rel_table_grad_workspace_bytes(int P, int heads, int T) {
  const long long W = (long long)table_fold_factor(heads * T) * heads * T;
  return (long long)kMaxPartials * W * sizeof(float);
}

extern "C" int vs_rel_table_grad(int dtype, const float* part, void* out, void* ws, int P, int heads, int T,
                                 void* stream) {
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");
  VS_CHECK(P > 0 && heads > 0 && T > 0, "empty partials");
  VS_CHECK(part && out && ws, "null pointer");
  const int R = heads * T, F = table_fold_factor(R), W = F * R;
  VS_CHECK(P % F == 0, "the partial rows must fold into a multiple-of-8 width (P % F == 0)");
  VS_CHECK(W <= 8 * kColBlock, "table too large");
  hipStream_t st = (hipStream_t)stream;
  float* p2 = (float*)ws;
  const int M = P / F;
  const int Nb = std::min(W, kColBlock), rowsets = kThreads / (Nb / 8);
  const int grid = blocks_for(M, rowsets * 16, kMaxPartials);
  const dim3 g2(grid, (W + kColBlock - 1) / kColBlock);
  const size_t lds = (size_t)rowsets * Nb * sizeof(float);
  hipLaunchKernelGGL(colsum_kernel<float>, g2, dim3(kThreads), lds, st, part, p2, M, W);
  if (dtype == VS_BF16)
    hipLaunchKernelGGL(table_fold_kernel<bf16>, dim3((R + 31) / 32), dim3(kCsThreads), 0, st, p2, (bf16*)out, grid, F,
                       heads, T);
  else
    hipLaunchKernelGGL(table_fold_kernel<float>, dim3((R + 31) / 32), dim3(kCsThreads), 0, st, p2, (float*)out, grid,
                       F, heads, T);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" long long vs_column_sum_segments_workspace_bytes(int B, int N, int nseg) {
  return (long long)std::max(kMaxPartials, nseg * std::max(B, 1)) * N * sizeof(float);
}

extern "C" int vs_column_sum_segments(int dtype, const void* x, float* out, void* ws, int B, int S, int N,
                                      const int* seg_start, int nseg, void* stream) {
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");
  VS_CHECK(B >= 0 && S >= 0 && N > 0 && N % 8 == 0 && N / 8 <= kThreads, "N must be a multiple of 8, <= 2048");
  VS_CHECK(nseg >= 1 && nseg <= 8 && seg_start, "1..8 segments");
  VS_CHECK(out && ws && (B * (long long)S == 0 || x), "null pointer");
  RowSegments seg{};
  seg.nseg = nseg;
  for (int k = 0; k <= nseg; ++k) {
    seg.start[k] = seg_start[k];
    VS_CHECK(seg_start[k] >= 0 && seg_start[k] <= S && (k == 0 || seg_start[k] >= seg_start[k - 1]),
             "segment starts must be non-decreasing within [0, S]");
  }
  hipStream_t st = (hipStream_t)stream;
  if (B == 0) return hipMemsetAsync(out, 0, (size_t)nseg * N * sizeof(float), st) == hipSuccess ? VS_OK : VS_ERR_HIP;
  float* part = (float*)ws;
  const int rowsets = kThreads / (N / 8);
  int maxrows = 0;
  for (int k = 0; k < nseg; ++k) maxrows = std::max(maxrows, seg.start[k + 1] - seg.start[k]);
  const int nblk = std::max(1, std::min(blocks_for(maxrows, rowsets * 16, kMaxPartials), kMaxPartials / (nseg * B)));
  const size_t lds = (size_t)rowsets * N * sizeof(float);
  if (dtype == VS_BF16)
    hipLaunchKernelGGL(colsum_seg_kernel<bf16>, dim3(nblk, nseg * B), dim3(kThreads), lds, st, (const bf16*)x, part,
                       B, S, N, seg);
  else
    hipLaunchKernelGGL(colsum_seg_kernel<float>, dim3(nblk, nseg * B), dim3(kThreads), lds, st, (const float*)x,
                       part, B, S, N, seg);
  hipLaunchKernelGGL(colsum_partials_kernel<float>, dim3((N + 31) / 32, nseg), dim3(kCsThreads), 0, st, part, out,
                     (float*)nullptr, nblk * B, N, N);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_splitk_sum(int dtype, const float* partials, int num_parts, long long n, const float* extra,
                             void* out, void* stream) {
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");
  VS_CHECK(num_parts >= 0 && n >= 0 && n % 4 == 0, "n must be a multiple of 4");
  VS_CHECK(out && (num_parts == 0 || partials), "null pointer");
  if (n == 0) return VS_OK;
  hipStream_t st = (hipStream_t)stream;
  const long long n4 = n / 4;
  bool phased = num_parts >= 16;             // VS_SPLITK_PHASED=0: one thread per quad
  if (const char* e = getenv("VS_SPLITK_PHASED")) phased = phased && atoi(e) != 0;
  if (phased) {
    constexpr int PH = 8;
    const long long blocks = (n4 + kThreads / PH - 1) / (kThreads / PH);
    VS_CHECK(blocks < (1LL << 31), "split-K output too large");
    if (dtype == VS_BF16)
      hipLaunchKernelGGL((splitk_sum_phased_kernel<bf16, PH>), dim3((unsigned)blocks), dim3(kThreads), 0, st,
                         partials, extra, (bf16*)out, num_parts, n4);
    else
      hipLaunchKernelGGL((splitk_sum_phased_kernel<float, PH>), dim3((unsigned)blocks), dim3(kThreads), 0, st,
                         partials, extra, (float*)out, num_parts, n4);
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
  const int grid = (int)std::min<long long>((n4 + kThreads - 1) / kThreads, 256 * 16);
  if (dtype == VS_BF16)
    hipLaunchKernelGGL(splitk_sum_kernel<bf16>, dim3(grid), dim3(kThreads), 0, st, partials, extra, (bf16*)out,
                       num_parts, n4);
  else
    hipLaunchKernelGGL(splitk_sum_kernel<float>, dim3(grid), dim3(kThreads), 0, st, partials, extra, (float*)out,
                       num_parts, n4);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

// dx = dy * act'(x) (act 0: ReLU, 1: exact GELU) and dx_colsum[N] = column sums of dx as
// stored; x is the activation's INPUT.  ws: vs_column_sum_workspace_bytes(M, N) bytes.
extern "C" int vs_act_backward_colsum(int dtype, int act, const void* dy, const void* x, void* dx, void* dx_colsum,
                                      void* ws, int M, int N, void* stream) {
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");
  VS_CHECK(act == 0 || act == 1, "act must be 0 (ReLU) or 1 (GELU)");
  VS_CHECK(M >= 0 && N > 0 && N % 8 == 0 && N <= 8 * kColBlock, "N must be a multiple of 8, <= 16384");
  VS_CHECK(dx_colsum && ws && (M == 0 || (dy && x && dx)), "null pointer");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  const int Nb = std::min(N, kColBlock), rowsets = kThreads / (Nb / 8);
  const int grid = blocks_for(M, rowsets * 16, kMaxPartials);
  const dim3 g2(grid, (N + kColBlock - 1) / kColBlock);
  const size_t lds = (size_t)rowsets * Nb * sizeof(float);
#define VS_ACTB(TT, A)                                                                                          \
  hipLaunchKernelGGL((act_bwd_colsum_kernel<TT, A>), g2, dim3(kThreads), lds, st, (const TT*)dy,                \
                     (const TT*)x, (TT*)dx, part, M, N)
  if (dtype == VS_BF16) {
    if (act) VS_ACTB(bf16, 1); else VS_ACTB(bf16, 0);
    hipLaunchKernelGGL(colsum_partials_kernel<bf16>, dim3((N + 31) / 32), dim3(kCsThreads), 0, st, part,
                       (bf16*)dx_colsum, (bf16*)nullptr, grid, N, N);
  } else {
    if (act) VS_ACTB(float, 1); else VS_ACTB(float, 0);
    hipLaunchKernelGGL(colsum_partials_kernel<float>, dim3((N + 31) / 32), dim3(kCsThreads), 0, st, part,
                       (float*)dx_colsum, (float*)nullptr, grid, N, N);
  }
#undef VS_ACTB
  VS_LAUNCH_CHECK();
  return VS_OK;
}
