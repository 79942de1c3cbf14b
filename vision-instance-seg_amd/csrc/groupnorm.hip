// GroupNorm over channels-last activations (NHWC memory), forward + backward, optional
// fused ReLU.
//
// The pixel decoder's ConvGN blocks (upstream MSDeformAttnPixelDecoder: Conv2d + GroupNorm
// (32 groups), HF:m2f Mask2FormerPixelDecoder lateral / output convs, input projections)
// see MIOpen's channels-last conv outputs; torch's GroupNorm first copies them to NCHW.
// Here x is [B, HW, C] with groups of exactly 8 channels (C = 8 G): one 16-B bf16 chunk
// (two float4 for f32) per (row, group), so a thread owns one group of one row at a time.
//
// Forward: (1) per (chunk of rows, image) partial sum / sum of squares per group (f32),
// (2) finalize mean / rstd per (image, group) in f64, (3) normalise (+ ReLU).
// Backward: (1) per chunk partials of sum(g) and sum(g * xhat) per group and of
// sum(dy * xhat), sum(dy) per channel (g = dy * w, masked by the recomputed ReLU),
// (2) finalize the group coefficients and reduce dw / db over chunks (fixed order),
// (3) dx = rstd (g - mean(g) - xhat mean(g xhat)).  Semantics of
// torch.nn.functional.group_norm (biased variance) followed by relu when requested.
#include "common.h"

#include <algorithm>

namespace vs {
namespace {

constexpr int kT = 256;
// rows per chunk: max(kMinRows, HW / kMaxChunks).  Up to 256 chunks per image so the
// statistics passes launch ~1024 blocks at B = 4 (16 KB of loads in flight per block;
// 64 chunks left them at 1.2-2.2 TB/s, profiles/r6_gn_parallel_ab.txt).
constexpr int kMinRows = 32;
constexpr int kMaxChunks = 256;
constexpr int kPartsPerSlice = 32;  // dw / db level-1 slices: >= 32 parts each, <= 64 slices
constexpr int kMaxSlices = 64;

template <typename T>
__device__ __forceinline__ void ld8f(const T* p, float* v) {
  Vec16<T>::load(p, v);
  if constexpr (Vec16<T>::N == 4) Vec16<T>::load(p + 4, v + 4);
}

template <typename T>
__device__ __forceinline__ void st8f(T* p, const float* v) {
  Vec16<T>::store(p, v);
  if constexpr (Vec16<T>::N == 4) Vec16<T>::store(p + 4, v + 4);
}

// partials: part[b][chunk][g][2] = (sum, sumsq) over the chunk's rows and the group's 8 ch
template <typename T>
__global__ void __launch_bounds__(kT) gn_stats_kernel(const T* __restrict__ x, float* __restrict__ part, int HW, int G,
                                                      int nchunk, int rpc) {
  extern __shared__ float red[];             // [rowlanes][G][2]
  const int chunk = blockIdx.x, b = blockIdx.y;
  const int rowlanes = kT / G;               // threads per group column (G <= 256)
  const int g = threadIdx.x % G, rl = threadIdx.x / G;
  const int C = 8 * G;
  const int r0 = chunk * rpc, r1 = min(HW, r0 + rpc);
  float s = 0.f, q = 0.f;
  if (rl < rowlanes) {
    const T* xb = x + (size_t)b * HW * C + g * 8;
    for (int r = r0 + rl; r < r1; r += 4 * rowlanes) {
      float v[4][8];                          // 4 rows' loads in flight
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (r + u * rowlanes < r1) {
          ld8f(xb + (size_t)(r + u * rowlanes) * C, v[u]);
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) v[u][i] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          s += v[u][i];
          q += v[u][i] * v[u][i];
        }
    }
    red[(rl * G + g) * 2 + 0] = s;
    red[(rl * G + g) * 2 + 1] = q;
  }
  __syncthreads();
  for (int gg = threadIdx.x; gg < G; gg += kT) {
    float a = 0.f, c = 0.f;
    for (int k = 0; k < rowlanes; ++k) {
      a += red[(k * G + gg) * 2 + 0];
      c += red[(k * G + gg) * 2 + 1];
    }
    float* o = part + (((size_t)b * nchunk + chunk) * G + gg) * 2;
    o[0] = a;
    o[1] = c;
  }
}

// butterfly over the 64 lanes: every pair adds the same two operands, so all lanes end with
// the same, schedule-independent value
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// one wave per (b, g): lane l sums chunks l, l + 64, ... in f64, then a wave butterfly
__device__ __forceinline__ bool group_sums(const float* __restrict__ part, int i, int G, int nchunk, double& s,
                                          double& q) {
  const int l = threadIdx.x & 63;
  const int b = i / G, g = i % G;
  s = 0.0;
  q = 0.0;
  for (int c = l; c < nchunk; c += 64) {
    const float2 p = *reinterpret_cast<const float2*>(part + (((size_t)b * nchunk + c) * G + g) * 2);
    s += p.x;
    q += p.y;
  }
  s = wave_sum_f64(s);
  q = wave_sum_f64(q);
  return l == 0;
}

__global__ void __launch_bounds__(kT) gn_finalize_kernel(const float* __restrict__ part, float* __restrict__ mean,
                                                         float* __restrict__ rstd, int B, int HW, int G, int nchunk,
                                                         float eps) {
  const int i = blockIdx.x * (kT / 64) + (threadIdx.x >> 6);   // (b, g), wave-uniform
  if (i >= B * G) return;
  double s, q;
  if (!group_sums(part, i, G, nchunk, s, q)) return;
  const double n = (double)HW * 8.0;
  const double m = s / n;
  const double var = fmax(q / n - m * m, 0.0);
  mean[i] = (float)m;
  rstd[i] = (float)(1.0 / sqrt(var + (double)eps));
}

template <typename T, bool RELU>
__global__ void __launch_bounds__(kT) gn_apply_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                      const T* __restrict__ bias, const float* __restrict__ mean,
                                                      const float* __restrict__ rstd, T* __restrict__ y, int B, int HW,
                                                      int G) {
  const long long n = (long long)B * HW * G;     // (row, group) chunks
  for (long long i = (long long)blockIdx.x * kT + threadIdx.x; i < n; i += (long long)gridDim.x * kT) {
    const int g = (int)(i % G);
    const long long row = i / G;
    const int b = (int)(row / HW);
    const float m = mean[b * G + g], rs = rstd[b * G + g];
    float v[8], wv[8], bv[8];
    ld8f(x + i * 8, v);
    ld8f(w + g * 8, wv);
    ld8f(bias + g * 8, bv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float o = (v[k] - m) * rs * wv[k] + bv[k];
      v[k] = RELU ? fmaxf(o, 0.f) : o;
    }
    st8f(y + i * 8, v);
  }
}

// backward partials: gpart[b][chunk][g][2] = (sum g, sum g*xhat); cpart[b*nchunk+chunk][C][2]
// = (sum dy*xhat, sum dy) with dy masked by the ReLU
template <typename T, bool RELU>
__global__ void __launch_bounds__(kT) gn_bwd_stats_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                          const T* __restrict__ w, const T* __restrict__ bias,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ rstd, float* __restrict__ gpart,
                                                          float* __restrict__ cpart, int HW, int G, int nchunk,
                                                          int rpc) {
  extern __shared__ float red[];             // [rowlanes][G][2 + 16]
  const int chunk = blockIdx.x, b = blockIdx.y;
  const int rowlanes = kT / G;
  const int g = threadIdx.x % G, rl = threadIdx.x / G;
  const int C = 8 * G;
  const int r0 = chunk * rpc, r1 = min(HW, r0 + rpc);
  constexpr int W = 2 + 16;
  float s1 = 0.f, s2 = 0.f, cw[8], cb[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) cw[k] = cb[k] = 0.f;
  if (rl < rowlanes) {
    const float m = mean[b * G + g], rs = rstd[b * G + g];
    float wv[8], bv[8];
    ld8f(w + g * 8, wv);
    ld8f(bias + g * 8, bv);
    const size_t base = (size_t)b * HW * C + g * 8;
    for (int r = r0 + rl; r < r1; r += 2 * rowlanes) {
      float xv[2][8], dv[2][8];               // 2 rows' loads in flight
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (r + u * rowlanes < r1) {
          ld8f(x + base + (size_t)(r + u * rowlanes) * C, xv[u]);
          ld8f(dy + base + (size_t)(r + u * rowlanes) * C, dv[u]);
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) xv[u][k] = dv[u][k] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float xh = (xv[u][k] - m) * rs;
        float d = dv[u][k];
        if (RELU && xh * wv[k] + bv[k] <= 0.f) d = 0.f;
        const float gg = d * wv[k];
        s1 += gg;
        s2 += gg * xh;
        cw[k] += d * xh;
        cb[k] += d;
      }
    }
    float* o = red + (rl * G + g) * W;
    o[0] = s1;
    o[1] = s2;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o[2 + k] = cw[k];
      o[10 + k] = cb[k];
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < G * W; j += kT) {
    const int gg = j / W, f = j % W;
    float a = 0.f;
    for (int k = 0; k < rowlanes; ++k) a += red[(k * G + gg) * W + f];
    if (f < 2) {
      gpart[(((size_t)b * nchunk + chunk) * G + gg) * 2 + f] = a;
    } else {
      const int ch = gg * 8 + (f - 2) % 8;
      const int which = (f - 2) / 8;    // 0: dw, 1: db
      cpart[(((size_t)b * nchunk + chunk) * C + ch) * 2 + which] = a;
    }
  }
}

// Blocks [0, nfin): group coefficients c1 = mean(g), c2 = mean(g xhat), one wave per (b, g).
// Blocks [nfin, ...): level 1 of dw / db -- a block sums one slice of pps consecutive parts
// for 64 (channel, which) columns (lane = column, 4 waves interleaved over the slice) into
// wpart[slice][2C]; gn_bwd_apply_kernel adds the slices in order.  Fixed order throughout.
__global__ void __launch_bounds__(kT) gn_bwd_finalize_kernel(const float* __restrict__ gpart, float* __restrict__ c12,
                                                             const float* __restrict__ cpart,
                                                             float* __restrict__ wpart, int B, int HW, int G,
                                                             int nchunk, int nfin, int pps) {
  if ((int)blockIdx.x < nfin) {
    const int i = blockIdx.x * (kT / 64) + (threadIdx.x >> 6);
    if (i >= B * G) return;
    double a, c;
    if (!group_sums(gpart, i, G, nchunk, a, c)) return;
    const double n = (double)HW * 8.0;
    c12[i * 2 + 0] = (float)(a / n);
    c12[i * 2 + 1] = (float)(c / n);
    return;
  }
  __shared__ float red[4][64];
  const int C2 = 16 * G;                         // (channel, which) columns
  const int ncb = (C2 + 63) / 64;
  const int nb = blockIdx.x - nfin, cb = nb % ncb, sl = nb / ncb;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = cb * 64 + lane;
  const int k1 = min(B * nchunk, (sl + 1) * pps);
  float a0 = 0.f, a1 = 0.f;
  if (col < C2) {
    int k = sl * pps + w;
    for (; k + 4 < k1; k += 8) {
      a0 += cpart[(size_t)k * C2 + col];
      a1 += cpart[(size_t)(k + 4) * C2 + col];
    }
    if (k < k1) a0 += cpart[(size_t)k * C2 + col];
  }
  red[w][lane] = a0 + a1;
  __syncthreads();
  if (w == 0 && col < C2) wpart[(size_t)sl * C2 + col] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

template <typename T, bool RELU>
__global__ void __launch_bounds__(kT) gn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                          const T* __restrict__ w, const T* __restrict__ bias,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ rstd,
                                                          const float* __restrict__ c12, T* __restrict__ dx, int B,
                                                          int HW, int G, const float* __restrict__ wpart, int nslice,
                                                          T* __restrict__ dw, T* __restrict__ db) {
  if ((int)blockIdx.x * kT < 16 * G) {           // level 2 of dw / db: slices in order
    const int col = blockIdx.x * kT + threadIdx.x;
    if (col < 16 * G) {
      float t = 0.f;
      for (int s = 0; s < nslice; ++s) t += wpart[(size_t)s * 16 * G + col];
      ((col & 1) ? db : dw)[col >> 1] = from_f32<T>(t);
    }
  }
  const long long n = (long long)B * HW * G;
  for (long long i = (long long)blockIdx.x * kT + threadIdx.x; i < n; i += (long long)gridDim.x * kT) {
    const int g = (int)(i % G);
    const int b = (int)((i / G) / HW);
    const int bg = b * G + g;
    const float m = mean[bg], rs = rstd[bg], c1 = c12[bg * 2], c2 = c12[bg * 2 + 1];
    float xv[8], dv[8], wv[8], bv[8];
    ld8f(x + i * 8, xv);
    ld8f(dy + i * 8, dv);
    ld8f(w + g * 8, wv);
    ld8f(bias + g * 8, bv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float xh = (xv[k] - m) * rs;
      float d = dv[k];
      if (RELU && xh * wv[k] + bv[k] <= 0.f) d = 0.f;
      xv[k] = rs * (d * wv[k] - c1 - xh * c2);
    }
    st8f(dx + i * 8, xv);
  }
}

// ---------------------------------------------------------------------------------
// NCHW layout: a group is Cg = C / G consecutive channel planes of HW contiguous elements,
// so every pass is a contiguous stream.  One block per (b, c) plane for the statistics.
template <typename T, bool VEC>
__device__ __forceinline__ void plane_load8(const T* p, long long j, float* v) {
  if constexpr (VEC) {
    ld8f(p + 8 * j, v);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = to_f32(p[8 * j + k]);
  }
}

__device__ __forceinline__ void block_sum2(float& a, float& b, float* sh) {
  for (int o = 32; o >= 1; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) {
    sh[2 * w] = a;
    sh[2 * w + 1] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float x = 0.f, y = 0.f;
    for (int i = 0; i < kT / 64; ++i) {
      x += sh[2 * i];
      y += sh[2 * i + 1];
    }
    sh[2 * (kT / 64)] = x;
    sh[2 * (kT / 64) + 1] = y;
  }
  __syncthreads();
  a = sh[2 * (kT / 64)];
  b = sh[2 * (kT / 64) + 1];
}

// cpart[b*C + c] = (sum, sumsq) of the plane
template <typename T, bool VEC>
__global__ void __launch_bounds__(kT) gn_nchw_stats_kernel(const T* __restrict__ x, float* __restrict__ cpart, int HW) {
  __shared__ float sh[2 * (kT / 64) + 2];
  const int plane = blockIdx.x;
  const T* p = x + (size_t)plane * HW;
  float s = 0.f, q = 0.f;
  const int nv = HW / 8;
  int j = threadIdx.x;
  for (; j + 3 * kT < nv; j += 4 * kT) {
    float v[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) plane_load8<T, VEC>(p, j + u * kT, v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s += v[u][k];
        q += v[u][k] * v[u][k];
      }
  }
  for (; j < nv; j += kT) {
    float v[8];
    plane_load8<T, VEC>(p, j, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s += v[k];
      q += v[k] * v[k];
    }
  }
  for (int i = nv * 8 + threadIdx.x; i < HW; i += kT) {
    const float v = to_f32(p[i]);
    s += v;
    q += v * v;
  }
  block_sum2(s, q, sh);
  if (threadIdx.x == 0) {
    cpart[plane * 2] = s;
    cpart[plane * 2 + 1] = q;
  }
}

__global__ void __launch_bounds__(kT) gn_nchw_finalize_kernel(const float* __restrict__ cpart, float* __restrict__ mean,
                                                              float* __restrict__ rstd, int B, int HW, int C, int G,
                                                              float eps) {
  const int i = blockIdx.x * kT + threadIdx.x;   // (b, g)
  if (i >= B * G) return;
  const int Cg = C / G;
  double s = 0.0, q = 0.0;
  for (int c = 0; c < Cg; ++c) {
    s += cpart[((size_t)i * Cg + c) * 2];
    q += cpart[((size_t)i * Cg + c) * 2 + 1];
  }
  const double n = (double)HW * Cg;
  const double m = s / n;
  const double var = fmax(q / n - m * m, 0.0);
  mean[i] = (float)m;
  rstd[i] = (float)(1.0 / sqrt(var + (double)eps));
}

template <typename T, bool RELU, bool VEC>
__global__ void __launch_bounds__(kT) gn_nchw_apply_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                           const T* __restrict__ bias, const float* __restrict__ mean,
                                                           const float* __restrict__ rstd, T* __restrict__ y, int B,
                                                           int HW, int C, int G) {
  const int Cg = C / G;
  if constexpr (VEC) {
    const long long n = (long long)B * C * HW / 8;
    for (long long i = (long long)blockIdx.x * kT + threadIdx.x; i < n; i += (long long)gridDim.x * kT) {
      const int plane = (int)(i * 8 / HW);
      const int c = plane % C, bg = plane / Cg;      // plane = b*C + c, group index b*G + c/Cg
      const float m = mean[bg], rs = rstd[bg], wv = to_f32(w[c]), bv = to_f32(bias[c]);
      float v[8];
      ld8f(x + i * 8, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float o = (v[k] - m) * rs * wv + bv;
        v[k] = RELU ? fmaxf(o, 0.f) : o;
      }
      st8f(y + i * 8, v);
    }
  } else {
    const long long n = (long long)B * C * HW;
    for (long long i = (long long)blockIdx.x * kT + threadIdx.x; i < n; i += (long long)gridDim.x * kT) {
      const int plane = (int)(i / HW);
      const int c = plane % C, bg = plane / Cg;
      const float o = (to_f32(x[i]) - mean[bg]) * rstd[bg] * to_f32(w[c]) + to_f32(bias[c]);
      y[i] = from_f32<T>(RELU ? fmaxf(o, 0.f) : o);
    }
  }
}

// cpart[b*C + c] = (sum dy*xhat, sum dy) with dy masked by the recomputed ReLU
template <typename T, bool RELU, bool VEC>
__global__ void __launch_bounds__(kT) gn_nchw_bwd_stats_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                               const T* __restrict__ w, const T* __restrict__ bias,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ rstd,
                                                               float* __restrict__ cpart, int HW, int C, int G) {
  __shared__ float sh[2 * (kT / 64) + 2];
  const int plane = blockIdx.x;
  const int c = plane % C, bg = plane / (C / G);
  const float m = mean[bg], rs = rstd[bg], wv = to_f32(w[c]), bv = to_f32(bias[c]);
  const T* px = x + (size_t)plane * HW;
  const T* pd = dy + (size_t)plane * HW;
  float sw = 0.f, sb = 0.f;
  const int nv = HW / 8;
  int j = threadIdx.x;
  for (; j + kT < nv; j += 2 * kT) {
    float xv[2][8], dv[2][8];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      plane_load8<T, VEC>(px, j + u * kT, xv[u]);
      plane_load8<T, VEC>(pd, j + u * kT, dv[u]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float xh = (xv[u][k] - m) * rs;
        float d = dv[u][k];
        if (RELU && xh * wv + bv <= 0.f) d = 0.f;
        sw += d * xh;
        sb += d;
      }
  }
  for (; j < nv; j += kT) {
    float xv[8], dv[8];
    plane_load8<T, VEC>(px, j, xv);
    plane_load8<T, VEC>(pd, j, dv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float xh = (xv[k] - m) * rs;
      float d = dv[k];
      if (RELU && xh * wv + bv <= 0.f) d = 0.f;
      sw += d * xh;
      sb += d;
    }
  }
  for (int i = nv * 8 + threadIdx.x; i < HW; i += kT) {
    const float xh = (to_f32(px[i]) - m) * rs;
    float d = to_f32(pd[i]);
    if (RELU && xh * wv + bv <= 0.f) d = 0.f;
    sw += d * xh;
    sb += d;
  }
  block_sum2(sw, sb, sh);
  if (threadIdx.x == 0) {
    cpart[plane * 2] = sw;
    cpart[plane * 2 + 1] = sb;
  }
}

// c12[b*G + g] = (mean over the group of w*dy, mean of w*dy*xhat) from the channel sums;
// dw[c] / db[c] = sums over the batch (fixed order)
template <typename T>
__global__ void __launch_bounds__(kT) gn_nchw_bwd_finalize_kernel(const float* __restrict__ cpart,
                                                                  const T* __restrict__ w, float* __restrict__ c12,
                                                                  T* __restrict__ dw, T* __restrict__ db, int B,
                                                                  int HW, int C, int G) {
  const int i = blockIdx.x * kT + threadIdx.x;
  const int Cg = C / G;
  if (i < B * G) {
    double a = 0.0, c = 0.0;
    for (int k = 0; k < Cg; ++k) {
      const int ch = (i % G) * Cg + k;
      const double wv = (double)to_f32(w[ch]);
      a += wv * cpart[((size_t)i * Cg + k) * 2 + 1];
      c += wv * cpart[((size_t)i * Cg + k) * 2];
    }
    const double n = (double)HW * Cg;
    c12[i * 2] = (float)(a / n);
    c12[i * 2 + 1] = (float)(c / n);
  }
  if (i < C) {
    float sw = 0.f, sb = 0.f;
    for (int b = 0; b < B; ++b) {
      sw += cpart[((size_t)b * C + i) * 2];
      sb += cpart[((size_t)b * C + i) * 2 + 1];
    }
    dw[i] = from_f32<T>(sw);
    db[i] = from_f32<T>(sb);
  }
}

template <typename T, bool RELU, bool VEC>
__global__ void __launch_bounds__(kT) gn_nchw_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                               const T* __restrict__ w, const T* __restrict__ bias,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ rstd,
                                                               const float* __restrict__ c12, T* __restrict__ dx,
                                                               int B, int HW, int C, int G) {
  const int Cg = C / G;
  if constexpr (VEC) {
    const long long n = (long long)B * C * HW / 8;
    for (long long i = (long long)blockIdx.x * kT + threadIdx.x; i < n; i += (long long)gridDim.x * kT) {
      const int plane = (int)(i * 8 / HW);
      const int c = plane % C, bg = plane / Cg;
      const float m = mean[bg], rs = rstd[bg], c1 = c12[bg * 2], c2 = c12[bg * 2 + 1];
      const float wv = to_f32(w[c]), bv = to_f32(bias[c]);
      float xv[8], dv[8];
      ld8f(x + i * 8, xv);
      ld8f(dy + i * 8, dv);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float xh = (xv[k] - m) * rs;
        float d = dv[k];
        if (RELU && xh * wv + bv <= 0.f) d = 0.f;
        xv[k] = rs * (d * wv - c1 - xh * c2);
      }
      st8f(dx + i * 8, xv);
    }
  } else {
    const long long n = (long long)B * C * HW;
    for (long long i = (long long)blockIdx.x * kT + threadIdx.x; i < n; i += (long long)gridDim.x * kT) {
      const int plane = (int)(i / HW);
      const int c = plane % C, bg = plane / Cg;
      const float m = mean[bg], rs = rstd[bg], wv = to_f32(w[c]), bv = to_f32(bias[c]);
      const float xh = (to_f32(x[i]) - m) * rs;
      float d = to_f32(dy[i]);
      if (RELU && xh * wv + bv <= 0.f) d = 0.f;
      dx[i] = from_f32<T>(rs * (d * wv - c12[bg * 2] - xh * c12[bg * 2 + 1]));
    }
  }
}

int rows_per_chunk(int HW) { return std::max(kMinRows, (HW + kMaxChunks - 1) / kMaxChunks); }

int chunks_for(int HW) { return (HW + rows_per_chunk(HW) - 1) / rows_per_chunk(HW); }

int apply_grid(long long n) { return (int)std::min<long long>((n + kT - 1) / kT, 256 * 32); }

// dw / db level-1 slicing of the B * nchunk channel partials
int parts_per_slice(int nparts) { return std::max(kPartsPerSlice, (nparts + kMaxSlices - 1) / kMaxSlices); }

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" long long vs_group_norm_workspace_bytes(int B, int HW, int C, int G) {
  const long long nchunk = chunks_for(HW);
  // forward: group partials; backward: group partials + channel partials + c12 + dw/db slices
  return (long long)B * nchunk * G * 2 * 4 + (long long)B * nchunk * C * 2 * 4 + (long long)B * G * 2 * 4 +
         (long long)kMaxSlices * C * 2 * 4 + 256;
}

#define VS_GN_CHECK()                                                                           \
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");             \
  VS_CHECK(B > 0 && HW > 0 && G > 0 && G <= kT && C == 8 * G, "groups of exactly 8 channels"); \
  VS_CHECK(kT % G == 0, "G must divide 256")

extern "C" int vs_group_norm_forward(int dtype, const void* x, const void* weight, const void* bias, void* y,
                                     float* mean, float* rstd, void* workspace, int B, int HW, int C, int G,
                                     float eps, int relu, void* stream) {
  VS_GN_CHECK();
  VS_CHECK(x && weight && bias && y && mean && rstd && workspace, "null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int nchunk = chunks_for(HW);
  float* part = (float*)workspace;
  const size_t lds = (size_t)kT * 2 * sizeof(float);
  const long long n = (long long)B * HW * G;
  if (dtype == VS_BF16)
    hipLaunchKernelGGL(gn_stats_kernel<bf16>, dim3(nchunk, B), dim3(kT), lds, st, (const bf16*)x, part, HW, G, nchunk,
                       rows_per_chunk(HW));
  else
    hipLaunchKernelGGL(gn_stats_kernel<float>, dim3(nchunk, B), dim3(kT), lds, st, (const float*)x, part, HW, G,
                       nchunk, rows_per_chunk(HW));
  hipLaunchKernelGGL(gn_finalize_kernel, dim3((B * G + 3) / 4), dim3(kT), 0, st, part, mean, rstd, B, HW, G, nchunk,
                     eps);
#define VS_GN_APPLY(TT, R)                                                                                    \
  hipLaunchKernelGGL((gn_apply_kernel<TT, R>), dim3(apply_grid(n)), dim3(kT), 0, st, (const TT*)x,           \
                     (const TT*)weight, (const TT*)bias, mean, rstd, (TT*)y, B, HW, G)
  if (dtype == VS_BF16) {
    if (relu) VS_GN_APPLY(bf16, true); else VS_GN_APPLY(bf16, false);
  } else {
    if (relu) VS_GN_APPLY(float, true); else VS_GN_APPLY(float, false);
  }
#undef VS_GN_APPLY
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_group_norm_backward(int dtype, const void* grad_y, const void* x, const void* weight,
                                      const void* bias, const float* mean, const float* rstd, void* grad_x,
                                      void* grad_weight, void* grad_bias, void* workspace, int B, int HW, int C,
                                      int G, int relu, void* stream) {
  VS_GN_CHECK();
  VS_CHECK(grad_y && x && weight && bias && mean && rstd && grad_x && grad_weight && grad_bias && workspace,
           "null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int nchunk = chunks_for(HW);
  float* gpart = (float*)workspace;
  float* cpart = gpart + (size_t)B * nchunk * G * 2;
  float* c12 = cpart + (size_t)B * nchunk * C * 2;
  float* wpart = c12 + (size_t)B * G * 2;
  const size_t lds = (size_t)kT * 18 * sizeof(float);
  const long long n = (long long)B * HW * G;
  const int nfin = (B * G + 3) / 4;
  const int pps = parts_per_slice(B * nchunk);
  const int nslice = (B * nchunk + pps - 1) / pps;
  const int nwb = ((2 * C + 63) / 64) * nslice;
  const int agrid = std::max(apply_grid(n), (2 * C + kT - 1) / kT);
#define VS_GN_BWD(TT, R)                                                                                          \
  hipLaunchKernelGGL((gn_bwd_stats_kernel<TT, R>), dim3(nchunk, B), dim3(kT), lds, st, (const TT*)grad_y,         \
                     (const TT*)x, (const TT*)weight, (const TT*)bias, mean, rstd, gpart, cpart, HW, G, nchunk,    \
                     rows_per_chunk(HW));                                                                         \
  hipLaunchKernelGGL(gn_bwd_finalize_kernel, dim3(nfin + nwb), dim3(kT), 0, st, gpart, c12, cpart, wpart, B, HW, G, \
                     nchunk, nfin, pps);                                                                          \
  hipLaunchKernelGGL((gn_bwd_apply_kernel<TT, R>), dim3(agrid), dim3(kT), 0, st, (const TT*)grad_y, (const TT*)x, \
                     (const TT*)weight, (const TT*)bias, mean, rstd, c12, (TT*)grad_x, B, HW, G, wpart, nslice,   \
                     (TT*)grad_weight, (TT*)grad_bias)
  if (dtype == VS_BF16) {
    if (relu) { VS_GN_BWD(bf16, true); } else { VS_GN_BWD(bf16, false); }
  } else {
    if (relu) { VS_GN_BWD(float, true); } else { VS_GN_BWD(float, false); }
  }
#undef VS_GN_BWD
  VS_LAUNCH_CHECK();
  return VS_OK;
}

// ------------------------------------------------------------------------ NCHW entry points
extern "C" long long vs_group_norm_nchw_workspace_bytes(int B, int C, int G) {
  return (long long)B * C * 2 * 4 + (long long)B * G * 2 * 4 + 256;
}

#define VS_GN_NCHW_CHECK()                                                                        \
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");               \
  VS_CHECK(B > 0 && HW > 0 && G > 0 && C > 0 && C % G == 0, "channels must be a multiple of groups")

extern "C" int vs_group_norm_nchw_forward(int dtype, const void* x, const void* weight, const void* bias, void* y,
                                          float* mean, float* rstd, void* workspace, int B, int C, int HW, int G,
                                          float eps, int relu, void* stream) {
  VS_GN_NCHW_CHECK();
  VS_CHECK(x && weight && bias && y && mean && rstd && workspace, "null pointer");
  hipStream_t st = (hipStream_t)stream;
  float* cpart = (float*)workspace;
  const bool vec = HW % 8 == 0;
  const long long n = (long long)B * C * HW / (vec ? 8 : 1);
#define VS_GN_NCHW_FWD(TT, R, V)                                                                                  \
  hipLaunchKernelGGL((gn_nchw_stats_kernel<TT, V>), dim3(B * C), dim3(kT), 0, st, (const TT*)x, cpart, HW);         \
  hipLaunchKernelGGL(gn_nchw_finalize_kernel, dim3((B * G + kT - 1) / kT), dim3(kT), 0, st, cpart, mean, rstd, B, \
                     HW, C, G, eps);                                                                              \
  hipLaunchKernelGGL((gn_nchw_apply_kernel<TT, R, V>), dim3(apply_grid(n)), dim3(kT), 0, st, (const TT*)x,        \
                     (const TT*)weight, (const TT*)bias, mean, rstd, (TT*)y, B, HW, C, G)
  if (dtype == VS_BF16) {
    if (vec) { if (relu) { VS_GN_NCHW_FWD(bf16, true, true); } else { VS_GN_NCHW_FWD(bf16, false, true); } }
    else { if (relu) { VS_GN_NCHW_FWD(bf16, true, false); } else { VS_GN_NCHW_FWD(bf16, false, false); } }
  } else {
    if (vec) { if (relu) { VS_GN_NCHW_FWD(float, true, true); } else { VS_GN_NCHW_FWD(float, false, true); } }
    else { if (relu) { VS_GN_NCHW_FWD(float, true, false); } else { VS_GN_NCHW_FWD(float, false, false); } }
  }
#undef VS_GN_NCHW_FWD
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_group_norm_nchw_backward(int dtype, const void* grad_y, const void* x, const void* weight,
                                           const void* bias, const float* mean, const float* rstd, void* grad_x,
                                           void* grad_weight, void* grad_bias, void* workspace, int B, int C, int HW,
                                           int G, int relu, void* stream) {
  VS_GN_NCHW_CHECK();
  VS_CHECK(grad_y && x && weight && bias && mean && rstd && grad_x && grad_weight && grad_bias && workspace,
           "null pointer");
  hipStream_t st = (hipStream_t)stream;
  float* cpart = (float*)workspace;
  float* c12 = cpart + (size_t)B * C * 2;
  const bool vec = HW % 8 == 0;
  const long long n = (long long)B * C * HW / (vec ? 8 : 1);
  const int fin = (std::max(B * G, C) + kT - 1) / kT;
#define VS_GN_NCHW_BWD(TT, R, V)                                                                                   \
  hipLaunchKernelGGL((gn_nchw_bwd_stats_kernel<TT, R, V>), dim3(B * C), dim3(kT), 0, st, (const TT*)grad_y,        \
                     (const TT*)x, (const TT*)weight, (const TT*)bias, mean, rstd, cpart, HW, C, G);               \
  hipLaunchKernelGGL((gn_nchw_bwd_finalize_kernel<TT>), dim3(fin), dim3(kT), 0, st, cpart, (const TT*)weight, c12, \
                     (TT*)grad_weight, (TT*)grad_bias, B, HW, C, G);                                               \
  hipLaunchKernelGGL((gn_nchw_bwd_apply_kernel<TT, R, V>), dim3(apply_grid(n)), dim3(kT), 0, st,                   \
                     (const TT*)grad_y, (const TT*)x, (const TT*)weight, (const TT*)bias, mean, rstd, c12,         \
                     (TT*)grad_x, B, HW, C, G)
  if (dtype == VS_BF16) {
    if (vec) { if (relu) { VS_GN_NCHW_BWD(bf16, true, true); } else { VS_GN_NCHW_BWD(bf16, false, true); } }
    else { if (relu) { VS_GN_NCHW_BWD(bf16, true, false); } else { VS_GN_NCHW_BWD(bf16, false, false); } }
  } else {
    if (vec) { if (relu) { VS_GN_NCHW_BWD(float, true, true); } else { VS_GN_NCHW_BWD(float, false, true); } }
    else { if (relu) { VS_GN_NCHW_BWD(float, true, false); } else { VS_GN_NCHW_BWD(float, false, false); } }
  }
#undef VS_GN_NCHW_BWD
  VS_LAUNCH_CHECK();
  return VS_OK;
}
