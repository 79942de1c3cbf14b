// Pixel-decoder FPN merge: out = cur + upsample_bilinear(src)  (HF:m2f:1405-1413,
// `F.interpolate(..., mode="bilinear", align_corners=False)` added to the lateral
// branch), and its backward for src.
//
// cur / out are NCHW planes [B, C, H, W] (the 1/4-resolution blocks run NCHW for
// MIOpen's 3x3 conv); src is the encoder's token-major level [B, Hs*Ws, C] (a view of
// the encoder output, batch stride given).  The torch composition is an NHWC upsample
// (its input is a channels-last view), an add of an NHWC and an NCHW tensor that falls
// off the vectorised path, and a scatter-style upsample backward: ~1 ms per step.  Here:
//   forward:  block = (64 output columns, one output row, 32 channels, image); the two
//             source rows' needed tokens are staged in LDS (64-B channel runs, coalesced),
//             outputs written along x (coalesced NCHW).  up is rounded to the dtype before
//             the add, as the unfused graph does.
//   backward: block = (32 source columns, one source row, 32 channels, image); the output
//             rows/columns whose bilinear taps reach them are staged from dL/dout and
//             every source element is a fixed-order gather (no atomics), written once,
//             token-major.
// Source index: ATen area_pixel_compute_source_index (align_corners=False):
// s = (in/out) * (dst + 0.5) - 0.5, clamped at 0; i1 = min(i0 + 1, in - 1).
#include "common.h"

namespace vs {
namespace {

constexpr int kCB = 32;    // channels per block

__device__ __forceinline__ void up_index(int dst, int in, int out, int& i0, int& i1, float& l0, float& l1) {
  const float scale = (float)in / (float)out;
  float s = scale * ((float)dst + 0.5f) - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = (int)s;
  i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  l1 = s - (float)i0;
  l0 = 1.f - l1;
}

// grid (ceil(W / 64), H, B * C / 32), 256 threads
template <typename T>
__global__ void __launch_bounds__(256) upsample_add_fwd_kernel(const T* __restrict__ cur, const T* __restrict__ src,
                                                               T* __restrict__ out, int C, int H, int W, int Hs,
                                                               int Ws, long long src_bstride) {
  constexpr int kMaxCols = 2 * 64 + 4;        // source columns a 64-wide output tile can touch (scale <= 2)
  __shared__ float sS[2][kMaxCols][kCB + 1];
  const int x0 = blockIdx.x * 64, y = blockIdx.y;
  const int cb = blockIdx.z % (C / kCB), b = blockIdx.z / (C / kCB);
  const int c0 = cb * kCB;
  int ya, yb, xa_, xb_;
  float ly0, ly1, lxa, lxb;
  up_index(y, Hs, H, ya, yb, ly0, ly1);
  up_index(x0, Ws, W, xa_, xb_, lxa, lxb);
  const int xlast = min(W, x0 + 64) - 1;
  int xl0, xl1;
  up_index(xlast, Ws, W, xl0, xl1, lxa, lxb);
  const int sx0 = xa_, ncols = xl1 - sx0 + 1;  // source columns [sx0, xl1]
  const T* sb = src + (size_t)b * src_bstride + c0;
  for (int i = threadIdx.x; i < 2 * ncols * kCB; i += 256) {
    const int c = i % kCB, col = (i / kCB) % ncols, r = i / (kCB * ncols);
    const int sy = r ? yb : ya;
    sS[r][col][c] = to_f32(sb[((size_t)sy * Ws + sx0 + col) * C + c]);
  }
  __syncthreads();
  const int xi = threadIdx.x & 63;
  const int x = x0 + xi;
  if (x >= W) return;
  int xs0, xs1;
  float lx0, lx1;
  up_index(x, Ws, W, xs0, xs1, lx0, lx1);
  xs0 -= sx0;
  xs1 -= sx0;
  for (int c = threadIdx.x >> 6; c < kCB; c += 4) {
    const float up = ly0 * (lx0 * sS[0][xs0][c] + lx1 * sS[0][xs1][c]) +
                     ly1 * (lx0 * sS[1][xs0][c] + lx1 * sS[1][xs1][c]);
    const size_t o = (((size_t)b * C + c0 + c) * H + y) * W + x;
    out[o] = from_f32<T>(to_f32(cur[o]) + to_f32(from_f32<T>(up)));
  }
}

// grid (ceil(Ws / 32), Hs, B * C / 32), 256 threads; dsrc [B, Hs*Ws, C] contiguous
template <typename T>
__global__ void __launch_bounds__(256) upsample_bwd_kernel(const T* __restrict__ dout, T* __restrict__ dsrc, int C,
                                                           int H, int W, int Hs, int Ws) {
  constexpr int kMaxRows = 5, kMaxCols = 72;   // output rows (nonzero weight) / columns reaching a source row / 32 columns (scale <= 2)
  __shared__ float sD[kMaxRows][kMaxCols][kCB + 1];     // [row][column][channel]: lanes = channels
  __shared__ float sWy[kMaxRows];
  __shared__ int sRow[kMaxRows];
  const int sx0 = blockIdx.x * 32, sy = blockIdx.y;
  const int cb = blockIdx.z % (C / kCB), b = blockIdx.z / (C / kCB);
  const int c0 = cb * kCB;
  // output rows whose taps touch source row sy (scan a conservative window)
  const float sc_y = (float)H / (float)Hs;
  const int ylo = max(0, (int)floorf((sy - 1) * sc_y) - 2), yhi = min(H - 1, (int)ceilf((sy + 2) * sc_y) + 2);
  if (threadIdx.x == 0) {
    int n = 0;
    for (int y = ylo; y <= yhi && n < kMaxRows; ++y) {
      int y0, y1;
      float l0, l1;
      up_index(y, Hs, H, y0, y1, l0, l1);
      const float w = (y0 == sy ? l0 : 0.f) + (y1 == sy ? l1 : 0.f);
      if (w != 0.f) {
        sRow[n] = y;
        sWy[n] = w;
        ++n;
      }
    }
    for (int k = n; k < kMaxRows; ++k) {
      sRow[k] = -1;
      sWy[k] = 0.f;
    }
  }
  // output columns reaching source columns [sx0, sx0 + 32)
  const float sc_x = (float)W / (float)Ws;
  const int xlo = max(0, (int)floorf((sx0 - 1) * sc_x) - 2);
  const int xhi = min(W - 1, min(xlo + kMaxCols - 1, (int)ceilf((sx0 + 33) * sc_x) + 2));
  const int ncols = xhi - xlo + 1;
  __syncthreads();
  int nr = 0;
  while (nr < kMaxRows && sRow[nr] >= 0) ++nr;
  // stage the valid rows only; 4 consecutive columns per thread
  const int nq = (ncols + 3) >> 2;
  for (int i = threadIdx.x; i < kCB * nr * nq; i += 256) {
    const int xq = i % nq, r = (i / nq) % nr, c = i / (nq * nr);
    const T* row = dout + (((size_t)b * C + c0 + c) * H + sRow[r]) * W + xlo;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int xx = 4 * xq + k;
      if (xx < ncols) sD[r][xx][c] = to_f32(row[xx]);
    }
  }
  __syncthreads();
  const int c = threadIdx.x & 31;
  for (int sxi = threadIdx.x >> 5; sxi < 32; sxi += 8) {
    const int sx = sx0 + sxi;
    if (sx >= Ws) break;
    float acc = 0.f;
    // only the few output columns whose taps can reach sx (~2 per unit of scale)
    const int xb = max(xlo, (int)floorf((sx - 1) * sc_x) - 1);
    const int xe = min(xhi, (int)ceilf((sx + 2) * sc_x) + 1);
    for (int x = xb; x <= xe; ++x) {
      int x0_, x1_;
      float l0, l1;
      up_index(x, Ws, W, x0_, x1_, l0, l1);
      const float wx = (x0_ == sx ? l0 : 0.f) + (x1_ == sx ? l1 : 0.f);
      if (wx != 0.f) {
        float col = 0.f;
        for (int r = 0; r < nr; ++r) col += sWy[r] * sD[r][x - xlo][c];
        acc += wx * col;
      }
    }
    dsrc[((size_t)b * Hs * Ws + (size_t)sy * Ws + sx) * C + c0 + c] = from_f32<T>(acc);
  }
}

// Backward for the exact 2x case (H = 2 Hs, W = 2 Ws: the 1024^2 pixel decoder), separable:
// block = (32 channels, 4 source rows, 32 source columns, image).  Pass 1 (vertical): a
// thread takes (channel, source row, 8 output columns) and reads the <= 4 output rows
// whose taps reach the source row as 16-B vectors (NCHW rows are contiguous along x),
// weighting them by the row adjoint; the 8 column sums go to LDS.  Pass 2 (horizontal):
// (source column, channel) per thread, the <= 4 output columns' sums weighted by the
// column adjoint, written token-major (channel runs contiguous).  Weights come from the
// forward's source-index rule (up_index), boundaries included.  ~1.2x the bytes of dL/dout
// read (halo columns), none re-read from HBM.
constexpr int kR2 = 4, kC2 = 32, kX2 = 80;   // source rows / columns per block, staged output columns

__device__ __forceinline__ float adj_w(int y, int s, int in, int out) {
  int i0, i1;
  float l0, l1;
  up_index(y, in, out, i0, i1, l0, l1);
  return (i0 == s ? l0 : 0.f) + (i1 == s ? l1 : 0.f);
}

template <typename T>
__global__ void __launch_bounds__(256) upsample_bwd2x_kernel(const T* __restrict__ dout, T* __restrict__ dsrc, int C,
                                                             int H, int W, int Hs, int Ws) {
  __shared__ float sV[kCB][kR2][kX2 + 1];
  const int sx0 = blockIdx.x * kC2, sy0 = blockIdx.y * kR2;
  const int cb = blockIdx.z % (C / kCB), b = blockIdx.z / (C / kCB);
  const int c0 = cb * kCB;
  const int xbase = 2 * sx0 - 8;             // first staged output column (16-B aligned: W % 8 == 0)
  // pass 1: items (c, r, chunk of 8 columns) = 32 x 4 x 10
  for (int it = threadIdx.x; it < kCB * kR2 * (kX2 / 8); it += 256) {
    const int ch = it % (kX2 / 8), r = (it / (kX2 / 8)) % kR2, c = it / ((kX2 / 8) * kR2);
    const int sy = sy0 + r, x = xbase + 8 * ch;
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    if (sy < Hs && x >= 0 && x < W) {
      const T* plane = dout + ((size_t)b * C + c0 + c) * H * W;
#pragma unroll
      for (int dy = -1; dy <= 2; ++dy) {
        const int y = 2 * sy + dy;
        if (y < 0 || y >= H) continue;
        const float w = adj_w(y, sy, Hs, H);
        if (w == 0.f) continue;
        float v[8];
        Vec16<T>::load(plane + (size_t)y * W + x, v);
        if (Vec16<T>::N == 4) Vec16<T>::load(plane + (size_t)y * W + x + 4, v + 4);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += w * v[k];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) sV[c][r][8 * ch + k] = acc[k];
  }
  __syncthreads();
  // pass 2: items (r, source column, channel) = 4 x 32 x 32, channel fastest
  for (int it = threadIdx.x; it < kR2 * kC2 * kCB; it += 256) {
    const int c = it % kCB, sxi = (it / kCB) % kC2, r = it / (kCB * kC2);
    const int sy = sy0 + r, sx = sx0 + sxi;
    if (sy >= Hs || sx >= Ws) continue;
    float acc = 0.f;
#pragma unroll
    for (int dx = -1; dx <= 2; ++dx) {
      const int x = 2 * sx + dx;
      if (x < 0 || x >= W) continue;
      acc += adj_w(x, sx, Ws, W) * sV[c][r][x - xbase];
    }
    dsrc[((size_t)b * Hs * Ws + (size_t)sy * Ws + sx) * C + c0 + c] = from_f32<T>(acc);
  }
}

// Channels-last variants (the pixel decoder's NHWC 1/4-resolution tail: cur / out / dout
// are [B, H, W, C], src / dsrc token-major [B, Hs*Ws, C]).  A thread owns 16 bytes of
// channels of one pixel: the forward reads the four source tokens' runs (L2-resident:
// neighbouring outputs share them) and writes out coalesced; the backward gathers, for one
// source token, the <= 4 x 4 output pixels whose taps reach it (adjoint weights from the
// forward's index rule, boundaries included), fixed order, written once.
template <typename T>
__global__ void __launch_bounds__(256) upsample_add_nhwc_kernel(const T* __restrict__ cur, const T* __restrict__ src,
                                                                T* __restrict__ out, int C, int H, int W, int Hs,
                                                                int Ws, long long src_bstride, long long nvec) {
  constexpr int V = Vec16<T>::N;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= nvec) return;
  const int cv = C / V;
  const int c = (int)(idx % cv) * V;
  const long long pix = idx / cv;
  const int x = (int)(pix % W);
  const long long by = pix / W;
  const int y = (int)(by % H), b = (int)(by / H);
  int y0, y1, x0, x1;
  float ly0, ly1, lx0, lx1;
  up_index(y, Hs, H, y0, y1, ly0, ly1);
  up_index(x, Ws, W, x0, x1, lx0, lx1);
  const T* sb = src + (size_t)b * src_bstride + c;
  float s00[V], s01[V], s10[V], s11[V], cv_[V], o[V];
  Vec16<T>::load(sb + ((size_t)y0 * Ws + x0) * C, s00);
  Vec16<T>::load(sb + ((size_t)y0 * Ws + x1) * C, s01);
  Vec16<T>::load(sb + ((size_t)y1 * Ws + x0) * C, s10);
  Vec16<T>::load(sb + ((size_t)y1 * Ws + x1) * C, s11);
  Vec16<T>::load(cur + pix * C + c, cv_);
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const float up = ly0 * (lx0 * s00[k] + lx1 * s01[k]) + ly1 * (lx0 * s10[k] + lx1 * s11[k]);
    o[k] = cv_[k] + to_f32(from_f32<T>(up));
  }
  Vec16<T>::store(out + pix * C + c, o);
}

template <typename T>
__global__ void __launch_bounds__(256) upsample_bwd_nhwc_kernel(const T* __restrict__ dout, T* __restrict__ dsrc, int C,
                                                                int H, int W, int Hs, int Ws, long long nvec) {
  constexpr int V = Vec16<T>::N, kMax = 8;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= nvec) return;
  const int cv = C / V;
  const int c = (int)(idx % cv) * V;
  const long long sp = idx / cv;
  const int sx = (int)(sp % Ws);
  const long long bsy = sp / Ws;
  const int sy = (int)(bsy % Hs), b = (int)(bsy / Hs);
  const float scy = (float)H / (float)Hs, scx = (float)W / (float)Ws;
  const int ylo = max(0, (int)floorf(scy * (sy - 0.5f) - 0.5f) - 1);
  const int yhi = min(H - 1, min(ylo + kMax - 1, (int)ceilf(scy * (sy + 1.5f) - 0.5f) + 1));
  const int xlo = max(0, (int)floorf(scx * (sx - 0.5f) - 0.5f) - 1);
  const int xhi = min(W - 1, min(xlo + kMax - 1, (int)ceilf(scx * (sx + 1.5f) - 0.5f) + 1));
  float wx[kMax];
#pragma unroll
  for (int k = 0; k < kMax; ++k) wx[k] = (xlo + k <= xhi) ? adj_w(xlo + k, sx, Ws, W) : 0.f;
  float acc[V];
#pragma unroll
  for (int k = 0; k < V; ++k) acc[k] = 0.f;
  const T* base = dout + (size_t)b * H * W * C + c;
  for (int y = ylo; y <= yhi; ++y) {
    const float wy = adj_w(y, sy, Hs, H);
    if (wy == 0.f) continue;
    float row[V];
#pragma unroll
    for (int k = 0; k < V; ++k) row[k] = 0.f;
#pragma unroll
    for (int j = 0; j < kMax; ++j) {
      if (wx[j] == 0.f) continue;
      float v[V];
      Vec16<T>::load(base + ((size_t)y * W + xlo + j) * C, v);
#pragma unroll
      for (int k = 0; k < V; ++k) row[k] += wx[j] * v[k];
    }
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] += wy * row[k];
  }
  Vec16<T>::store(dsrc + sp * C + c, acc);
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" int vs_upsample_add_forward(int dtype, const void* cur, const void* src, void* out, int B, int C, int H,
                                       int W, int Hs, int Ws, long long src_batch_stride, void* stream) {
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");
  VS_CHECK(B > 0 && C > 0 && C % kCB == 0 && H > 0 && W > 0 && Hs > 0 && Ws > 0, "bad sizes (C % 32 == 0)");
  VS_CHECK(Hs <= H && Ws <= W && 2 * Hs >= H && 2 * Ws >= W, "upsampling factor must lie in [1, 2]");
  VS_CHECK(cur && src && out, "null pointer");
  dim3 grid((W + 63) / 64, H, B * (C / kCB));
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VS_BF16)
    hipLaunchKernelGGL(upsample_add_fwd_kernel<bf16>, grid, dim3(256), 0, st, (const bf16*)cur, (const bf16*)src,
                       (bf16*)out, C, H, W, Hs, Ws, src_batch_stride);
  else
    hipLaunchKernelGGL(upsample_add_fwd_kernel<float>, grid, dim3(256), 0, st, (const float*)cur, (const float*)src,
                       (float*)out, C, H, W, Hs, Ws, src_batch_stride);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_upsample_backward(int dtype, const void* grad_out, void* grad_src, int B, int C, int H, int W,
                                    int Hs, int Ws, void* stream) {
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");
  VS_CHECK(B > 0 && C > 0 && C % kCB == 0 && H > 0 && W > 0 && Hs > 0 && Ws > 0, "bad sizes (C % 32 == 0)");
  VS_CHECK(Hs <= H && Ws <= W && 2 * Hs >= H && 2 * Ws >= W, "upsampling factor must lie in [1, 2]");
  VS_CHECK(grad_out && grad_src, "null pointer");
  hipStream_t st = (hipStream_t)stream;
  if (H == 2 * Hs && W == 2 * Ws && W % 8 == 0) {
    dim3 g2((Ws + kC2 - 1) / kC2, (Hs + kR2 - 1) / kR2, B * (C / kCB));
    if (dtype == VS_BF16)
      hipLaunchKernelGGL(upsample_bwd2x_kernel<bf16>, g2, dim3(256), 0, st, (const bf16*)grad_out, (bf16*)grad_src,
                         C, H, W, Hs, Ws);
    else
      hipLaunchKernelGGL(upsample_bwd2x_kernel<float>, g2, dim3(256), 0, st, (const float*)grad_out,
                         (float*)grad_src, C, H, W, Hs, Ws);
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
  dim3 grid((Ws + 31) / 32, Hs, B * (C / kCB));
  if (dtype == VS_BF16)
    hipLaunchKernelGGL(upsample_bwd_kernel<bf16>, grid, dim3(256), 0, st, (const bf16*)grad_out, (bf16*)grad_src, C,
                       H, W, Hs, Ws);
  else
    hipLaunchKernelGGL(upsample_bwd_kernel<float>, grid, dim3(256), 0, st, (const float*)grad_out, (float*)grad_src,
                       C, H, W, Hs, Ws);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_upsample_add_forward_nhwc(int dtype, const void* cur, const void* src, void* out, int B, int C,
                                            int H, int W, int Hs, int Ws, long long src_batch_stride, void* stream) {
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");
  VS_CHECK(B > 0 && C > 0 && C % 8 == 0 && H > 0 && W > 0 && Hs > 0 && Ws > 0, "bad sizes (C % 8 == 0)");
  VS_CHECK(Hs <= H && Ws <= W && 2 * Hs >= H && 2 * Ws >= W, "upsampling factor must lie in [1, 2]");
  VS_CHECK(cur && src && out, "null pointer");
  VS_CHECK(((uintptr_t)cur & 15) == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
               src_batch_stride % 8 == 0,
           "16-B aligned operands");
  const int V = dtype == VS_BF16 ? 8 : 4;
  const long long nvec = (long long)B * H * W * (C / V);
  const dim3 g((unsigned)((nvec + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VS_BF16)
    hipLaunchKernelGGL(upsample_add_nhwc_kernel<bf16>, g, dim3(256), 0, st, (const bf16*)cur, (const bf16*)src,
                       (bf16*)out, C, H, W, Hs, Ws, src_batch_stride, nvec);
  else
    hipLaunchKernelGGL(upsample_add_nhwc_kernel<float>, g, dim3(256), 0, st, (const float*)cur, (const float*)src,
                       (float*)out, C, H, W, Hs, Ws, src_batch_stride, nvec);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_upsample_backward_nhwc(int dtype, const void* grad_out, void* grad_src, int B, int C, int H, int W,
                                         int Hs, int Ws, void* stream) {
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");
  VS_CHECK(B > 0 && C > 0 && C % 8 == 0 && H > 0 && W > 0 && Hs > 0 && Ws > 0, "bad sizes (C % 8 == 0)");
  VS_CHECK(Hs <= H && Ws <= W && 2 * Hs >= H && 2 * Ws >= W, "upsampling factor must lie in [1, 2]");
  VS_CHECK(grad_out && grad_src, "null pointer");
  VS_CHECK(((uintptr_t)grad_out & 15) == 0 && ((uintptr_t)grad_src & 15) == 0, "16-B aligned operands");
  const int V = dtype == VS_BF16 ? 8 : 4;
  const long long nvec = (long long)B * Hs * Ws * (C / V);
  const dim3 g((unsigned)((nvec + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VS_BF16)
    hipLaunchKernelGGL(upsample_bwd_nhwc_kernel<bf16>, g, dim3(256), 0, st, (const bf16*)grad_out, (bf16*)grad_src,
                       C, H, W, Hs, Ws, nvec);
  else
    hipLaunchKernelGGL(upsample_bwd_nhwc_kernel<float>, g, dim3(256), 0, st, (const float*)grad_out,
                       (float*)grad_src, C, H, W, Hs, Ws, nvec);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
