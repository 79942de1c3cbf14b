// 3 x 3 convolution, stride 1, padding 1, no dilation, on channels-last (NHWC) bf16
// planes: the pixel decoder's output conv (HF:m2f:1394-1419, `output_convs` of the FPN's
// 1/4-resolution level: Conv2d(256, 256, 3, padding=1, bias=False) + GroupNorm(32) + ReLU).
//
// MIOpen ran this conv (C2: 4 x 256 x 256 x 256, 309 GFLOP per direction) as NHWC kernels
// wrapped in 8-9 NCHW <-> NHWC transposes, ~1.5 ms a step.  Here the planes stay NHWC
// (the token-major layout of the rest of the decoder) and the three products are
// hand-written for the bf16 MFMA:
//
// * forward and input gradient: implicit GEMM on the token-GEMM skeleton (token_gemm.hip):
//   Y[p, o] = sum_{tap, i} X[p + d(tap), i] Wt[o, tap, i] with M = pixels, N = Co,
//   K = 9 Ci.  A K-step (64 channels of one tap) stages, per output pixel, the 128 bytes of
//   its tap neighbour by LDS-DMA; a neighbour outside the image takes its bytes from a zero
//   row in global memory, so padding costs nothing.  The input gradient is the same product
//   of dY with the spatially flipped, transposed weights (Wb[i, tap', o] = W[o, i, 8 - tap']:
//   dX[p] = sum dY[p - d(tap)] W[tap] = sum dY[p + d(tap')] Wb[tap']).
// * weight gradient: dW[o, i, tap] = sum_p dY[p, o] X[p + d(tap), i], a product over pixels
//   (the strided dimension of both operands): a workgroup owns 128 o x 128 i for the three
//   taps of one kernel row and streams 64-pixel row segments; the dY segment and the 66
//   input pixels under it (+-1 column) are staged by LDS-DMA in their natural [pixel]
//   [channel] layout and read as MFMA operands with the transposed read ds_read_b64_tr_b16,
//   the three horizontal taps as row offsets 0, 1, 2 of the same staged input image.  The
//   pixels are split over S workgroups per output block; their f32 partial blocks are
//   summed in a fixed order by a second kernel that writes the torch [Co, Ci, 3, 3] layout.
#include <stdlib.h>

#include "lds_dma.h"

namespace vs {
namespace {

constexpr int kRowB = 128;   // bytes of a row per K-step (implicit GEMM)

// physical byte offset of (row, 16-B chunk) in an implicit-GEMM staged tile (128-B rows)
__device__ __forceinline__ int tile_off(int row, int chunk) { return row * kRowB + ((chunk ^ ((row >> 1) & 7)) << 4); }

// ---------------------------------------------------------------------------------------
// forward / input gradient: Y[M, N] = sum_{tap, c} X[nbr(p, tap), c] Wt[n, tap, c]
// Tile GM x GN waves of TM x TN 32 x 32 MFMA tiles (pixels x output channels), as the token
// GEMM: <2, 4, 4, 2> = 256 x 256 (512 threads, 128 KB of staging, 1 workgroup / CU).
template <int GM, int GN, int TM, int TN>
__global__ void __launch_bounds__(64 * GM * GN) conv3x3_igemm_kernel(const bf16* __restrict__ X,
                                                                     const bf16* __restrict__ Wt,
                                                                     const bf16* __restrict__ bias,
                                                                     bf16* __restrict__ Y, int M, int H, int Wd,
                                                                     int Ci, int N) {
  constexpr int BM = GM * TM * 32, BN = GN * TN * 32, NW = GM * GN, NT = 64 * NW;
  constexpr int XB = BM * kRowB, WB = BN * kRowB, STB = XB + WB;
  constexpr int NI = (BM + BN) / 8 / NW;               // DMA instructions per wave per K-step
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * STB];
  const int CC = Ci / 64;                              // K-steps per tap
  const int nks = 9 * CC;
  const int rowB = 9 * Ci * 2;                         // bytes of a weight row
  const int tilesM = (M + BM - 1) / BM, tilesN = (N + BN - 1) / BN;
  const int wg = xcd_swizzle(blockIdx.x, tilesM * tilesN);
  const int tm = wg / tilesN, tn = wg - tm * tilesN;
  const int m0 = tm * BM, n0 = tn * BN;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int wm = w % GM, wn = w / GM;
  const int HW = H * Wd;

  // the output pixel of every X row this lane stages (-1: past M), with its (h, w)
  int xm[NI], xh[NI], xw[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int row = (w * NI + j) * 8 + (l >> 3);
    const int m = m0 + row;
    xm[j] = (row < BM && m < M) ? m : -1;
    const int hw = xm[j] >= 0 ? m % HW : 0;
    xh[j] = hw / Wd;
    xw[j] = hw - xh[j] * Wd;
  }

  auto issue = [&](int ks, int st) {
    unsigned char* base = smem + st * STB;
    const int tap = ks / CC, cc = ks - tap * CC;
    const int ty = tap / 3, dy = ty - 1, dx = tap - 3 * ty - 1;
    const int shift = dy * Wd + dx;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int blk = w * NI + j;
      const int row = blk * 8 + (l >> 3);
      const bool isx = row < BM;
      const int rr = isx ? row : row - BM;
      const int chunk = (l & 7) ^ ((rr >> 1) & 7);
      const unsigned char* src;
      if (isx) {
        const bool ok = xm[j] >= 0 && (unsigned)(xh[j] + dy) < (unsigned)H && (unsigned)(xw[j] + dx) < (unsigned)Wd;
        src = ok ? reinterpret_cast<const unsigned char*>(X + ((size_t)(xm[j] + shift) * Ci + cc * 64)) + chunk * 16
                 : g_dma_zero_row + chunk * 16;
      } else {
        src = reinterpret_cast<const unsigned char*>(Wt) + (size_t)min(n0 + rr, N - 1) * rowB + ks * kRowB + chunk * 16;
      }
      glds16(src, base + blk * 1024);
    }
  };

  f32x16_t acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) zero16(acc[a][b]);
  auto xrow = [&](int t) { return wm * TM * 32 + t * 32 + r; };
  auto wrow = [&](int t) { return wn * TN * 32 + t * 32 + r; };

  issue(0, 0);
  for (int ks = 0; ks < nks; ++ks) {
    const int st = ks & 1;
    wait_vm<0>();
    raw_barrier();
    if (ks + 1 < nks) issue(ks + 1, st ^ 1);
    const unsigned char* sx = smem + st * STB;
    const unsigned char* sw = sx + XB;
    bf16x8_t xa[2][TM], wa[2][TN];
    auto load = [&](int kk, int bsel) {
#pragma unroll
      for (int t = 0; t < TM; ++t) xa[bsel][t] = *reinterpret_cast<const bf16x8_t*>(sx + tile_off(xrow(t), 2 * kk + hh));
#pragma unroll
      for (int t = 0; t < TN; ++t) wa[bsel][t] = *reinterpret_cast<const bf16x8_t*>(sw + tile_off(wrow(t), 2 * kk + hh));
    };
    load(0, 0);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (kk + 1 < 4) load(kk + 1, (kk + 1) & 1);
      const int bs = kk & 1;
#pragma unroll
      for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TM; ++b) acc[a][b] = mfma16(wa[bs][a], xa[bs][b], acc[a][b]);
    }
  }

  // epilogue through LDS (the token GEMM's): 16-B stores of whole row segments
  constexpr int NCK = BN / 8;
  auto so_off = [](int row, int chunk) { return row * (BN * 2) + ((chunk ^ (row & 15)) << 4); };
  raw_barrier();
#pragma unroll
  for (int b = 0; b < TM; ++b) {
    const int row = xrow(b);
#pragma unroll
    for (int a = 0; a < TN; ++a) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int f = wn * TN * 32 + a * 32 + 8 * g + 4 * hh, n = n0 + f;
        const bf16x4_t bv = (bias && n < N) ? *reinterpret_cast<const bf16x4_t*>(bias + n) : bf16x4_t{0, 0, 0, 0};
        bf16x4_t o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = bf16_bits(acc[a][b][4 * g + e] + bf16_bits_to_f32((unsigned short)bv[e]));
        *reinterpret_cast<bf16x4_t*>(smem + so_off(row, f >> 3) + (f & 7) * 2) = o;
      }
    }
  }
  raw_barrier();
  for (int idx = threadIdx.x; idx < BM * NCK; idx += NT) {
    const int row = idx / NCK, chunk = idx - (idx / NCK) * NCK;
    const int m = m0 + row, n = n0 + chunk * 8;
    if (m < M && n < N)
      *reinterpret_cast<uint4*>(Y + (size_t)m * N + n) = *reinterpret_cast<const uint4*>(smem + so_off(row, chunk));
  }
}

// ---------------------------------------------------------------------------------------
// weight gradient
constexpr int kSeg = 64;                       // pixels per row segment
constexpr int kWBlk = 128;                     // output / input channels per workgroup
constexpr int kXRows = 68;                     // staged input pixels: the segment +- 1 (66), whole 1-KB DMA blocks
constexpr int kDyBytes = kSeg * 256, kXBytes = kXRows * 256, kStage = kDyBytes + kXBytes;
constexpr int kDyBlk = kDyBytes / 1024, kXBlk = kXBytes / 1024;   // 16 + 17 DMA blocks
constexpr int kWStages = 4;                   // ring of segment buffers: 3 segments in flight (132 KB)

// grid: S x tiles workgroups (tiles = Co/128 x Ci/128 x 3 kernel rows), 512 threads;
// part [S][Co][9][Ci] f32
__global__ void __launch_bounds__(512) conv3x3_wgrad_kernel(const bf16* __restrict__ dY, const bf16* __restrict__ X,
                                                            float* __restrict__ part, int B, int H, int Wd, int Ci,
                                                            int Co, int S) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[kWStages * kStage];
  const int cib_n = Ci / kWBlk;
  const int tiles = (Co / kWBlk) * cib_n * 3;
  const int wg = xcd_swizzle(blockIdx.x, S * tiles);
  const int s = wg / tiles, tile = wg - s * tiles;    // a split's tiles are neighbours (same XCD, same pixels)
  const int ky = tile % 3, cib = (tile / 3) % cib_n, cob = tile / (3 * cib_n);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int co_w = (w & 1) * 64, ci_w = (w >> 1) * 32;  // this wave: 64 o x 32 i, three taps
  const int cpr = (Wd + kSeg - 1) / kSeg;               // segments per image row
  const long long nseg = (long long)B * H * cpr;
  const long long sb = nseg * s / S, se = nseg * (s + 1) / S;

  auto issue = [&](long long sg, int st) {
    unsigned char* base = smem + st * kStage;
    const long long rowid = sg / cpr;                  // b * H + h
    const int w0 = (int)(sg - rowid * cpr) * kSeg;
    const int h = (int)(rowid % H);
    const bool xrow_ok = (unsigned)(h + ky - 1) < (unsigned)H;
    const long long xpix0 = (rowid + ky - 1) * Wd;     // first pixel of the input row (same image when ok)
    for (int blk = w; blk < kDyBlk + kXBlk; blk += 8) {
      const unsigned char* src;
      if (blk < kDyBlk) {
        const int row = blk * 4 + (l >> 4), ch = (l & 15) ^ img_swz(row);
        const int x = w0 + row;
        src = x < Wd ? reinterpret_cast<const unsigned char*>(dY + ((size_t)(rowid * Wd + x) * Co + cob * kWBlk)) + ch * 16
                     : g_dma_zero_row + ch * 16;
      } else {
        const int row = (blk - kDyBlk) * 4 + (l >> 4), ch = (l & 15) ^ img_swz(row);
        const int x = w0 - 1 + row;
        const bool ok = xrow_ok && row < kSeg + 2 && (unsigned)x < (unsigned)Wd;
        src = ok ? reinterpret_cast<const unsigned char*>(X + ((size_t)(xpix0 + x) * Ci + cib * kWBlk)) + ch * 16
                 : g_dma_zero_row + ch * 16;
      }
      glds16(src, base + blk * 1024);
    }
  };

  f32x16_t acc[3][2];
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) zero16(acc[a][b]);
  // wave 0 issues 5 DMA blocks per segment (33 = 4 x 8 + 1), the others 4: the counted waits
  // retire exactly the oldest segment
#pragma unroll
  for (int j = 0; j < kWStages - 1; ++j)
    if (sb + j < se) issue(sb + j, j);
  int st = 0;
  for (long long sg = sb; sg < se; ++sg) {
    if (sg + kWStages - 2 < se) {
      if (w == 0)
        wait_vm<5 * (kWStages - 2)>();
      else
        wait_vm<4 * (kWStages - 2)>();
    } else {
      wait_vm<0>();
    }
    raw_barrier();                                    // segment sg landed everywhere; sg - 1 consumed
    if (sg + kWStages - 1 < se) issue(sg + kWStages - 1, st == 0 ? kWStages - 1 : st - 1);
    const unsigned char* sd = smem + st * kStage;
    const unsigned char* sx = sd + kDyBytes;
    st = st == kWStages - 1 ? 0 : st + 1;
    // operands of 16-pixel step k from asm transposed reads (lds_dma.h), one step ahead
    bf16x8_t a[2][3], b[2][2];
    auto load = [&](int k, int p) {
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) a[p][kx] = tr_frag_asm(sx, 16 * k + kx, ci_w, l);   // X^T: rows i, k = pixel
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) b[p][ct] = tr_frag_asm(sd, 16 * k, co_w + 32 * ct, l);   // dY: cols o
    };
    constexpr int RD = 10;                            // ds_read_tr per step
    load(0, 0);
#pragma unroll
    for (int k = 0; k < kSeg / 16; ++k) {
      const int p = k & 1;
      if (k + 1 < kSeg / 16) {
        load(k + 1, p ^ 1);
        lgkm_wait<RD>(a[p][0]);
      } else {
        lgkm_wait<0>(a[p][0]);
      }
      lgkm_wait<RD>(a[p][1]);
      lgkm_wait<RD>(a[p][2]);
      lgkm_wait<RD>(b[p][0]);
      lgkm_wait<RD>(b[p][1]);
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) acc[kx][ct] = mfma16(a[p][kx], b[p][ct], acc[kx][ct]);
    }
  }
  // partials in FRAGMENT order, whole 1-KB stores (token_wgrad.hip's layout): the
  // workgroup's 128 o x 128 i x 3 taps block is [wave][kx][ct][g][lane][4 registers]
  float* pw = part + ((size_t)s * tiles + tile) * (3 * kWBlk * kWBlk) + (size_t)w * 6144 + l * 4;
#pragma unroll
  for (int kx = 0; kx < 3; ++kx)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(pw + ((kx * 2 + ct) * 4 + g) * 256) =
            make_float4(acc[kx][ct][4 * g], acc[kx][ct][4 * g + 1], acc[kx][ct][4 * g + 2], acc[kx][ct][4 * g + 3]);
}

// dW[o, i, tap] (torch [Co, Ci, 3, 3]) = sum over splits of the fragment-order partials,
// fixed order.  A thread owns (o, tap, 4 consecutive i) -- one float4 of one lane per split;
// consecutive threads take consecutive o (consecutive lanes).  A 256-thread block = 64 items x
// 4 split groups (g, g + 4, ...), the group sums added in LDS in group order.
template <typename T>
__global__ void __launch_bounds__(256) conv3x3_wgrad_reduce_kernel(const float* __restrict__ part, T* __restrict__ dw,
                                                                   int Ci, int Co, int S) {
  __shared__ float4 sp[4][64];
  const int it = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const long long q = (long long)blockIdx.x * 64 + it;    // (tap, i / 4, o), o fastest
  const long long nq = (long long)Co * 9 * (Ci / 4);
  const bool live = q < nq;
  const long long qq = live ? q : 0;
  const int o = (int)(qq % Co);
  const long long rest = qq / Co;
  const int i = (int)(rest % (Ci / 4)) * 4, tap = (int)(rest / (Ci / 4));
  const int cib_n = Ci / kWBlk, tiles = (Co / kWBlk) * cib_n * 3;
  const int ky = tap / 3, kx = tap - 3 * ky;
  const int cob = o / kWBlk, cib = i / kWBlk, oo = o % kWBlk, ii = i % kWBlk;
  const int tile = (cob * cib_n + cib) * 3 + ky;
  const int w = (ii >> 5) * 2 + (oo >> 6), ct = (oo & 63) >> 5, r = oo & 31;
  const int row = ii & 31, g = row >> 3, hh = (row >> 2) & 1;
  const size_t stride = (size_t)tiles * 3 * kWBlk * kWBlk;
  const float* p = part + (size_t)tile * (3 * kWBlk * kWBlk) + (size_t)w * 6144 + ((kx * 2 + ct) * 4 + g) * 256 +
                   (hh * 32 + r) * 4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (live) {
    int s = grp;
    for (; s + 4 < S; s += 8) {
      const float4 v0 = *reinterpret_cast<const float4*>(p + s * stride);
      const float4 v1 = *reinterpret_cast<const float4*>(p + (s + 4) * stride);
      a.x += v0.x; a.y += v0.y; a.z += v0.z; a.w += v0.w;
      a.x += v1.x; a.y += v1.y; a.z += v1.z; a.w += v1.w;
    }
    for (; s < S; s += 4) {
      const float4 v = *reinterpret_cast<const float4*>(p + s * stride);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  sp[grp][it] = a;
  __syncthreads();
  if (grp == 0 && live) {
    const float4 b = sp[1][it], c = sp[2][it], d = sp[3][it];
    T* dd = dw + ((size_t)o * Ci + i) * 9 + tap;
    dd[0] = from_f32<T>(((a.x + b.x) + c.x) + d.x);
    dd[9] = from_f32<T>(((a.y + b.y) + c.y) + d.y);
    dd[18] = from_f32<T>(((a.z + b.z) + c.z) + d.z);
    dd[27] = from_f32<T>(((a.w + b.w) + c.w) + d.w);
  }
}

// w [Co, Ci, 3, 3] -> wf [Co, 3, 3, Ci] (forward) and wb [Ci, 3, 3, Co] flipped (input gradient)
__global__ void __launch_bounds__(256) conv3x3_weight_layouts_kernel(const bf16* __restrict__ w, bf16* __restrict__ wf,
                                                                     bf16* __restrict__ wb, int Co, int Ci) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= Co * Ci * 9) return;
  const int tap = idx % 9, i = (idx / 9) % Ci, o = idx / (9 * Ci);
  const bf16 v = w[idx];
  if (wf) wf[((size_t)o * 9 + tap) * Ci + i] = v;
  if (wb) wb[((size_t)i * 9 + (8 - tap)) * Co + o] = v;
}

int wgrad_splits(int B, int H, int Wd, int Ci, int Co) {
  const long long tiles = (long long)(Co / kWBlk) * (Ci / kWBlk) * 3;
  const long long nseg = (long long)B * H * ((Wd + kSeg - 1) / kSeg);
  long long S = 256 / tiles;                                      // one workgroup per CU (196 VGPRs: 8 waves)
  if (S > nseg) S = nseg;
  if (S < 1) S = 1;
  return (int)S;
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" int vs_conv3x3_forward(const void* x, const void* wt, const void* bias, void* y, int B, int H, int W, int Ci,
                                  int Co, void* stream) {
  VS_CHECK(x && wt && y, "null pointer");
  VS_CHECK(B > 0 && H > 0 && W > 0, "empty image");
  VS_CHECK(Ci > 0 && Ci % 64 == 0 && Co > 0 && Co % 8 == 0, "Ci % 64 == 0 and Co % 8 == 0");
  VS_CHECK((long long)B * H * W < (1ll << 31) && (long long)B * H * W * (Ci > Co ? Ci : Co) < (1ll << 40), "too large");
  VS_CHECK(((uintptr_t)x & 15) == 0 && ((uintptr_t)wt & 15) == 0 && ((uintptr_t)y & 15) == 0 &&
               (!bias || ((uintptr_t)bias & 7) == 0),
           "x / wt / y must be 16-B aligned, bias 8-B");
  const int M = B * H * W;
  const bool big = Co >= 256 && (long long)((M + 255) / 256) * ((Co + 255) / 256) >= 256;
  const int bm = big ? 256 : 128;
  const long long tiles = (long long)((M + bm - 1) / bm) * ((Co + bm - 1) / bm);
  hipStream_t st = (hipStream_t)stream;
  if (big)
    hipLaunchKernelGGL((conv3x3_igemm_kernel<2, 4, 4, 2>), dim3((unsigned)tiles), dim3(512), 0, st, (const bf16*)x,
                       (const bf16*)wt, (const bf16*)bias, (bf16*)y, M, H, W, Ci, Co);
  else
    hipLaunchKernelGGL((conv3x3_igemm_kernel<2, 2, 2, 2>), dim3((unsigned)tiles), dim3(256), 0, st, (const bf16*)x,
                       (const bf16*)wt, (const bf16*)bias, (bf16*)y, M, H, W, Ci, Co);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_conv3x3_weight_layouts(const void* w, void* w_fwd, void* w_bwd, int Co, int Ci, void* stream) {
  VS_CHECK(w && (w_fwd || w_bwd), "null pointer");
  VS_CHECK(Co > 0 && Ci > 0, "empty weight");
  const int n = Co * Ci * 9;
  hipLaunchKernelGGL(conv3x3_weight_layouts_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)w, (bf16*)w_fwd, (bf16*)w_bwd, Co, Ci);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" long long vs_conv3x3_wgrad_workspace_bytes(int B, int H, int W, int Ci, int Co) {
  if (B <= 0 || H <= 0 || W <= 0 || Ci % kWBlk || Co % kWBlk || Ci <= 0 || Co <= 0) return 0;
  return (long long)wgrad_splits(B, H, W, Ci, Co) * Co * 9 * Ci * 4;
}

extern "C" int vs_conv3x3_wgrad(int dtype, const void* dy, const void* x, void* dw, void* workspace, int B, int H,
                                int W, int Ci, int Co, void* stream) {
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype (of dw) must be VS_F32 or VS_BF16");
  VS_CHECK(dy && x && dw && workspace, "null pointer");
  VS_CHECK(B > 0 && H > 0 && W > 0, "empty image");
  VS_CHECK(Ci % kWBlk == 0 && Co % kWBlk == 0 && Ci > 0 && Co > 0, "Ci and Co must be multiples of 128");
  VS_CHECK((long long)B * H * W < (1ll << 31), "too large");
  VS_CHECK(((uintptr_t)dy & 15) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)workspace & 15) == 0,
           "dy / x / workspace must be 16-B aligned");
  const int S = wgrad_splits(B, H, W, Ci, Co);
  const int tiles = (Co / kWBlk) * (Ci / kWBlk) * 3;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(conv3x3_wgrad_kernel, dim3((unsigned)(S * tiles)), dim3(512), 0, st, (const bf16*)dy,
                     (const bf16*)x, (float*)workspace, B, H, W, Ci, Co, S);
  VS_LAUNCH_CHECK();
  const long long nq = (long long)Co * 9 * (Ci / 4);
  const dim3 g((unsigned)((nq + 63) / 64));
  if (dtype == VS_BF16)
    hipLaunchKernelGGL(conv3x3_wgrad_reduce_kernel<bf16>, g, dim3(256), 0, st, (const float*)workspace, (bf16*)dw, Ci,
                       Co, S);
  else
    hipLaunchKernelGGL(conv3x3_wgrad_reduce_kernel<float>, g, dim3(256), 0, st, (const float*)workspace, (float*)dw,
                       Ci, Co, S);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
