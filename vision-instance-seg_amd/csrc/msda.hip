// Multi-scale deformable attention sampling (MSDeformAttn), forward + backward.
//
// Semantics: upstream MSDeformAttn CUDA extension (ms_deform_attn_im2col_bilinear /
// col2im), oracle HF:m2f:798-837.  Layout: value [B,S,H,32], loc [B,Q,H,L,P,2] f32,
// attn [B,Q,H,L,P] f32, out [B,Q,H*32].
//
// Forward (HBM/L2 gather-bound): a "group" = one (b, q, head).  Each lane owns one
// 16-byte slice of the 32 head channels (8 bf16 or 4 f32), so a group is 4 (bf16) or
// 8 (f32) lanes and one wave serves 16 (bf16) / 8 (f32) groups.  Every corner tap is
// one 16-B load per lane, adjacent lanes read adjacent bytes; the group's loc/attn
// rows (96 B / 48 B, 16-B aligned) are read as float4.  Accumulation in f32.
//
// Backward: grad_value (f32, then cast) by f32 global atomics, bound by their rate (~1.1 TB/s
// of added bytes on gfx950, MI355X_MICROARCH §Global float atomics), so the kernels cut the
// added bytes; grad_loc / grad_attn ride in the same walk (or a gather kernel,
// msda_bwd_geom_kernel, for the f32 / small paths):
//   * bf16, P == 4, encoder problems (queries = the value grid; default):
//     msda_bwd_col_kernel -- a workgroup owns a PYRAMID COLUMN (8 x 16 finest-level queries
//     plus the coarser levels' blocks over the same area), grad_value per band of cells as
//     one MFMA product W[cell][query] x grad_out[query][c] accumulated over the column's
//     query chunks, one atomic row per (band, cell) for the whole column;
//   * bf16, P == 4, query subsets (Q != S): msda_bwd_mfma_wg_kernel -- the same product per
//     8 x 8 query tile (runs of 64 queries) and level, one atomic row per touched cell;
//   * f32 (parity mode): msda_bwd_binned_kernel -- 4 x 4 tiles, the tile's corners
//     counting-sorted by cell, register sums in exact f32, one atomic row per cell
//     (also bf16 with VS_MSDA_MFMA=0, for A/B and the cross-check test);
//   * small problems / other P (VS_MSDA_RUN=0 forces it): one fused kernel
//     (msda_bwd_kernel, an atomic per corner).
// vs_msda_backward_tiled is the deterministic, atomic-free variant (grad_value by
// destination tile, written once in the value dtype; ops VS_MSDA_BWD=tiled).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "common.h"
#include "mfma_util.h"

namespace vs {
namespace {

constexpr int kD = 32;
constexpr int kMaxLevels = 4;

struct Levels {
  int h[kMaxLevels];
  int w[kMaxLevels];
  int start[kMaxLevels];
};

// pyramid columns (column backward, column-ordered forward): see col_geo
constexpr int kMsdaColDefault[2] = {8, 16};  // VS_MSDA_COL default (CY, CX); {0, 0}: tile kernel

struct ColGeo {
  int ty[kMaxLevels], tx[kMaxLevels];    // a column's query block per level (rows, cols)
  int ord[kMaxLevels];                   // levels in enumeration order (largest first)
  int ncx, per_image;                    // columns per block row / per image
};


// ---- tap geometry shared by every backward kernel (the same fp32 floor/frac math as the
// forward: a tap's corners and weights are identical everywhere).

struct Tap {
  int h0, w0;
  float lh, lw, hh, hw;
  bool inside;
};

__device__ __forceinline__ Tap tap_geom(float x, float y, int Hl, int Wl) {
  Tap t;
  const float him = __fmaf_rn(y, (float)Hl, -0.5f);
  const float wim = __fmaf_rn(x, (float)Wl, -0.5f);
  t.inside = him > -1.f && wim > -1.f && him < (float)Hl && wim < (float)Wl;
  const float fh0 = floorf(him), fw0 = floorf(wim);
  t.h0 = (int)fh0;
  t.w0 = (int)fw0;
  t.lh = him - fh0;
  t.lw = wim - fw0;
  t.hh = 1.f - t.lh;
  t.hw = 1.f - t.lw;
  return t;
}

template <typename T>
__global__ void __launch_bounds__(256) msda_fwd_kernel(const T* __restrict__ value,
                                                        const float* __restrict__ loc,
                                                        const float* __restrict__ attw,
                                                        T* __restrict__ out, Levels lv, int S,
                                                        int Hh, int Q, int L, int P,
                                                        long long groups) {
  constexpr int V = Vec16<T>::N;       // channels per lane
  constexpr int LPG = kD / V;          // lanes per group
  long long gid = (long long)xcd_swizzle(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  long long stride = (long long)gridDim.x * blockDim.x;
  const int LP = L * P;
  for (; gid < groups * LPG; gid += stride) {
    const long long grp = gid / LPG;
    const int sub = (int)(gid % LPG);
    const int h = (int)(grp % Hh);
    const long long b = grp / Hh / Q;
    const float* lp = loc + grp * LP * 2;
    const float* wp = attw + grp * LP;
    const size_t rowstride = (size_t)Hh * kD;  // elements between spatial positions
    const T* vb = value + ((size_t)b * S * Hh + h) * kD + sub * V;
    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
    for (int l = 0; l < L; ++l) {
      const int Hl = lv.h[l], Wl = lv.w[l];
      const T* vl = vb + (size_t)lv.start[l] * rowstride;
      const float fH = (float)Hl, fW = (float)Wl;
      for (int p = 0; p < P; ++p) {
        const float x = lp[(l * P + p) * 2 + 0];
        const float y = lp[(l * P + p) * 2 + 1];
        const float a = wp[l * P + p];
        const float him = y * fH - 0.5f;
        const float wim = x * fW - 0.5f;
        if (him > -1.f && wim > -1.f && him < fH && wim < fW) {
          const float fh0 = floorf(him), fw0 = floorf(wim);
          const int h0 = (int)fh0, w0 = (int)fw0;
          const float lh = him - fh0, lw = wim - fw0;
          const float hh = 1.f - lh, hw = 1.f - lw;
          const float cw[4] = {hh * hw, hh * lw, lh * hw, lh * lw};
          const bool ok[4] = {h0 >= 0 && w0 >= 0, h0 >= 0 && w0 + 1 <= Wl - 1,
                              h0 + 1 <= Hl - 1 && w0 >= 0, h0 + 1 <= Hl - 1 && w0 + 1 <= Wl - 1};
          const int off[4] = {h0 * Wl + w0, h0 * Wl + w0 + 1, (h0 + 1) * Wl + w0,
                              (h0 + 1) * Wl + w0 + 1};
          float val[V];
#pragma unroll
          for (int i = 0; i < V; ++i) val[i] = 0.f;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            if (ok[c]) {
              float t[V];
              Vec16<T>::load(vl + (size_t)off[c] * rowstride, t);
#pragma unroll
              for (int i = 0; i < V; ++i) val[i] += cw[c] * t[i];
            }
          }
#pragma unroll
          for (int i = 0; i < V; ++i) acc[i] += a * val[i];
        }
      }
    }
    Vec16<T>::store(out + grp * kD + sub * V, acc);
  }
}

// bf16, P == 4, L levels known at compile time (the production shapes): a level's 4
// sampling locations and weights arrive as three 16-B loads (the rows are 16-B aligned:
// 32 L and 16 L bytes per group) and the corner rows of two taps at a time are loaded raw
// (4 VGPRs each) before any is used, so 8 issue back to back instead of one tap's 4
// (msda_fwd_kernel's runtime-P loop).  Same arithmetic, same order.  T = 4 (a level's 16
// corner rows in flight) measured slower: 0.167 vs 0.156 ms at the C2 encoder shape.  Round 6:
// T = 1 (4 corner rows in flight, 84 VGPRs, 5 waves / SIMD) ties T = 2 (116 VGPRs, 4 waves /
// SIMD) in the C2 step, 0.142 vs 0.140 ms per launch (profiles/r6_msda_fwd_t_ab.txt), so T = 2
// stays; T = 2 forced to 5 waves spilled (0.295 ms).
//
// COL (encoder problems, queries = the value grid, round 6): the queries are visited in
// PYRAMID-COLUMN order (ColGeo, as the column backward: a column = an 8 x 16 block of the
// finest level and the blocks over the same image area at the coarser levels, slots padded
// to the block sizes), columns in raster order, and the blocks of consecutive columns on one
// XCD (xcd_swizzle).  In query order an XCD working on the coarse levels' queries gathered
// from the whole image at the finer levels (8 MB of level-0 value per image against a 4 MB
// L2): PMC reads were 1.63x the compulsory bytes.  Visiting order only: every query is
// computed exactly as before.  `cq` = slots per column, `ncol` = columns per image.
template <int L, int T, bool COL = false>
__global__ void __launch_bounds__(256) msda_fwd4_kernel(const bf16* __restrict__ value,
                                                         const float* __restrict__ loc,
                                                         const float* __restrict__ attw,
                                                         bf16* __restrict__ out, Levels lv, int S,
                                                         int Hh, int Q, long long groups, ColGeo cg, int cq) {
  constexpr int P = 4, LP = L * P, V = 8, LPG = kD / V;
  long long gid = (long long)xcd_swizzle(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  long long stride = (long long)gridDim.x * blockDim.x;
  for (; gid < groups * LPG; gid += stride) {
    long long grp = gid / LPG;
    const int sub = (int)(gid % LPG);
    const int h = (int)(grp % Hh);
    long long b = grp / Hh / Q;
    if (COL) {                                // grp = ((b * ncol + col) * cq + slot) * Hh + h
      const unsigned t = (unsigned)(grp / Hh);
      unsigned k = t % (unsigned)cq;
      const unsigned cgl = t / (unsigned)cq;
      const unsigned col = cgl % (unsigned)cg.per_image;
      b = cgl / (unsigned)cg.per_image;
      const int cyy = (int)(col / (unsigned)cg.ncx), cxx = (int)(col % (unsigned)cg.ncx);
      int q = -1;
#pragma unroll
      for (int i = 0; i < L; ++i) {
        const int l = cg.ord[i];
        const unsigned n = (unsigned)(cg.ty[l] * cg.tx[l]);
        if (k < n) {
          const int y = cyy * cg.ty[l] + (int)(k / (unsigned)cg.tx[l]), x = cxx * cg.tx[l] + (int)(k % (unsigned)cg.tx[l]);
          if (y < lv.h[l] && x < lv.w[l]) q = lv.start[l] + y * lv.w[l] + x;
          break;
        }
        k -= n;
      }
      if (q < 0) continue;                    // a padding slot of a border column
      grp = (b * Q + q) * Hh + h;
    }
    const float4* lp = reinterpret_cast<const float4*>(loc + grp * LP * 2);
    const float4* wp = reinterpret_cast<const float4*>(attw + grp * LP);
    const size_t rowstride = (size_t)Hh * kD;
    const bf16* vb = value + ((size_t)b * S * Hh + h) * kD + sub * V;
    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
#pragma unroll 1
    for (int l = 0; l < L; ++l) {
      const int Hl = lv.h[l], Wl = lv.w[l];
      const bf16* vl = vb + (size_t)lv.start[l] * rowstride;
      const float fH = (float)Hl, fW = (float)Wl;
      const float4 w4 = wp[l];
      const float4 lq0 = lp[2 * l], lq1 = lp[2 * l + 1];
      const float xa[4] = {lq0.x, lq0.z, lq1.x, lq1.z}, ya[4] = {lq0.y, lq0.w, lq1.y, lq1.w};
      const float aa[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll 1
      for (int hf = 0; hf < P / T; ++hf) {    // T taps (4T corner rows) in flight at a time
        float xs[T], ys[T], as[T];
#pragma unroll
        for (int p = 0; p < T; ++p) {          // select chain: keeps the loop rolled (VGPRs)
          xs[p] = xa[p];
          ys[p] = ya[p];
          as[p] = aa[p];
#pragma unroll
          for (int h = 1; h < P / T; ++h)
            if (hf == h) {
              xs[p] = xa[h * T + p];
              ys[p] = ya[h * T + p];
              as[p] = aa[h * T + p];
            }
        }
        uint4 raw[T][4];
        float cw[T][4];
#pragma unroll
        for (int p = 0; p < T; ++p) {
          const float him = ys[p] * fH - 0.5f;
          const float wim = xs[p] * fW - 0.5f;
          const bool in = him > -1.f && wim > -1.f && him < fH && wim < fW;
          const float fh0 = floorf(him), fw0 = floorf(wim);
          const int h0 = (int)fh0, w0 = (int)fw0;
          const float lh = him - fh0, lw = wim - fw0;
          const float hh = 1.f - lh, hw = 1.f - lw;
          cw[p][0] = in ? hh * hw : 0.f;        // a tap outside adds nothing (NaN-safe)
          cw[p][1] = in ? hh * lw : 0.f;
          cw[p][2] = in ? lh * hw : 0.f;
          cw[p][3] = in ? lh * lw : 0.f;
          const bool ok[4] = {in && h0 >= 0 && w0 >= 0, in && h0 >= 0 && w0 + 1 <= Wl - 1,
                              in && h0 + 1 <= Hl - 1 && w0 >= 0, in && h0 + 1 <= Hl - 1 && w0 + 1 <= Wl - 1};
          const int off[4] = {h0 * Wl + w0, h0 * Wl + w0 + 1, (h0 + 1) * Wl + w0, (h0 + 1) * Wl + w0 + 1};
#pragma unroll
          for (int c = 0; c < 4; ++c)
            raw[p][c] = ok[c] ? *reinterpret_cast<const uint4*>(vl + (size_t)off[c] * rowstride)
                              : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int p = 0; p < T; ++p) {
          float val[V];
#pragma unroll
          for (int i = 0; i < V; ++i) val[i] = 0.f;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const unsigned wd[4] = {raw[p][c].x, raw[p][c].y, raw[p][c].z, raw[p][c].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              val[2 * j] += cw[p][c] * __uint_as_float(wd[j] << 16);
              val[2 * j + 1] += cw[p][c] * __uint_as_float(wd[j] & 0xffff0000u);
            }
          }
#pragma unroll
          for (int i = 0; i < V; ++i) acc[i] += as[p] * val[i];
        }
      }
    }
    Vec16<bf16>::store(out + grp * kD + sub * V, acc);
  }
}


template <typename T>
__global__ void __launch_bounds__(256) msda_bwd_kernel(
    const T* __restrict__ value, const float* __restrict__ loc, const float* __restrict__ attw,
    const T* __restrict__ gout, float* __restrict__ gvalue, float* __restrict__ gloc,
    float* __restrict__ gattw, Levels lv, int S, int Hh, int Q, int L, int P, long long groups) {
  // lane = channel, 32 lanes per (b, q, head); every corner is one f32 atomic add
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long grp = gid >> 5;
  const int c = (int)(gid & 31);
  if (grp >= groups) return;  // uniform per 32-lane half-wave
  const int LP = L * P;
  const int h = (int)(grp % Hh);
  const long long bq = grp / Hh;
  const long long b = bq / Q;
  const float* lp = loc + grp * LP * 2;
  const float* wp = attw + grp * LP;
  const size_t rowstride = (size_t)Hh * kD;
  const size_t vbase = ((size_t)b * S * Hh + h) * kD + c;
  const float g = to_f32(gout[grp * kD + c]);
  for (int l = 0; l < L; ++l) {
    const int Hl = lv.h[l], Wl = lv.w[l];
    const size_t lbase = vbase + (size_t)lv.start[l] * rowstride;
    const float fH = (float)Hl, fW = (float)Wl;
    for (int p = 0; p < P; ++p) {
      const int tap = l * P + p;
      const float a = wp[tap];
      const Tap t = tap_geom(lp[tap * 2 + 0], lp[tap * 2 + 1], Hl, Wl);
      float r_w = 0.f, r_x = 0.f, r_y = 0.f;
      if (t.inside) {
        const int h0 = t.h0, w0 = t.w0;
        const float lh = t.lh, lw = t.lw, hh = t.hh, hw = t.hw;
        const float ga = g * a;
        float v1 = 0.f, v2 = 0.f, v3 = 0.f, v4 = 0.f;
        if (h0 >= 0 && w0 >= 0) {
          const size_t o = lbase + (size_t)(h0 * Wl + w0) * rowstride;
          v1 = to_f32(value[o]);
          atomicAdd(gvalue + o, hh * hw * ga);
        }
        if (h0 >= 0 && w0 + 1 <= Wl - 1) {
          const size_t o = lbase + (size_t)(h0 * Wl + w0 + 1) * rowstride;
          v2 = to_f32(value[o]);
          atomicAdd(gvalue + o, hh * lw * ga);
        }
        if (h0 + 1 <= Hl - 1 && w0 >= 0) {
          const size_t o = lbase + (size_t)((h0 + 1) * Wl + w0) * rowstride;
          v3 = to_f32(value[o]);
          atomicAdd(gvalue + o, lh * hw * ga);
        }
        if (h0 + 1 <= Hl - 1 && w0 + 1 <= Wl - 1) {
          const size_t o = lbase + (size_t)((h0 + 1) * Wl + w0 + 1) * rowstride;
          v4 = to_f32(value[o]);
          atomicAdd(gvalue + o, lh * lw * ga);
        }
        const float val = hh * hw * v1 + hh * lw * v2 + lh * hw * v3 + lh * lw * v4;
        r_w = g * val;
        const float dh = -hw * v1 - lw * v2 + hw * v3 + lw * v4;   // d val / d him
        const float dw = -hh * v1 + hh * v2 - lh * v3 + lh * v4;   // d val / d wim
        r_x = fW * ga * dw;
        r_y = fH * ga * dh;
      }
#pragma unroll
      for (int s = 16; s >= 1; s >>= 1) {
        r_w += __shfl_xor(r_w, s, 32);
        r_x += __shfl_xor(r_x, s, 32);
        r_y += __shfl_xor(r_y, s, 32);
      }
      if (c == 0) {
        gattw[grp * LP + tap] = r_w;
        gloc[(grp * LP + tap) * 2 + 0] = r_x;
        gloc[(grp * LP + tap) * 2 + 1] = r_y;
      }
    }
  }
}

// msda_bwd_geom_kernel — grad_attn / grad_loc of the split backward.  Gather-only, laid
// out like the forward (a lane owns a 16-B channel slice, 4 (bf16) / 8 (f32) lanes per
// (b, q, head)), partial dot products reduced over the group's lanes with shuffles.
template <typename T>
__global__ void __launch_bounds__(256) msda_bwd_geom_kernel(
    const T* __restrict__ value, const float* __restrict__ loc, const float* __restrict__ attw,
    const T* __restrict__ gout, float* __restrict__ gloc, float* __restrict__ gattw, Levels lv, int S,
    int Hh, int Q, int L, int P, long long groups) {
  constexpr int V = Vec16<T>::N;       // channels per lane
  constexpr int LPG = kD / V;          // lanes per group (4 bf16, 8 f32), a power of two
  constexpr int kGroups = 256 / LPG;   // groups per workgroup (consecutive)
  constexpr int kMaxLP = 16;
  __shared__ float s_w[kGroups * kMaxLP], s_xy[kGroups * kMaxLP * 2];
  const long long blk = xcd_swizzle(blockIdx.x, gridDim.x);
  const long long gid = blk * blockDim.x + threadIdx.x;
  const long long grp0 = blk * kGroups;
  const long long grp = gid / LPG;
  const int sub = (int)(gid % LPG);
  const int LP = L * P;
  const bool staged = LP <= kMaxLP;    // outputs staged in LDS and written coalesced
  if (grp < groups) {
  const int h = (int)(grp % Hh);
  const long long b = grp / Hh / Q;
  const float* lp = loc + grp * LP * 2;
  const float* wp = attw + grp * LP;
  const size_t rowstride = (size_t)Hh * kD;
  const T* vb = value + ((size_t)b * S * Hh + h) * kD + sub * V;
  float g[V];
  Vec16<T>::load(gout + grp * kD + sub * V, g);
  for (int l = 0; l < L; ++l) {
    const int Hl = lv.h[l], Wl = lv.w[l];
    const T* vl = vb + (size_t)lv.start[l] * rowstride;
    const float fH = (float)Hl, fW = (float)Wl;
    for (int p = 0; p < P; ++p) {
      const int t = l * P + p;
      const float a = wp[t];
      const Tap tg = tap_geom(lp[t * 2 + 0], lp[t * 2 + 1], Hl, Wl);
      float r_w = 0.f, r_x = 0.f, r_y = 0.f;
      if (tg.inside) {
        const int h0 = tg.h0, w0 = tg.w0;
        const bool ok[4] = {h0 >= 0 && w0 >= 0, h0 >= 0 && w0 + 1 <= Wl - 1, h0 + 1 <= Hl - 1 && w0 >= 0,
                            h0 + 1 <= Hl - 1 && w0 + 1 <= Wl - 1};
        const int off[4] = {h0 * Wl + w0, h0 * Wl + w0 + 1, (h0 + 1) * Wl + w0, (h0 + 1) * Wl + w0 + 1};
        float d[4];                     // sum_c g[c] * value[corner][c] over this lane's slice
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          d[k] = 0.f;
          if (ok[k]) {
            float v[V];
            Vec16<T>::load(vl + (size_t)off[k] * rowstride, v);
#pragma unroll
            for (int i = 0; i < V; ++i) d[k] += g[i] * v[i];
          }
        }
        const float lh = tg.lh, lw = tg.lw, hh = tg.hh, hw = tg.hw;
        r_w = hh * hw * d[0] + hh * lw * d[1] + lh * hw * d[2] + lh * lw * d[3];
        r_x = fW * a * (-hh * d[0] + hh * d[1] - lh * d[2] + lh * d[3]);
        r_y = fH * a * (-hw * d[0] - lw * d[1] + hw * d[2] + lw * d[3]);
      }
#pragma unroll
      for (int s = LPG / 2; s >= 1; s >>= 1) {
        r_w += __shfl_xor(r_w, s, LPG);
        r_x += __shfl_xor(r_x, s, LPG);
        r_y += __shfl_xor(r_y, s, LPG);
      }
      if (sub == 0) {
        if (staged) {
          const int gl = (int)(grp - grp0);
          s_w[gl * LP + t] = r_w;
          s_xy[(gl * LP + t) * 2 + 0] = r_x;
          s_xy[(gl * LP + t) * 2 + 1] = r_y;
        } else {
          gattw[grp * LP + t] = r_w;
          gloc[(grp * LP + t) * 2 + 0] = r_x;
          gloc[(grp * LP + t) * 2 + 1] = r_y;
        }
      }
    }
  }
  }
  if (staged) {
    __syncthreads();
    const int ng = (int)min((long long)kGroups, groups - grp0);
    for (int i = threadIdx.x; i < ng * LP; i += 256) gattw[grp0 * LP + i] = s_w[i];
    for (int i = threadIdx.x; i < ng * LP * 2; i += 256) gloc[grp0 * LP * 2 + i] = s_xy[i];
  }
}

constexpr int kSplitMin = 16 * 8192;    // (b, q, head) groups from which the split backward pays

// ---------------------------------------------------------------------------------
// Exclusive prefix scan of per-tile counts (1024-entry blocks + a block prefix), used by
// the destination-tile backward below.
constexpr int kScanBlock = 1024;

__global__ void __launch_bounds__(256) sort_scan_local_kernel(const int* __restrict__ count, int* __restrict__ local,
                                                              int* __restrict__ bsum, long long n) {
  __shared__ int sw[4];
  const long long base = (long long)blockIdx.x * kScanBlock + threadIdx.x * 4;
  int v[4], s = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = base + k < n ? count[base + k] : 0;
    s += v[k];
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int incl = s;                                   // inclusive scan of s over the wave
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) sw[wave] = incl;
  __syncthreads();
  int wpre = 0;
  for (int w = 0; w < wave; ++w) wpre += sw[w];
  int run = wpre + incl - s;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (base + k < n) local[base + k] = run;
    run += v[k];
  }
  if (threadIdx.x == 255) bsum[blockIdx.x] = wpre + incl;
}

// exclusive scan of the block totals (one workgroup, any count); bprefix[nb] = total
__global__ void __launch_bounds__(1024) sort_scan_blocks_kernel(const int* __restrict__ bsum, int* __restrict__ bprefix,
                                                                int nb) {
  __shared__ int sw[16];
  __shared__ int carry;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < nb; base += 1024) {
    const int i = base + threadIdx.x;
    const int s = i < nb ? bsum[i] : 0;
    int incl = s;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane == 63) sw[wave] = incl;
    __syncthreads();
    int wpre = 0;
    for (int w = 0; w < wave; ++w) wpre += sw[w];
    const int c0 = carry;
    if (i < nb) bprefix[i] = c0 + wpre + incl - s;
    __syncthreads();
    if (threadIdx.x == 1023) carry = c0 + wpre + incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) bprefix[nb] = carry;
}

// one group of LPG lanes per key (grad_value row of one head), V channels per lane
// ---------------------------------------------------------------------------------
// grad_value by destination TILES, without float atomics (default backward).
//
// gfx950 measurement (tools/micro/lds_atomic_bench.hip): LDS float atomics (ds_add_f32)
// retire ~0.33 lane-ops/clk/CU -- slower than global f32 atomics (~1.1 TB/s of added
// bytes) and ~18x slower than a plain LDS read-modify-write -- which is why every earlier
// LDS-atomic variant (bands, destination tiles) lost to the global-atomic carry scatter.
// This path has ONE wave own each destination tile, so its accumulation is plain LDS
// read-modify-write:
//   count:  per tap (natural order), the distinct tiles its valid corners fall in (1, 2
//           or 4) -> count[tile] += 1, one atomic per distinct tile per wave (ballot)
//   scan:   offset(tile) = exclusive prefix of count (the sort_scan kernels)
//   fill:   records[offset(tile) + rank] = q * P + p   (4 B; geometry is recomputed)
//   accum:  one wave per tile: per record, lanes = 2 corner rows x 32 channels add
//           w * attw * grad_out[q, h, c] into the tile's te x te x 32 f32 LDS block
//           (rows (y, y+1) land in opposite LDS bank halves), then every cell of the
//           tile is written once, in the value dtype.  No memset, no float atomics.
// A tile is (image, head, level, te x te cells), te chosen per level so that tiles carry
// about the same number of taps (te = 8 / 4 / 2 for ~5 / 21 / 84 taps per cell).
constexpr int kTileMaxEdge = 8;

struct TileGeo {
  int sh[kMaxLevels];     // log2(te) per level
  int ntx[kMaxLevels];    // tiles per row
  int nty[kMaxLevels];    // tile rows
  int base[kMaxLevels + 1];
  int per_bh;             // tiles per (image, head)
};

// distinct tiles of a tap's valid corners, -1 padded (the tap must be inside)
__device__ __forceinline__ void tap_tiles(const TileGeo& tg, int l, const Tap& t, int Hl, int Wl, int* id) {
  const int sh = tg.sh[l];
  const int ya = t.h0 >= 0 ? t.h0 : t.h0 + 1, yb = t.h0 + 1 <= Hl - 1 ? t.h0 + 1 : t.h0;
  const int xa = t.w0 >= 0 ? t.w0 : t.w0 + 1, xb = t.w0 + 1 <= Wl - 1 ? t.w0 + 1 : t.w0;
  const int ty0 = ya >> sh, ty1 = yb >> sh, tx0 = xa >> sh, tx1 = xb >> sh;
  const int nx = tg.ntx[l], b0 = tg.base[l];
  id[0] = b0 + ty0 * nx + tx0;
  id[1] = tx1 != tx0 ? b0 + ty0 * nx + tx1 : -1;
  id[2] = ty1 != ty0 ? b0 + ty1 * nx + tx0 : -1;
  id[3] = (ty1 != ty0 && tx1 != tx0) ? b0 + ty1 * nx + tx1 : -1;
}

// ctr[id] += 1 for every lane with id >= 0, one atomic per distinct id of the wave;
// returns this lane's slot (value before its own increment).  Wave-uniform call.
__device__ __forceinline__ int wave_agg_inc(int* ctr, int id) {
  const int lane = threadIdx.x & 63;
  unsigned long long pend = __ballot(id >= 0);
  int mine = 0;
  while (pend) {
    const int leader = __ffsll((long long)pend) - 1;
    const int lid = __shfl(id, leader, 64);
    const unsigned long long m = __ballot(id == lid) & pend;
    int base = 0;
    if (lane == leader) base = atomicAdd(ctr + lid, (int)__popcll(m));
    base = __shfl(base, leader, 64);
    if ((m >> lane) & 1ull) mine = base + (int)__popcll(m & ((1ull << lane) - 1ull));
    pend &= ~m;
  }
  return mine;
}

// FILL = false: count;  FILL = true: write records.  One thread per tap, natural order.
template <bool FILL>
__global__ void __launch_bounds__(256) msda_tile_bucket_kernel(const float* __restrict__ loc, int* __restrict__ ctr,
                                                               const int* __restrict__ local,
                                                               const int* __restrict__ bprefix, int* __restrict__ rec,
                                                               Levels lv, TileGeo tg, int Hh, int Q, int L, int P,
                                                               long long taps) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  int id[4] = {-1, -1, -1, -1};
  int q = 0, lp = 0;
  if (i < taps) {
    const int LP = L * P;
    lp = (int)(i % LP);
    const long long grp = i / LP;
    const int h = (int)(grp % Hh);
    const long long bq = grp / Hh;
    q = (int)(bq % Q);
    const long long b = bq / Q;
    const int l = lp / P;
    const int Hl = lv.h[l], Wl = lv.w[l];
    const float2 xy = reinterpret_cast<const float2*>(loc)[i];
    const Tap t = tap_geom(xy.x, xy.y, Hl, Wl);
    if (t.inside) {
      tap_tiles(tg, l, t, Hl, Wl, id);
      const int off = (int)((b * Hh + h) * tg.per_bh);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (id[k] >= 0) id[k] += off;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int slot = wave_agg_inc(ctr, id[k]);
    if (FILL && id[k] >= 0) rec[local[id[k]] + bprefix[id[k] / kScanBlock] + slot] = q * P + (lp % P);
  }
}

// one wave per tile (4 tiles per workgroup); grad_value written in the value dtype.
// Records are taken 64 at a time: lane j loads record j's tap (loc, attw) and its
// grad_out row (64 B of bf16 / 128 B of f32) into LDS, so every global load of the chunk
// is in flight at once; the accumulation then walks the chunk with the tap geometry read
// by v_readlane (wave-uniform) and grad_out from LDS.
template <typename T>
__global__ void __launch_bounds__(256) msda_tile_accum_kernel(const float* __restrict__ loc,
                                                              const float* __restrict__ attw,
                                                              const T* __restrict__ gout, const int* __restrict__ local,
                                                              const int* __restrict__ bprefix,
                                                              const int* __restrict__ rec, T* __restrict__ gvalue,
                                                              Levels lv, TileGeo tg, int S, int Hh, int Q, int L, int P,
                                                              int ntiles) {
  constexpr int kCells = kTileMaxEdge * (kTileMaxEdge + 1);
  __shared__ __attribute__((aligned(16))) float sAcc[4][kCells * kD];
  __shared__ __attribute__((aligned(16))) float sG[4][64 * (kD + 1)];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, half = lane >> 5, c = lane & 31;
  const int tile = blockIdx.x * 4 + wave;
  if (tile >= ntiles) return;                      // wave-uniform; no block barriers below
  const int bh = tile / tg.per_bh, lt = tile % tg.per_bh;
  const int h = bh % Hh, b = bh / Hh;
  int l = 0;
  while (l + 1 < L && lt >= tg.base[l + 1]) ++l;
  const int tl = lt - tg.base[l];
  const int sh = tg.sh[l], te = 1 << sh, tp = te + 1;
  const int ty0 = (tl / tg.ntx[l]) << sh, tx0 = (tl % tg.ntx[l]) << sh;
  const int Hl = lv.h[l], Wl = lv.w[l];
  float* acc = sAcc[wave];
  float* sg = sG[wave];
  for (int k = lane; k < te * tp * kD; k += 64) acc[k] = 0.f;
  const int r0 = local[tile] + bprefix[tile / kScanBlock];
  const int r1 = tile + 1 < ntiles ? local[tile + 1] + bprefix[(tile + 1) / kScanBlock]
                                  : bprefix[(ntiles - 1) / kScanBlock + 1];
  const int LP = L * P;
  const long long gbase = (long long)b * Q * Hh + h;    // (b, q=0, h) group index
  for (int r = r0; r < r1; r += 64) {
    const int n = min(64, r1 - r);
    // ---- lane j: record r + j -> tap geometry (registers) and grad_out row (LDS)
    int h0 = -(1 << 20), w0 = -(1 << 20);
    float lh = 0.f, lw = 0.f, a = 0.f;
    if (lane < n) {
      const int e = rec[r + lane];
      const int q = e / P, p = e - q * P;
      const long long grp = gbase + (long long)q * Hh;
      const long long ti = grp * LP + l * P + p;
      const float2 xy = reinterpret_cast<const float2*>(loc)[ti];
      a = attw[ti];
      const Tap t = tap_geom(xy.x, xy.y, Hl, Wl);
      h0 = t.h0;
      w0 = t.w0;
      lh = t.lh;
      lw = t.lw;
      const T* grow = gout + grp * kD;
      constexpr int V = Vec16<T>::N;
      float gv[kD];
#pragma unroll
      for (int k = 0; k < kD; k += V) Vec16<T>::load(grow + k, gv + k);
#pragma unroll
      for (int k = 0; k < kD; ++k) sg[lane * (kD + 1) + k] = gv[k] * a;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- walk the chunk: half 0 adds corner row h0, half 1 row h0 + 1 (distinct rows)
    for (int j = 0; j < n; ++j) {
      const int jh0 = __builtin_amdgcn_readlane(h0, j), jw0 = __builtin_amdgcn_readlane(w0, j);
      const float jlh = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lh), j));
      const float jlw = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lw), j));
      const int y = jh0 + half;
      const int ly = y - ty0, lx = jw0 - tx0;
      if (ly >= 0 && ly < te && y < Hl) {
        const float gw = sg[j * (kD + 1) + c] * (half ? jlh : 1.f - jlh);
        float* row = acc + (ly * tp) * kD + c;
        if (lx >= 0 && lx < te && jw0 >= 0) row[lx * kD] += gw * (1.f - jlw);
        if (lx + 1 < te && lx + 1 >= 0 && jw0 + 1 < Wl) row[(lx + 1) * kD] += gw * jlw;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  const size_t rowstride = (size_t)Hh * kD;
  T* gb = gvalue + (((size_t)b * S + lv.start[l]) * Hh + h) * kD + c;
  for (int cell = half; cell < te * te; cell += 2) {
    const int y = cell >> sh, x = cell & (te - 1);
    if (ty0 + y < Hl && tx0 + x < Wl) {
      const float v = acc[(y * tp + x) * kD + c];
      gb[((size_t)(ty0 + y) * Wl + tx0 + x) * rowstride] = from_f32<T>(v);
    }
  }
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }


// ---------------------------------------------------------------------------------
// Query tiles of the grad_value kernel.
struct QueryTiles {
  int mode;                              // 1: grid tiles per level, 0: runs of consecutive queries
  int prefix[kMaxLevels + 1];            // grid mode: tile-index prefix per query level
  int ntx[kMaxLevels];
  int per_image;                         // tiles per image
};

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) v = min(v, __shfl_xor(v, s, 64));
  return v;
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) v = max(v, __shfl_xor(v, s, 64));
  return v;
}

// ---------------------------------------------------------------------------------
// grad_value by QUERY tiles, binned per tile (default): one wave per (tile of 16
// queries, image, head), all 32 channels, lane = (query, point) = one tap.
//
// Per value level l the tile's taps cover a small box of cells (smooth encoder
// offsets: a few dozen cells).  Instead of adding every corner into an LDS window with
// a chain of dependent read-modify-writes, the wave BINS the tile's 256 corner
// contributions by cell: a counting sort inside the wave -- ranks from LDS INTEGER
// atomics (ds_add_rtn_u32, ~12 lane-ops/clk/CU on gfx950, 35x the rate of ds_add_f32:
// tools/micro/lds_atomic_bench.hip), one wave-wide scan, a scatter of {query, weight}
// records -- and then sums each non-empty cell's records in REGISTERS (lane = cell
// parity x 32 channels: independent LDS reads and FMAs, no dependent chain) and adds the
// cell to grad_value with ONE f32 atomic per channel: two 128-B rows per atomic
// wave-instruction (the full-rate shape, MI355X_MICROARCH §Global float atomics).
// Boxes wider than kCellCap cells are clipped; the corners outside go straight to
// grad_value (one 128-B atomic row each).
constexpr int kCellCap = 512;

template <int TX, int TY>
__device__ __forceinline__ int btile_query(const QueryTiles& qt, const Levels& lv, int L, int tile, int idx, int Q) {
  if (qt.mode == 0) {
    const int q = tile * TX * TY + idx;
    return q < Q ? q : -1;
  }
  int lq = 0;
  while (lq + 1 < L && tile >= qt.prefix[lq + 1]) ++lq;
  const int t = tile - qt.prefix[lq];
  const int y = (t / qt.ntx[lq]) * TY + idx / TX, x = (t % qt.ntx[lq]) * TX + idx % TX;
  return (y < lv.h[lq] && x < lv.w[lq]) ? lv.start[lq] + y * lv.w[lq] + x : -1;
}

// TX x TY queries per tile (<= 64: one query per lane); NT = taps per lane
template <typename T, int TX, int TY>
__global__ void __launch_bounds__(64) msda_bwd_binned_kernel(const float* __restrict__ loc,
                                                             const float* __restrict__ attw,
                                                             const T* __restrict__ gout, float* __restrict__ gvalue,
                                                             Levels lv, QueryTiles qt, int S, int Hh, int Q, int L,
                                                             int nblk) {
  constexpr int P = 4;
  constexpr int NQ = TX * TY;                 // queries per tile
  static_assert(NQ * P % 64 == 0 && NQ <= 64, "whole taps per lane");
  constexpr int NT = NQ * P / 64;             // taps per lane
  constexpr int NR = NQ * P * 4;              // corner records per level
  __shared__ float sg[NQ * kD];
  __shared__ int cnt[kCellCap];
  __shared__ int offs[kCellCap];
  __shared__ int cells[kCellCap];
  __shared__ int2 srt[NR];
  const int blk = xcd_swizzle(blockIdx.x, nblk);
  const int h = blk % Hh;
  const int tile = (blk / Hh) % qt.per_image;
  const int b = blk / Hh / qt.per_image;
  const int lane = threadIdx.x;
  const int LP = L * P;
  // tap i of the lane: (query (lane + 64 i) % NQ, point (lane + 64 i) / NQ)
  int tq[NT], tpt[NT], qid[NT];
  long long grp[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    const int t = lane + 64 * i;
    tq[i] = t % NQ;
    tpt[i] = t / NQ;
    qid[i] = btile_query<TX, TY>(qt, lv, L, tile, tq[i], Q);
    grp[i] = ((long long)b * Q + (qid[i] < 0 ? 0 : qid[i])) * Hh + h;
  }
  // every tap of the lane on every level, loaded up front (one global round trip)
  float2 pxy[kMaxLevels][NT];
  float paw[kMaxLevels][NT];
#pragma unroll
  for (int l = 0; l < kMaxLevels; ++l)
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      pxy[l][i] = make_float2(0.f, 0.f);
      paw[l][i] = 0.f;
      if (l < L && qid[i] >= 0) {
        pxy[l][i] = *reinterpret_cast<const float2*>(loc + (grp[i] * LP + l * P + tpt[i]) * 2);
        paw[l][i] = attw[grp[i] * LP + l * P + tpt[i]];
      }
    }
  {
    // grad_out rows of the tile's queries: lane = (query, 8-channel part)
    constexpr int V = Vec16<T>::N;
    constexpr int parts = kD / V;
    for (int r = lane / parts; r < NQ; r += 64 / parts) {
      const int q = btile_query<TX, TY>(qt, lv, L, tile, r, Q);
      float v[V];
#pragma unroll
      for (int j = 0; j < V; ++j) v[j] = 0.f;
      if (q >= 0) Vec16<T>::load(gout + (((long long)b * Q + q) * Hh + h) * kD + (lane % parts) * V, v);
#pragma unroll
      for (int j = 0; j < V; ++j) sg[r * kD + (lane % parts) * V + j] = v[j];
    }
  }
  for (int i = lane; i < kCellCap; i += 64) cnt[i] = 0;
  const int hp = lane >> 5, ch = lane & 31;
  const size_t rowstride = (size_t)Hh * kD;
  const size_t vbase = ((size_t)b * S * Hh + h) * kD;
  for (int l = 0; l < L; ++l) {
    const int Hl = lv.h[l], Wl = lv.w[l];
    const size_t lbase = vbase + (size_t)lv.start[l] * rowstride;
    int cy[NT][4], cx[NT][4];
    float cw[NT][4];
    bool ok[NT][4];
    int ylo = 1 << 30, xlo = 1 << 30, yhi = -1, xhi = -1;
    bool anyok = false;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      float2 xy = pxy[0][i];
      float aw = paw[0][i];
#pragma unroll
      for (int k = 1; k < kMaxLevels; ++k)
        if (l == k) {
          xy = pxy[k][i];
          aw = paw[k][i];
        }
      const Tap t = tap_geom(xy.x, xy.y, Hl, Wl);
      const bool tv = qid[i] >= 0 && t.inside;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        cy[i][k] = t.h0 + (k >> 1);
        cx[i][k] = t.w0 + (k & 1);
        ok[i][k] = tv && cy[i][k] >= 0 && cy[i][k] < Hl && cx[i][k] >= 0 && cx[i][k] < Wl;
        cw[i][k] = ((k >> 1) ? t.lh : t.hh) * ((k & 1) ? t.lw : t.hw) * aw;
        if (ok[i][k]) {
          anyok = true;
          ylo = min(ylo, cy[i][k]);
          yhi = max(yhi, cy[i][k]);
          xlo = min(xlo, cx[i][k]);
          xhi = max(xhi, cx[i][k]);
        }
      }
    }
    if (__ballot(anyok) == 0ull) continue;
    const int oy = wave_min(ylo), ox = wave_min(xlo);
    const int BX = min(wave_max(xhi) - ox + 1, kCellCap);
    const int BY = min(wave_max(yhi) - oy + 1, kCellCap / BX);
    const int ncell = BX * BY;
    // ranks within the corner's cell (LDS integer atomics)
    int cell[NT][4], rk[NT][4];
    bool out[NT][4];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool in = ok[i][k] && (unsigned)(cy[i][k] - oy) < (unsigned)BY && (unsigned)(cx[i][k] - ox) < (unsigned)BX;
        out[i][k] = ok[i][k] && !in;
        cell[i][k] = in ? (cy[i][k] - oy) * BX + (cx[i][k] - ox) : -1;
        rk[i][k] = in ? atomicAdd(&cnt[cell[i][k]], 1) : 0;
      }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // exclusive scan of the counts + compaction of the non-empty cells: lane owns cells
    // [CPL lane, CPL lane + CPL); one wave scan of (records << 12 | non-empty cells)
    constexpr int CPL = kCellCap / 64;
    int c4[CPL], pk = 0;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int e = CPL * lane + j;
      c4[j] = e < ncell ? cnt[e] : 0;
      pk += (c4[j] << 12) + (c4[j] > 0);
    }
    int inc = pk;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int u = __shfl_up(inc, d, 64);
      if (lane >= d) inc += u;
    }
    const int total = __shfl(inc, 63, 64);
    int ex = inc - pk;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int e = CPL * lane + j;
      if (e < ncell) {
        offs[e] = ex >> 12;
        if (c4[j] > 0) cells[ex & 4095] = e;
        ex += (c4[j] << 12) + (c4[j] > 0);
      }
    }
    const int nlist = total & 4095;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (cell[i][k] >= 0) srt[offs[cell[i][k]] + rk[i][k]] = make_int2(tq[i] * kD, __float_as_int(cw[i][k]));
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // per non-empty cell: sum its records in registers (4 records in flight), one atomic
    // per channel
    {
      for (int i = hp; i < nlist; i += 2) {
        const int e = cells[i];
        const int o = offs[e], n = cnt[e];
        float v0 = 0.f, v1 = 0.f;
        int j = o;
        for (; j + 4 <= o + n; j += 4) {
          const int2 r0 = srt[j], r1 = srt[j + 1], r2 = srt[j + 2], r3 = srt[j + 3];
          const float g0 = sg[r0.x + ch], g1 = sg[r1.x + ch], g2 = sg[r2.x + ch], g3 = sg[r3.x + ch];
          v0 = __fmaf_rn(__int_as_float(r0.y), g0, v0);
          v1 = __fmaf_rn(__int_as_float(r1.y), g1, v1);
          v0 = __fmaf_rn(__int_as_float(r2.y), g2, v0);
          v1 = __fmaf_rn(__int_as_float(r3.y), g3, v1);
        }
        for (; j < o + n; ++j) {
          const int2 r = srt[j];
          v0 = __fmaf_rn(__int_as_float(r.y), sg[r.x + ch], v0);
        }
        const int y = oy + e / BX, x = ox + e % BX;
        atomicAdd(gvalue + lbase + (size_t)(y * Wl + x) * rowstride + ch, v0 + v1);
      }
    }
    // clipped corners: one 128-B atomic row each
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        unsigned long long m = __ballot(out[i][k]);
        while (m) {
          const int src = __ffsll((long long)m) - 1;
          m &= m - 1;
          const int y = __shfl(cy[i][k], src, 64), x = __shfl(cx[i][k], src, 64), qq = __shfl(tq[i], src, 64);
          const float w = __shfl(cw[i][k], src, 64);
          if (lane < kD)
            atomicAdd(gvalue + lbase + (size_t)(y * Wl + x) * rowstride + lane, w * sg[qq * kD + lane]);
        }
      }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    for (int i = lane; i < ncell; i += 64) cnt[i] = 0;
  }
}

// ---------------------------------------------------------------------------------
// grad_value by query tiles as a dense MFMA product (default for bf16, P == 4).
// Per value level the taps of a tile of queries span a small box of cells; grad_value
// over the box is
//     Gv[cell][c] = sum_q W[cell][q] g[q][c],
// W[cell][q] = sum over q's 4 points of the bilinear x attention weight of the corner at
// the cell: a [box x queries] by [queries x 32] product on v_mfma_f32_32x32x16_bf16 (W in
// f32 split into bf16 hi + lo parts, exact to ~2^-17; g is bf16 already), then one 128-B
// f32 atomic row per non-empty cell.  W is built in LDS by plain read-modify-writes: a
// query's 4 points take turns, so the lanes of a turn (distinct queries = distinct
// columns) never collide -- no integer atomics, no sort (the binned kernel's counting
// sort and per-cell record walk measured no faster at 4 x 4 tiles; the win is the tile
// size: tools/kbench.py --only msda, 0.95 -> 0.67 ms per backward at C2).
// msda_bwd_mfma_wg_kernel: 8 x 8 query tiles, a 4-wave workgroup, thread = tap (query
// tid / 4, point tid % 4), ONE box per level for the 64 queries, so the cells
// that neighbouring 4 x 4 tiles would each flush are added once (grad_value is bound by
// the float-atomic rate: ~1.1 TB/s of added bytes on gfx950).  W[cell][64 queries] is
// built band by band (kBandCap cells; bands with no corner are skipped), each wave writes
// its 16 queries' columns with the points taking turns, and the row tiles of the band's
// product ([32 cells] x K = 64 queries, 4 K-steps x hi/lo) are spread over the waves.
// GEOM: grad_loc / grad_attn in the same walk (replacing the geom gather kernel): a tap
// needs d_k = grad_out[q] . value[corner k] for its 4 corners, and over a band those are
// entries of the product Dm[q][cell] = grad_out[q][:] . value[cell][:] -- one MFMA GEMM
// ([64 queries] x K = 32 channels x [band cells]) on the band's value rows, each loaded
// once per tile (the gather kernel requested 4 corner rows per tap: ~6x the bytes).
// Dm goes to LDS (over W, after the band's atomics), every tap reads its corners' entries.
// Band skeleton (template SKEL; VS_MSDA_SKEL selects the variant at run time):
//  * SKEL 2 (ZAFTER, default): W is cleared AFTER a band's last barrier, each wave clearing
//    only the W columns it writes (its 16 queries), so the next band starts on zeroed LDS
//    with no zero-fill pass + barrier of its own (5 barriers a non-empty band instead of
//    6), and the hit flags are replaced by "product != 0": C2 encoder shape 0.539 ->
//    0.517 ms ("smooth" offsets), 0.674 -> 0.643 ms (iid +-4 px), tools/kbench.py;
//  * SKEL 0: zero-fill + barrier at the start of every band, per-cell hit flags.
//  Measured and dropped: a per-level bitmask of the non-empty bands in place of the
//  per-band vote (its barrier gone too) cost more than the barrier it removed (LDS atomics:
//  0.62 ms; a wave-shuffle OR with integer band divisions: 0.535 ms vs 0.517).
constexpr int kBandCap = 128;
constexpr int kWP8 = 68;       // W row pitch (floats): 64 queries + 4
constexpr int kWFloats = kBandCap * kWP8;
constexpr int kMsdaSkelDefault = 2;
constexpr int kDP = 132;       // Dm row pitch (floats) of the SKEL 0 walk: 128 band cells + 4

template <int TX, int TY, bool GEOM, int SKEL = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) msda_bwd_mfma_wg_kernel(const float* __restrict__ loc,
                                                               const float* __restrict__ attw,
                                                               const bf16* __restrict__ gout,
                                                               float* __restrict__ gvalue, Levels lv, QueryTiles qt,
                                                               int S, int Hh, int Q, int L, int nblk,
                                                               const bf16* __restrict__ value, float* __restrict__ gloc,
                                                               float* __restrict__ gattw, int lbmask) {
  constexpr int P = 4;
  constexpr int NQ = TX * TY;
  static_assert(NQ == 64, "64 queries x 4 points = one tap per thread");
  __shared__ __attribute__((aligned(16))) short sg[NQ * kD];
  __shared__ __attribute__((aligned(16))) float sW[kBandCap * kWP8];
  __shared__ int sHit[kBandCap];
  __shared__ int sBox[4][4];
  const int blk = xcd_swizzle(blockIdx.x, nblk);
  const int h = blk % Hh;
  const int tile = (blk / Hh) % qt.per_image;
  const int b = blk / Hh / qt.per_image;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  // lbmask bit i: barrier i of the band walk orders LDS only (lds_barrier), so the band's
  // fire-and-forget grad_value atomics stay in flight across it (else __syncthreads)
  auto bar = [&](int bit) {
    if (lbmask & bit) lds_barrier();
    else __syncthreads();
  };
  const bool LB = (lbmask & 2) != 0;
  constexpr bool ZAFTER = (SKEL & 2) != 0;   // band skeleton variant (see kMsdaSkelDefault)
  __shared__ int sAny[2][4];
  int band_par = 0;
  if (ZAFTER) {                               // every band starts on a zeroed W
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i = tid; i < kWFloats / 4; i += 256) reinterpret_cast<float4*>(sW)[i] = z4;
  }
  const int LP = L * P;
  const int tq = tid >> 2, tpt = tid & 3;
  const int qid = btile_query<TX, TY>(qt, lv, L, tile, tq, Q);
  const long long grp = ((long long)b * Q + (qid < 0 ? 0 : qid)) * Hh + h;
  // this tap's location / weight, one level ahead (registers for all levels cost occupancy)
  float2 nxy = make_float2(0.f, 0.f);
  float naw = 0.f;
  if (qid >= 0) {
    nxy = *reinterpret_cast<const float2*>(loc + (grp * LP + tpt) * 2);
    naw = attw[grp * LP + tpt];
  }
  {  // grad_out rows: thread = (query, 8-channel part)
    const int part = tid & 3;
    bf16x8_t v = zero8();
    if (qid >= 0) v = ld8(gout + (((long long)b * Q + qid) * Hh + h) * kD + part * 8);
    *reinterpret_cast<bf16x8_t*>(sg + tq * kD + part * 8) = v;
  }
  __syncthreads();
  bf16x8_t bq[4];                             // B operand per K-step: k = query 16 ks + 8 hh + j
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int j = 0; j < 8; ++j) bq[ks][j] = sg[(16 * ks + 8 * hh + j) * kD + r];

  const size_t rowstride = (size_t)Hh * kD;
  const size_t vbase = ((size_t)b * S * Hh + h) * kD;
  for (int l = 0; l < L; ++l) {
    const int Hl = lv.h[l], Wl = lv.w[l];
    const size_t lbase = vbase + (size_t)lv.start[l] * rowstride;
    const float2 xy = nxy;
    const float aw = naw;
    if (l + 1 < L && qid >= 0) {
      nxy = *reinterpret_cast<const float2*>(loc + (grp * LP + (l + 1) * P + tpt) * 2);
      naw = attw[grp * LP + (l + 1) * P + tpt];
    }
    const Tap t = tap_geom(xy.x, xy.y, Hl, Wl);
    const bool tv = qid >= 0 && t.inside;
    int cy[4], cx[4];
    float cw[4];
    bool ok[4];
    int ylo = 1 << 30, xlo = 1 << 30, yhi = -1, xhi = -1;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      cy[k] = t.h0 + (k >> 1);
      cx[k] = t.w0 + (k & 1);
      ok[k] = tv && cy[k] >= 0 && cy[k] < Hl && cx[k] >= 0 && cx[k] < Wl;
      cw[k] = ((k >> 1) ? t.lh : t.hh) * ((k & 1) ? t.lw : t.hw) * aw;
      if (ok[k]) {
        ylo = min(ylo, cy[k]);
        yhi = max(yhi, cy[k]);
        xlo = min(xlo, cx[k]);
        xhi = max(xhi, cx[k]);
      }
    }
    {
      const int a = wave_min(ylo), bb = wave_max(yhi), c = wave_min(xlo), d = wave_max(xhi);
      if (lane == 0) {
        sBox[wave][0] = a;
        sBox[wave][1] = bb;
        sBox[wave][2] = c;
        sBox[wave][3] = d;
      }
    }
    bar(1);
    int oy = sBox[0][0], yh = sBox[0][1], ox = sBox[0][2], xh = sBox[0][3];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      oy = min(oy, sBox[w][0]);
      yh = max(yh, sBox[w][1]);
      ox = min(ox, sBox[w][2]);
      xh = max(xh, sBox[w][3]);
    }
    float dk[4] = {0.f, 0.f, 0.f, 0.f};       // GEOM: grad_out . value at the tap's corners
    const int BY = yh < 0 ? 0 : yh - oy + 1, BX = yh < 0 ? 1 : xh - ox + 1;   // yh < 0: no corner here
    const int SBX = min(BX, kBandCap), SBY = kBandCap / SBX;
    bar(1);                                   // sBox is rewritten by the next level
    for (int by0 = 0; by0 < BY; by0 += SBY) {
      for (int bx0 = 0; bx0 < BX; bx0 += SBX) {
        const int bw = min(SBX, BX - bx0), bh = min(SBY, BY - by0);
        int cell[4];
        bool any = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int yy = cy[k] - oy - by0, xx = cx[k] - ox - bx0;
          const bool in = ok[k] && (unsigned)yy < (unsigned)bh && (unsigned)xx < (unsigned)bw;
          cell[k] = in ? yy * bw + xx : -1;
          any |= in;
        }
        bool band_any;
        if (LB) {                             // double-buffered per-wave flags: a wave cannot
          const bool wany = __ballot(any) != 0;   // lap a slower one by 2; the ballot runs in
          if (lane == 0) sAny[band_par][wave] = wany;   // all lanes (inside `if (lane == 0)` it saw one)
          lds_barrier();
          band_any = sAny[band_par][0] | sAny[band_par][1] | sAny[band_par][2] | sAny[band_par][3];
          band_par ^= 1;
        } else {
          band_any = __syncthreads_or(any);
        }
        if (!band_any) continue;              // empty band (also the barrier after the last one)
        const int ncell = bw * bh, nmt = (ncell + 31) >> 5;
        const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
        // Dm pitch: the band's cell tiles + 4 (keeps the Dm overlay inside the rows W used)
        const int dp = ZAFTER ? nmt * 32 + 4 : kDP;
        if (!ZAFTER) {
          for (int i = tid; i < nmt * 32 * (kWP8 / 4); i += 256) reinterpret_cast<float4*>(sW)[i] = z4;
          for (int i = tid; i < nmt * 32; i += 256) sHit[i] = 0;
          bar(4);
        }
#pragma unroll
        for (int pt = 0; pt < P; ++pt) {      // a query's 4 points are lanes of one wave: take turns
          if (tpt == pt) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
              if (cell[k] >= 0) {
                sW[cell[k] * kWP8 + tq] += cw[k];
                if (!ZAFTER) sHit[cell[k]] = 1;
              }
          }
          wave_sync();
        }
        bar(8);
        for (int m = wave; m < nmt; m += 4) {
          f32x16_t acc;
          zero16(acc);
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            const float* wr = sW + (32 * m + r) * kWP8 + 16 * ks + 8 * hh;
            const float4 w0 = *reinterpret_cast<const float4*>(wr);
            const float4 w1 = *reinterpret_cast<const float4*>(wr + 4);
            const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
            bf16x8_t ahi, alo;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const short hb = bf16_bits(wv[j]);
              ahi[j] = hb;
              alo[j] = bf16_bits(wv[j] - bf16_bits_to_f32((unsigned short)hb));
            }
            acc = mfma16(ahi, bq[ks], acc);
            acc = mfma16(alo, bq[ks], acc);
          }
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int c = 32 * m + crow(i, hh);
            // ZAFTER: a cell no tap touched has an all-zero W row, so its product is +0
            // exactly and is skipped like an unhit cell (adding 0 would not change
            // grad_value either: it starts at +0 and never becomes -0; grad_out finite)
            if (c < ncell && (ZAFTER ? acc[i] != 0.f : sHit[c] != 0)) {
              const int y = oy + by0 + c / bw, x = ox + bx0 + c % bw;
              atomicAdd(gvalue + lbase + (size_t)(y * Wl + x) * rowstride + r, acc[i]);
            }
          }
        }
        bar(16);                              // W / hit flags are rewritten by the next band
        if (GEOM) {
          // Dm[q][cell] over the band: wave w takes cell tile w (value rows loaded once)
          float* sD = sW;
          if (wave < nmt) {
            bf16x8_t bv[2] = {zero8(), zero8()};
            const int c = 32 * wave + r;
            if (c < ncell) {
              const int y = oy + by0 + c / bw, x = ox + bx0 + c % bw;
              const bf16* vr = value + lbase + (size_t)(y * Wl + x) * rowstride + 8 * hh;
              bv[0] = ld8(vr);
              bv[1] = ld8(vr + 16);
            }
#pragma unroll
            for (int mq = 0; mq < 2; ++mq) {
              // A operand grad_out[q = 32 mq + r][c = 16 ks + 8 hh + j], read from LDS here
              // (held in registers it cost occupancy: 4 -> 2 waves/SIMD)
              const short* ga = sg + (32 * mq + r) * kD + 8 * hh;
              f32x16_t acc;
              zero16(acc);
              acc = mfma16(*reinterpret_cast<const bf16x8_t*>(ga), bv[0], acc);
              acc = mfma16(*reinterpret_cast<const bf16x8_t*>(ga + 16), bv[1], acc);
#pragma unroll
              for (int i = 0; i < 16; ++i) sD[(32 * mq + crow(i, hh)) * dp + 32 * wave + r] = acc[i];
            }
          }
          bar(32);
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (cell[k] >= 0) dk[k] += sD[tq * dp + cell[k]];
          bar(64);                            // Dm is overwritten by the next band's W
        }
        if (ZAFTER) {
          // clear W for the next band: wave w clears only the columns it writes (its 16
          // queries), over every row this band's W or Dm touched, so no other wave's next
          // build can race with the clear and no barrier is needed; Dm leftovers in the
          // pad columns are never read as W, and Dm itself is always written before read
          // Rows in blocks of 16; within a 16-lane group the rows are 4 apart, so the group's
          // 16-B stores cover all 64 banks once (pitch 68: bank = 4 row + column).
          const int zr = GEOM ? min(kBandCap, max(nmt * 32, (64 * dp + kWP8 - 1) / kWP8)) : nmt * 32;
          const int zrow = 4 * ((lane >> 2) & 3) + (lane >> 4);
          for (int rb = 0; rb < zr; rb += 16)
            *reinterpret_cast<float4*>(sW + (rb + zrow) * kWP8 + 16 * wave + 4 * (lane & 3)) = z4;
        }
      }
    }
    if (GEOM && qid >= 0) {                   // same formulas as msda_bwd_geom_kernel
      const float fW = (float)Wl, fH = (float)Hl;
      float r_w = 0.f, r_x = 0.f, r_y = 0.f;
      if (tv) {
        r_w = t.hh * t.hw * dk[0] + t.hh * t.lw * dk[1] + t.lh * t.hw * dk[2] + t.lh * t.lw * dk[3];
        r_x = fW * aw * (-t.hh * dk[0] + t.hh * dk[1] - t.lh * dk[2] + t.lh * dk[3]);
        r_y = fH * aw * (-t.hw * dk[0] - t.lw * dk[1] + t.hw * dk[2] + t.lw * dk[3]);
      }
      const long long o = grp * LP + l * P + tpt;
      gattw[o] = r_w;
      *reinterpret_cast<float2*>(gloc + o * 2) = make_float2(r_x, r_y);
    }
  }
}

// ---------------------------------------------------------------------------------
// grad_value + grad_loc / grad_attn by PYRAMID COLUMNS (default for bf16 encoder problems:
// queries = the value grid, P == 4).  The tile kernel above flushes one f32 atomic row per
// (8 x 8 query tile, sampled level, touched cell), and a cell is touched by the tiles of
// every query level whose taps reach it: at the C2 shapes ~4.3 flushes per cell (a cell of
// the 32 x 32 level is reached by the 16 tiles of the 128 x 128 level above it), 553 MB
// written per launch for 187 MB of outputs (profiles/r3_pmc_traffic_top.txt).  Float
// atomics execute memory-side at ~1.3 TB/s of added bytes (MI355X_MICROARCH §Global float
// atomics), so those flushes bound the kernel.
// Here a workgroup owns one COLUMN of the pyramid: a CY x CX block of the finest level and
// the blocks over the same image area at every other level (ColGeo; 8 x 16, 4 x 8, 2 x 4
// at a 2x pyramid = 168 queries), enumerated largest level first, row-major, in chunks of
// 64 queries (thread = tap: query tid / 4, point tid % 4, as in the tile kernel).  Per
// sampled level the union box of the column's corners is walked in bands of <= kBandCap
// cells; a band's grad_value accumulates over ALL the chunks that reach it in the MFMA
// accumulators (W[cell][q] x g[q][c], K = one chunk's 64 queries, W in bf16 hi + lo) and
// is flushed ONCE: 128-B f32 atomic rows per non-zero cell.  grad_loc / grad_attn as in
// the tile kernel (Dm[q][cell] = g[q] . value[cell] per (band, chunk), the band's value
// rows loaded once and reused by every chunk, stored transposed over W: 16-B stores); a
// tap's corner dots stay in registers across bands (dk[chunk][corner]).  Band / chunk pairs are skipped from per-chunk boxes
// (no vote barrier).  2 LDS-only barriers per pair (W built -> product + Dm; Dm stored -> dots):
// the product / Dm^T overlay and the dots / W clear touch one wave's own rows / columns only
// (round 6; the round-5 kernel had a barrier after each of the four phases).

// MFMA operand (8 k-values of one column, k = rows k0 + 8hh + j, column lane & 31) from a
// row-major bf16 LDS image, by the gfx950 transposed read (cdna_hip_programming.md T10;
// EXEC all ones).  64-B row pitch keeps the 16-lane groups in distinct banks.
__device__ __forceinline__ bf16x8_t tr8(const short* img, int pitch, int k0, int lane) {
  const int hh = lane >> 5;
  const int row = k0 + 8 * hh + ((lane & 15) >> 2);
  const int col = (lane & 16) + 4 * (lane & 3);
  typedef __attribute__((address_space(3))) bf16x4_t lds_v4;
  const bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(img + row * pitch + col));
  const bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(img + (row + 4) * pitch + col));
  bf16x8_t v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return v;
}

__device__ __forceinline__ int sgpr(int v) { return __builtin_amdgcn_readfirstlane(v); }

// WINT (default): W built as FIXED-POINT integers with no-return ds_add_u32: the four points of
// a query hit the same cells, and as f32 they had to take turns (4 wave-synchronised rounds of
// read-modify-write per (band, chunk) pair; ds_add_f32 is 35x slower than the integer add on
// gfx950).  An entry W[cell][q] sums at most q's four points of the level, |W| <= sum_p |aw_p|
// (bilinear weights <= 1), so the quantum is 2^-e per (workgroup, level) with e = 30 while that
// bound is <= 1 (softmax-normalised weights, the encoder: every partial sum stays inside int32)
// and e lowered by ceil(log2(bound)) beyond it -- any attention weights the op is handed stay
// exact to the quantum (round-5 ADVICE: a fixed 2^-30 wrapped for weights summing past 2).  The
// product converts each W value back (exact power-of-two scaling) before the bf16 hi / lo split.
// DBG: the parts switched off in the round-5 timing split (profiles/r5_msda_split.txt; 1 no W
// build, 2 no product, 4 no Dm / dots, 8 no flush); only DBG = 0 is instantiated
template <int NCH, bool WINT = true, int DBG = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NCH <= 3 ? 3 : 2)))
msda_bwd_col_kernel(const float* __restrict__ loc, const float* __restrict__ attw, const bf16* __restrict__ gout,
                    const bf16* __restrict__ value, float* __restrict__ gvalue, float* __restrict__ gloc,
                    float* __restrict__ gattw, Levels lv, ColGeo cg, int S, int Hh, int Q, int L, int nblk) {
  constexpr int P = 4;
  __shared__ __attribute__((aligned(16))) short sg[NCH * 64 * kD];   // grad_out rows, column order
  __shared__ __attribute__((aligned(16))) float sW[kWFloats];        // W of a (band, chunk) / Dm overlay
  __shared__ int sBox[2][4][NCH][4];                                 // [level parity][wave][chunk] box
  __shared__ int sAwm[2][4];                                         // [level parity][wave] max sum_p |aw_p|
  const int blk = xcd_swizzle(blockIdx.x, nblk);                     // the 8 heads of a column: one XCD
  const int h = blk % Hh;
  const int col = (blk / Hh) % cg.per_image;
  const int b = blk / Hh / cg.per_image;
  const int cyy = col / cg.ncx, cxx = col - (col / cg.ncx) * cg.ncx;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int tq = tid >> 2, tpt = tid & 3;
  // this thread's query in every chunk (-1: none)
  int qid[NCH];
#pragma unroll
  for (int s = 0; s < NCH; ++s) qid[s] = -1;
  int nq = 0;
  for (int i = 0; i < L; ++i) {
    const int l = cg.ord[i];
    const int y0 = cyy * cg.ty[l], x0 = cxx * cg.tx[l];
    const int ny = min(cg.ty[l], lv.h[l] - y0), nx = min(cg.tx[l], lv.w[l] - x0);
    if (ny <= 0 || nx <= 0) continue;
#pragma unroll
    for (int s = 0; s < NCH; ++s) {
      const int k = 64 * s + tq - nq;
      if (k >= 0 && k < ny * nx) qid[s] = lv.start[l] + (y0 + k / nx) * lv.w[l] + x0 + k % nx;
    }
    nq += ny * nx;
  }
  const int nch = (nq + 63) >> 6;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int s = 0; s < NCH; ++s) {            // grad_out rows: thread = (query, 8-channel part)
    bf16x8_t v = zero8();
    if (qid[s] >= 0) v = ld8(gout + (((long long)b * Q + qid[s]) * Hh + h) * kD + tpt * 8);
    *reinterpret_cast<bf16x8_t*>(sg + (64 * s + tq) * kD + tpt * 8) = v;
  }
  for (int i = tid; i < kWFloats / 4; i += 256) reinterpret_cast<float4*>(sW)[i] = z4;
  __syncthreads();

  const int LP = L * P;
  const size_t rowstride = (size_t)Hh * kD;
  const size_t vbase = ((size_t)b * S * Hh + h) * kD;
  const int zrow = 4 * ((lane >> 2) & 3) + (lane >> 4);   // W clear: 16 rows x 4 quads per wave
  // a level's sampling locations / weights are requested one level ahead: loaded at the top
  // of their level, their round trip sat in front of the box reductions of every level
  float2 xyn[NCH];
  float awn[NCH];
  auto load_level = [&](int l) {
#pragma unroll
    for (int s = 0; s < NCH; ++s) {
      xyn[s] = make_float2(0.f, 0.f);
      awn[s] = 0.f;
      if (qid[s] >= 0) {
        const long long o = (((long long)b * Q + qid[s]) * Hh + h) * LP + l * P + tpt;
        xyn[s] = *reinterpret_cast<const float2*>(loc + o * 2);
        awn[s] = attw[o];
      }
    }
  };
  load_level(0);
  for (int l = 0; l < L; ++l) {
    const int Hl = lv.h[l], Wl = lv.w[l];
    const size_t lbase = vbase + (size_t)lv.start[l] * rowstride;
    float2 xy[NCH];
    float aw[NCH], dk[NCH][4];
#pragma unroll
    for (int s = 0; s < NCH; ++s) {
      xy[s] = xyn[s];
      aw[s] = awn[s];
      dk[s][0] = dk[s][1] = dk[s][2] = dk[s][3] = 0.f;
    }
    if (l + 1 < L) load_level(l + 1);
    // per-chunk boxes of the in-level corners
    const int par = l & 1;
#pragma unroll
    for (int s = 0; s < NCH; ++s) {
      int ylo = 1 << 30, xlo = 1 << 30, yhi = -1, xhi = -1;
      if (qid[s] >= 0) {
        const Tap t = tap_geom(xy[s].x, xy[s].y, Hl, Wl);
        if (t.inside) {
          ylo = max(t.h0, 0);
          yhi = min(t.h0 + 1, Hl - 1);
          xlo = max(t.w0, 0);
          xhi = min(t.w0 + 1, Wl - 1);
        }
      }
      const int a = wave_min(ylo), c = wave_max(yhi), d = wave_min(xlo), e = wave_max(xhi);
      if (lane == 0) {
        sBox[par][wave][s][0] = a;
        sBox[par][wave][s][1] = c;
        sBox[par][wave][s][2] = d;
        sBox[par][wave][s][3] = e;
      }
    }
    if (WINT) {                               // the fixed-point bound: max over queries of sum_p |aw_p|
      float am = 0.f;
#pragma unroll
      for (int s = 0; s < NCH; ++s) {
        float a = qid[s] >= 0 ? fabsf(aw[s]) : 0.f;
        a += __shfl_xor(a, 1, 64);                        // a query's 4 points are lanes 4k .. 4k + 3
        a += __shfl_xor(a, 2, 64);
        am = fmaxf(am, a);
      }
      const int amb = wave_max(__float_as_int(am));      // non-negative floats order as ints
      if (lane == 0) sAwm[par][wave] = amb;
    }
    lds_barrier();                            // (sBox is double-buffered by level parity)
    int qe = 30;                              // W quantum 2^-qe (WINT)
    if (WINT) {
      const float bound = __int_as_float(max(max(sAwm[par][0], sAwm[par][1]), max(sAwm[par][2], sAwm[par][3])));
      if (bound > 1.f) qe = bound < 0x1p20f ? 30 - (int)ceilf(log2f(bound)) : 10;
      qe = sgpr(qe);
    }
    int cb[NCH][4];
    int oy = 1 << 30, yh = -1, ox = 1 << 30, xh = -1;
#pragma unroll
    for (int s = 0; s < NCH; ++s) {
      int a = sBox[par][0][s][0], c = sBox[par][0][s][1], d = sBox[par][0][s][2], e = sBox[par][0][s][3];
#pragma unroll
      for (int w = 1; w < 4; ++w) {
        a = min(a, sBox[par][w][s][0]);
        c = max(c, sBox[par][w][s][1]);
        d = min(d, sBox[par][w][s][2]);
        e = max(e, sBox[par][w][s][3]);
      }
      cb[s][0] = sgpr(a);
      cb[s][1] = sgpr(c);
      cb[s][2] = sgpr(d);
      cb[s][3] = sgpr(e);
      if (cb[s][1] >= 0) {
        oy = min(oy, cb[s][0]);
        yh = max(yh, cb[s][1]);
        ox = min(ox, cb[s][2]);
        xh = max(xh, cb[s][3]);
      }
    }
    const int BY = yh < 0 ? 0 : yh - oy + 1, BX = yh < 0 ? 1 : xh - ox + 1;
    const int SBX = min(BX, kBandCap), SBY = kBandCap / SBX;
    for (int by0 = 0; by0 < BY; by0 += SBY) {
      for (int bx0 = 0; bx0 < BX; bx0 += SBX) {
        const int bw = min(SBX, BX - bx0), bh = min(SBY, BY - by0);
        const int y0 = oy + by0, x0 = ox + bx0;     // band origin (cells of level l)
        const int ncell = bw * bh, nmt = (ncell + 31) >> 5;
        const int zr = nmt * 32;                    // rows W / Dm^T touch
        bf16x8_t bv0 = zero8(), bv1 = zero8();      // value rows of this wave's cell tile
        if (wave < nmt) {
          const int c = 32 * wave + r;
          if (c < ncell) {
            const unsigned inv = (65536u + (unsigned)bw - 1u) / (unsigned)bw;   // c / bw by multiply-shift
            const unsigned cy = __umul24((unsigned)c, inv) >> 16, cx = (unsigned)c - __umul24(cy, (unsigned)bw);
            const bf16* vr = value + lbase + (size_t)((y0 + (int)cy) * Wl + x0 + (int)cx) * rowstride + 8 * hh;
            bv0 = ld8(vr);
            bv1 = ld8(vr + 16);
          }
        }
        f32x16_t acc;
        zero16(acc);
        bool any = false;
#pragma unroll
        for (int s = 0; s < NCH; ++s) {
          if (s >= nch) break;
          if (cb[s][1] < y0 || cb[s][0] >= y0 + bh || cb[s][3] < x0 || cb[s][2] >= x0 + bw) continue;
          any = true;
          int cell[4] = {-1, -1, -1, -1};
          float cw[4] = {0.f, 0.f, 0.f, 0.f};
          if (qid[s] >= 0) {
            const Tap t = tap_geom(xy[s].x, xy[s].y, Hl, Wl);
            if (t.inside) {
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                const int yy = t.h0 + (k >> 1) - y0, xx = t.w0 + (k & 1) - x0;
                // band cells are inside the level (the box holds in-level corners only)
                if ((unsigned)yy < (unsigned)bh && (unsigned)xx < (unsigned)bw) cell[k] = yy * bw + xx;
                cw[k] = ((k >> 1) ? t.lh : t.hh) * ((k & 1) ? t.lw : t.hw) * aw[s];
              }
            }
          }
          if (DBG & 1) {
          } else if (WINT) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
              if (cell[k] >= 0)
                __hip_atomic_fetch_add(reinterpret_cast<int*>(sW) + cell[k] * kWP8 + tq, __float2int_rn(ldexpf(cw[k], qe)),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          } else {
#pragma unroll
            for (int pt = 0; pt < P; ++pt) {  // a query's 4 points are lanes of one wave: take turns
              if (tpt == pt) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                  if (cell[k] >= 0) sW[cell[k] * kWP8 + tq] += cw[k];
              }
              wave_sync();
            }
          }
          lds_barrier();
          if (!(DBG & 2) && wave < nmt) {     // acc[cell][c] += W[cell][q] g[q][c]
            const short* gs = sg + 64 * s * kD;
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
              const float* wr = sW + (32 * wave + r) * kWP8 + 16 * ks + 8 * hh;
              float wv[8];
              if (WINT) {
                const int4 i0 = *reinterpret_cast<const int4*>(wr);
                const int4 i1 = *reinterpret_cast<const int4*>(wr + 4);
                const int iv[8] = {i0.x, i0.y, i0.z, i0.w, i1.x, i1.y, i1.z, i1.w};
#pragma unroll
                for (int j = 0; j < 8; ++j) wv[j] = ldexpf((float)iv[j], -qe);
              } else {
                const float4 w0 = *reinterpret_cast<const float4*>(wr);
                const float4 w1 = *reinterpret_cast<const float4*>(wr + 4);
                wv[0] = w0.x; wv[1] = w0.y; wv[2] = w0.z; wv[3] = w0.w;
                wv[4] = w1.x; wv[5] = w1.y; wv[6] = w1.z; wv[7] = w1.w;
              }
              bf16x8_t ahi, alo;
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const short hb = bf16_bits(wv[j]);
                ahi[j] = hb;
                alo[j] = bf16_bits(wv[j] - bf16_bits_to_f32((unsigned short)hb));
              }
              const bf16x8_t bq = tr8(gs, kD, 16 * ks, lane);
              acc = mfma16(ahi, bq, acc);
              acc = mfma16(alo, bq, acc);
            }
          }
          // W consumed: Dm^T overwrites it.  A wave's product reads only its own cell rows
          // (32 wave .. + 31) and its Dm^T store writes only those rows, so program order within
          // the wave suffices (wave_sync: a compiler fence across its lanes, no instruction)
          wave_sync();
          float* sD = sW;                     // Dm^T[cell][q], W's layout (pitch kWP8)
          if (!(DBG & 4) && wave < nmt) {     // Dm[q][cell] = g[q] . value[cell], cell tile = wave
#pragma unroll
            for (int mq = 0; mq < 2; ++mq) {
              const short* ga = sg + (64 * s + 32 * mq + r) * kD + 8 * hh;
              f32x16_t dm;
              zero16(dm);
              dm = mfma16(*reinterpret_cast<const bf16x8_t*>(ga), bv0, dm);
              dm = mfma16(*reinterpret_cast<const bf16x8_t*>(ga + 16), bv1, dm);
              // lane = cell 32 wave + r, registers 4i4..4i4+3 = queries 32mq + 8i4 + 4hh + 0..3:
              // one 16-B store each (pitch 68: a 16-lane group covers all 64 banks once)
              float* row = sD + (32 * wave + r) * kWP8 + 32 * mq + 4 * hh;
#pragma unroll
              for (int i4 = 0; i4 < 4; ++i4)
                *reinterpret_cast<float4*>(row + 8 * i4) =
                    make_float4(dm[4 * i4], dm[4 * i4 + 1], dm[4 * i4 + 2], dm[4 * i4 + 3]);
            }
          }
          lds_barrier();
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (cell[k] >= 0) dk[s][k] += sD[cell[k] * kWP8 + tq];
          // Dm read: clear W for the next pair.  A wave's dots read only its own query columns
          // (tq = 16 wave .. + 15), and it clears only those columns over every row W or Dm^T
          // touched -- the columns its next build writes, so no other wave's access meets them
          // before the next pair's first barrier: program order within the wave suffices
          wave_sync();
          for (int rb = 0; rb < zr; rb += 16)
            *reinterpret_cast<float4*>(sW + (rb + zrow) * kWP8 + 16 * wave + 4 * (lane & 3)) = z4;
        }
        if (!(DBG & 8) && any && wave < nmt) {   // one flush per (band, cell) for the whole column
          // cell -> (row, column) of the band by a multiply-shift (c < 128, bw <= 128: exact
          // with ceil(2^16 / bw)), 32-bit offsets from the (uniform) level base: the integer
          // division and 64-bit address of every flushed row were ~40 VALU per atomic
          const unsigned inv = (65536u + (unsigned)bw - 1u) / (unsigned)bw;
          float* gvb = gvalue + lbase;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int c = 32 * wave + crow(i, hh);
            if (c < ncell && acc[i] != 0.f) {
              // 24-bit multiplies: c * inv < 2^24, cells x rowstride < 2^24 at the encoder sizes
              // (checked on the host: S * heads * 32 < 2^24)
              const unsigned cy = __umul24((unsigned)c, inv) >> 16, cx = (unsigned)c - __umul24(cy, (unsigned)bw);
              const unsigned cell = __umul24((unsigned)(y0 + (int)cy), (unsigned)Wl) + (unsigned)(x0 + (int)cx);
              atomicAdd(gvb + (__umul24(cell, (unsigned)rowstride) + (unsigned)r), acc[i]);
            }
          }
        }
      }
    }
#pragma unroll
    for (int s = 0; s < NCH; ++s) {           // same formulas as msda_bwd_geom_kernel
      if (qid[s] < 0) continue;
      const Tap t = tap_geom(xy[s].x, xy[s].y, Hl, Wl);
      float r_w = 0.f, r_x = 0.f, r_y = 0.f;
      if (t.inside) {
        const float* d = dk[s];
        r_w = t.hh * t.hw * d[0] + t.hh * t.lw * d[1] + t.lh * t.hw * d[2] + t.lh * t.lw * d[3];
        r_x = (float)Wl * aw[s] * (-t.hh * d[0] + t.hh * d[1] - t.lh * d[2] + t.lh * d[3]);
        r_y = (float)Hl * aw[s] * (-t.hw * d[0] - t.lw * d[1] + t.hw * d[2] + t.lw * d[3]);
      }
      const long long o = (((long long)b * Q + qid[s]) * Hh + h) * LP + l * P + tpt;
      gattw[o] = r_w;
      *reinterpret_cast<float2*>(gloc + o * 2) = make_float2(r_x, r_y);
    }
  }
}


int fill_levels(Levels* lv, const int64_t* shapes, const int64_t* starts, int L, int S) {
  long long tot = 0;
  for (int l = 0; l < L; ++l) {
    lv->h[l] = (int)shapes[2 * l];
    lv->w[l] = (int)shapes[2 * l + 1];
    lv->start[l] = (int)starts[l];
    if (lv->h[l] <= 0 || lv->w[l] <= 0 || starts[l] != tot) return 0;
    tot += shapes[2 * l] * shapes[2 * l + 1];
  }
  return tot == S;
}

}  // namespace
}  // namespace vs

using namespace vs;

static int col_geo(const Levels& lv, int L, int CY, int CX, ColGeo* cg);

extern "C" int vs_msda_forward(int dtype, const void* value, const int64_t* shapes,
                               const int64_t* starts, const float* loc, const float* attw,
                               void* out, int B, int S, int Hh, int D, int L, int Q, int P,
                               void* stream) {
  VS_CHECK(D == kD, "channels per head must be 32");
  VS_CHECK(L >= 1 && L <= kMaxLevels, "1..4 levels supported");
  VS_CHECK(B > 0 && S > 0 && Hh > 0 && Q >= 0 && P > 0, "bad sizes");
  VS_CHECK(value && shapes && starts, "null pointer");
  Levels lv;
  VS_CHECK(fill_levels(&lv, shapes, starts, L, S), "spatial shapes / level starts inconsistent with S");
  if (Q == 0) return VS_OK;
  VS_CHECK(loc && attw && out, "null pointer");
  hipStream_t st = (hipStream_t)stream;
  const long long groups = (long long)B * Q * Hh;
  const int block = 256;
  const bool unrolled = P == 4;              // else the runtime-P kernel
  if (dtype == VS_BF16 && unrolled) {
    // encoder problems (Q == S: the queries are the value grid): pyramid-column visiting order
    // (msda_fwd4_kernel COL; VS_MSDA_FWD_COL=0: query order, A/B)
    ColGeo cg;
    int cq = 0;
    bool col = Q == S && L >= 2;
    if (const char* e = getenv("VS_MSDA_FWD_COL")) col = col && atoi(e) != 0;
    long long slots = groups;
    if (col && col_geo(lv, L, kMsdaColDefault[0], kMsdaColDefault[1], &cg) > 0) {
      for (int l = 0; l < L; ++l) cq += cg.ty[l] * cg.tx[l];
      slots = (long long)B * cg.per_image * cq * Hh;
      col = slots * 4 < (1LL << 31) && slots >= groups;
    } else {
      col = false;
    }
    if (!col) slots = groups;
    int grid = grid_for(slots * 4, block, 256 * 64);
#define VS_FWD4(LL)                                                                                          \
  if (col)                                                                                                   \
    hipLaunchKernelGGL((msda_fwd4_kernel<LL, 2, true>), dim3(grid), dim3(block), 0, st, (const bf16*)value,   \
                       loc, attw, (bf16*)out, lv, S, Hh, Q, slots, cg, cq);                                  \
  else                                                                                                       \
    hipLaunchKernelGGL((msda_fwd4_kernel<LL, 2>), dim3(grid), dim3(block), 0, st, (const bf16*)value, loc,    \
                       attw, (bf16*)out, lv, S, Hh, Q, groups, cg, 0)
    switch (L) {
      case 1: VS_FWD4(1); break;
      case 2: VS_FWD4(2); break;
      case 3: VS_FWD4(3); break;
      default: VS_FWD4(4); break;
    }
#undef VS_FWD4
  } else if (dtype == VS_BF16) {
    int grid = grid_for(groups * 4, block, 256 * 64);
    hipLaunchKernelGGL(msda_fwd_kernel<bf16>, dim3(grid), dim3(block), 0, st, (const bf16*)value,
                       loc, attw, (bf16*)out, lv, S, Hh, Q, L, P, groups);
  } else if (dtype == VS_F32) {
    int grid = grid_for(groups * 8, block, 256 * 64);
    hipLaunchKernelGGL(msda_fwd_kernel<float>, dim3(grid), dim3(block), 0, st, (const float*)value,
                       loc, attw, (float*)out, lv, S, Hh, Q, L, P, groups);
  } else {
    VS_CHECK(false, "dtype must be VS_F32 or VS_BF16");
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}

static void launch_geom(int dtype, const void* value, const float* loc, const float* attw, const void* gout,
                        float* gloc, float* gattw, const Levels& lv, int S, int Hh, int Q, int L, int P,
                        long long groups, hipStream_t st) {
  const int lpg = dtype == VS_BF16 ? 4 : 8;
  const int ggrid = (int)((groups * lpg + 255) / 256);
  if (dtype == VS_BF16)
    hipLaunchKernelGGL(msda_bwd_geom_kernel<bf16>, dim3(ggrid), dim3(256), 0, st, (const bf16*)value, loc, attw,
                       (const bf16*)gout, gloc, gattw, lv, S, Hh, Q, L, P, groups);
  else
    hipLaunchKernelGGL(msda_bwd_geom_kernel<float>, dim3(ggrid), dim3(256), 0, st, (const float*)value, loc, attw,
                       (const float*)gout, gloc, gattw, lv, S, Hh, Q, L, P, groups);
}

// Pyramid columns (msda_bwd_col_kernel): the finest level's CY x CX block and, at a level
// 2^k times coarser, CY >> k x CX >> k (>= 1).  Every level's blocks tile it (ncy / ncx =
// the most blocks any level needs), so each query is in exactly one column.  Returns the
// chunks of 64 queries a column needs (0: more than 6, use the tile kernel).
static int col_geo(const Levels& lv, int L, int CY, int CX, ColGeo* cg) {
  int f = 0;
  for (int l = 1; l < L; ++l)
    if ((long long)lv.h[l] * lv.w[l] > (long long)lv.h[f] * lv.w[f]) f = l;
  int ncy = 1, ncx = 1, nq = 0;
  for (int l = 0; l < kMaxLevels; ++l) {
    cg->ty[l] = cg->tx[l] = 1;
    cg->ord[l] = l;
  }
  for (int l = 0; l < L; ++l) {
    const int sy = std::min(30, std::max(0, (int)std::lround(std::log2((double)lv.h[f] / lv.h[l]))));
    const int sx = std::min(30, std::max(0, (int)std::lround(std::log2((double)lv.w[f] / lv.w[l]))));
    cg->ty[l] = std::max(1, CY >> sy);
    cg->tx[l] = std::max(1, CX >> sx);
    ncy = std::max(ncy, (lv.h[l] + cg->ty[l] - 1) / cg->ty[l]);
    ncx = std::max(ncx, (lv.w[l] + cg->tx[l] - 1) / cg->tx[l]);
    nq += cg->ty[l] * cg->tx[l];
  }
  for (int i = 1; i < L; ++i)                 // largest level first (stable)
    for (int j = i; j > 0; --j) {
      const int a = cg->ord[j - 1], c = cg->ord[j];
      if ((long long)lv.h[c] * lv.w[c] > (long long)lv.h[a] * lv.w[a]) std::swap(cg->ord[j - 1], cg->ord[j]);
      else break;
    }
  cg->ncx = ncx;
  cg->per_image = ncy * ncx;
  const int nch = (nq + 63) / 64;
  return nch <= 6 ? nch : 0;
}


static int msda_backward_impl(int dtype, const void* value, const int64_t* shapes, const int64_t* starts,
                              const float* loc, const float* attw, const void* gout, float* gvalue, float* gloc,
                              float* gattw, int B, int S, int Hh, int D, int L, int Q, int P, void* stream,
                              void* ws = nullptr) {
  VS_CHECK(D == kD, "channels per head must be 32");
  VS_CHECK(L >= 1 && L <= kMaxLevels, "1..4 levels supported");
  VS_CHECK(B > 0 && S > 0 && Hh > 0 && Q >= 0 && P > 0, "bad sizes");
  VS_CHECK(value && loc && attw && gout && gvalue && gloc && gattw && shapes && starts, "null pointer");
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");
  (void)ws;                                  // reserved (the destination-tile backward's far-tap list)
  Levels lv;
  VS_CHECK(fill_levels(&lv, shapes, starts, L, S), "spatial shapes / level starts inconsistent with S");
  hipStream_t st = (hipStream_t)stream;
  const long long groups = (long long)B * Q * Hh;
  // split backward (geom gather + grad_value product / binned kernel) when there are enough
  // queries to fill the chip; VS_MSDA_RUN=0 forces the single fused kernel
  bool split = groups >= kSplitMin;
  if (const char* e = getenv("VS_MSDA_RUN")) split = atoi(e) >= 1;   // tests: force either path
  split = split && P == 4;
  VS_HIP(hipMemsetAsync(gvalue, 0, sizeof(float) * (size_t)B * S * Hh * kD, st));
  if (Q == 0) return VS_OK;
  if (split) {
    bool mfma = dtype == VS_BF16;            // VS_MSDA_MFMA=0: the binned kernel for bf16 too
    if (const char* e = getenv("VS_MSDA_MFMA")) mfma = mfma && atoi(e) != 0;
    bool fused = mfma;                       // VS_MSDA_GEOM=0: the separate geom gather kernel
    if (const char* e = getenv("VS_MSDA_GEOM")) fused = fused && atoi(e) != 0;
    if (!fused) launch_geom(dtype, value, loc, attw, gout, gloc, gattw, lv, S, Hh, Q, L, P, groups, st);
    const int te = mfma ? 8 : 4;             // query tile edge
    QueryTiles bt;
    bt.mode = Q == S ? 1 : 0;                // grid tiles when the queries are the value grid
    bt.prefix[0] = 0;
    for (int l = 0; l < kMaxLevels; ++l) {
      const bool on = bt.mode == 1 && l < L;
      bt.ntx[l] = on ? (lv.w[l] + te - 1) / te : 1;
      bt.prefix[l + 1] = bt.prefix[l] + (on ? ((lv.h[l] + te - 1) / te) * bt.ntx[l] : 0);
    }
    bt.per_image = bt.mode == 1 ? bt.prefix[L] : (Q + te * te - 1) / (te * te);
    const long long nb2 = (long long)B * bt.per_image * Hh;
    VS_CHECK(nb2 < (1LL << 31), "too many query tiles");
    // every barrier of the tile kernel's band walk orders LDS only (msda_bwd_mfma_wg_kernel's
    // bar() mask: the band's fire-and-forget atomics stay in flight across them)
    const int lbmask = 127;
    // VS_MSDA_SKEL: band skeleton variant (2, default: clear-after; 0: zero-fill + barrier
    // at every band start)
    int skel = kMsdaSkelDefault;
    if (const char* e = getenv("VS_MSDA_SKEL")) skel = atoi(e);
    // VS_MSDA_COL: the pyramid-column kernel's block at the finest level, "CYxCX" (default
    // 8x16: 3 chunks; 16x16 takes the 6-chunk build); 0: the 8 x 8 tile kernel
    int ccy = kMsdaColDefault[0], ccx = kMsdaColDefault[1];
    if (const char* e = getenv("VS_MSDA_COL")) {
      if (sscanf(e, "%dx%d", &ccy, &ccx) != 2) ccy = ccx = atoi(e);
    }
    ColGeo cg;
    const int nch = ccy > 0 && ccx > 0 ? col_geo(lv, L, ccy, ccx, &cg) : 0;
    const long long nbc = nch > 0 ? (long long)B * cg.per_image * Hh : 0;
    if (mfma && fused && bt.mode == 1 && nch > 0 && nbc < (1LL << 31) && (long long)S * Hh * kD < (1LL << 24)) {
      // VS_MSDA_WINT=0: the f32 W build with the points taking turns (A/B)
      const char* we = getenv("VS_MSDA_WINT");
      const bool wint = !(we && atoi(we) == 0);
#define VS_COL(NC_, WI_)                                                                                        \
  hipLaunchKernelGGL((msda_bwd_col_kernel<NC_, WI_>), dim3((unsigned)nbc), dim3(256), 0, st, loc, attw,          \
                     (const bf16*)gout, (const bf16*)value, gvalue, gloc, gattw, lv, cg, S, Hh, Q, L, (int)nbc)
      if (nch <= 3) {
        if (wint) VS_COL(3, true);
        else VS_COL(3, false);
      } else {
        if (wint) VS_COL(6, true);
        else VS_COL(6, false);
      }
#undef VS_COL
    } else if (mfma && fused && skel == 2)
      hipLaunchKernelGGL((msda_bwd_mfma_wg_kernel<8, 8, true, 2>), dim3((unsigned)nb2), dim3(256), 0, st, loc, attw,
                         (const bf16*)gout, gvalue, lv, bt, S, Hh, Q, L, (int)nb2, (const bf16*)value, gloc, gattw,
                         lbmask);
    else if (mfma && fused)
      hipLaunchKernelGGL((msda_bwd_mfma_wg_kernel<8, 8, true>), dim3((unsigned)nb2), dim3(256), 0, st, loc, attw,
                         (const bf16*)gout, gvalue, lv, bt, S, Hh, Q, L, (int)nb2, (const bf16*)value, gloc, gattw,
                         lbmask);
    else if (mfma)
      hipLaunchKernelGGL((msda_bwd_mfma_wg_kernel<8, 8, false>), dim3((unsigned)nb2), dim3(256), 0, st, loc, attw,
                         (const bf16*)gout, gvalue, lv, bt, S, Hh, Q, L, (int)nb2, (const bf16*)nullptr, nullptr,
                         nullptr, 0);
    else if (dtype == VS_BF16)
      hipLaunchKernelGGL((msda_bwd_binned_kernel<bf16, 4, 4>), dim3((unsigned)nb2), dim3(64), 0, st, loc, attw,
                         (const bf16*)gout, gvalue, lv, bt, S, Hh, Q, L, (int)nb2);
    else
      hipLaunchKernelGGL((msda_bwd_binned_kernel<float, 4, 4>), dim3((unsigned)nb2), dim3(64), 0, st, loc, attw,
                         (const float*)gout, gvalue, lv, bt, S, Hh, Q, L, (int)nb2);
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
  const int grid = (int)((groups * 32 + 255) / 256);
  if (dtype == VS_BF16)
    hipLaunchKernelGGL((msda_bwd_kernel<bf16>), dim3(grid), dim3(256), 0, st, (const bf16*)value, loc, attw,
                       (const bf16*)gout, gvalue, gloc, gattw, lv, S, Hh, Q, L, P, groups);
  else
    hipLaunchKernelGGL((msda_bwd_kernel<float>), dim3(grid), dim3(256), 0, st, (const float*)value, loc, attw,
                       (const float*)gout, gvalue, gloc, gattw, lv, S, Hh, Q, L, P, groups);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_msda_backward(int dtype, const void* value, const int64_t* shapes, const int64_t* starts,
                                const float* loc, const float* attw, const void* gout, float* gvalue, float* gloc,
                                float* gattw, int B, int S, int Hh, int D, int L, int Q, int P, void* stream) {
  return msda_backward_impl(dtype, value, shapes, starts, loc, attw, gout, gvalue, gloc, gattw, B, S, Hh, D, L, Q,
                            P, stream);
}

// The destination-tile backward that used this workspace (its far-tap list) measured slower
// than the column kernel and is gone (round 6); the entry point stays for ABI stability.
extern "C" long long vs_msda_backward_workspace_bytes(int B, int Q, int Hh, int L, int P) {
  if (B < 0 || Q < 0 || Hh < 0 || L < 0 || P < 0) return -1;
  return 0;
}

extern "C" int vs_msda_backward_ex(int dtype, const void* value, const int64_t* shapes, const int64_t* starts,
                                   const float* loc, const float* attw, const void* gout, float* gvalue, float* gloc,
                                   float* gattw, void* workspace, int B, int S, int Hh, int D, int L, int Q, int P,
                                   void* stream) {
  return msda_backward_impl(dtype, value, shapes, starts, loc, attw, gout, gvalue, gloc, gattw, B, S, Hh, D, L, Q,
                            P, stream, workspace);
}

// ---- tiled grad_value (default backward; see msda_tile_accum_kernel) ----------------
static void tile_geo(TileGeo* tg, const int* hs, const int* ws, int L, int Q, int P) {
  int base = 0;
  for (int l = 0; l < kMaxLevels; ++l) {
    tg->sh[l] = 3;
    tg->ntx[l] = tg->nty[l] = 0;
    tg->base[l] = base;
    if (l >= L) continue;
    const double density = (double)Q * P / ((double)hs[l] * ws[l]);
    const int sh = density <= 8.0 ? 3 : density <= 32.0 ? 2 : 1;
    const int te = 1 << sh;
    tg->sh[l] = sh;
    tg->ntx[l] = (ws[l] + te - 1) / te;
    tg->nty[l] = (hs[l] + te - 1) / te;
    base += tg->ntx[l] * tg->nty[l];
  }
  tg->base[kMaxLevels] = base;
  tg->per_bh = base;
}

// workspace: ctr [T] | local [T] | bsum [nb] | bprefix [nb + 1] | records [4 * taps]
static void tiled_layout(long long ntiles, long long taps, size_t* off) {
  const long long nb = (ntiles + kScanBlock - 1) / kScanBlock;
  off[0] = 0;
  off[1] = align256(off[0] + ntiles * 4);
  off[2] = align256(off[1] + ntiles * 4);
  off[3] = align256(off[2] + nb * 4);
  off[4] = align256(off[3] + (nb + 1) * 4);
  off[5] = align256(off[4] + (size_t)taps * 4 * 4);
}

static int tiled_sizes(const int64_t* shapes, int B, int Hh, int L, int Q, int P, TileGeo* tg, long long* ntiles,
                       long long* taps) {
  int hs[kMaxLevels], ws[kMaxLevels];
  for (int l = 0; l < L; ++l) {
    hs[l] = (int)shapes[2 * l];
    ws[l] = (int)shapes[2 * l + 1];
    if (hs[l] <= 0 || ws[l] <= 0) return 0;
  }
  tile_geo(tg, hs, ws, L, Q, P);
  *ntiles = (long long)B * Hh * tg->per_bh;
  *taps = (long long)B * Q * Hh * L * P;
  return *ntiles < (1LL << 30) && *taps * 4 < (1LL << 31);
}

extern "C" long long vs_msda_backward_tiled_workspace_bytes(int B, int Hh, int L, int Q, int P,
                                                            const int64_t* shapes) {
  if (B <= 0 || Hh <= 0 || L < 1 || L > kMaxLevels || Q < 0 || P <= 0 || !shapes) return -1;
  TileGeo tg;
  long long ntiles, taps;
  if (!tiled_sizes(shapes, B, Hh, L, Q, P, &tg, &ntiles, &taps)) return -1;
  size_t off[6];
  tiled_layout(ntiles, taps, off);
  return (long long)off[5];
}

extern "C" int vs_msda_backward_tiled(int dtype, const void* value, const int64_t* shapes, const int64_t* starts,
                                      const float* loc, const float* attw, const void* gout, void* gvalue,
                                      float* gloc, float* gattw, void* workspace, int B, int S, int Hh, int D, int L,
                                      int Q, int P, void* stream) {
  VS_CHECK(D == kD, "channels per head must be 32");
  VS_CHECK(L >= 1 && L <= kMaxLevels, "1..4 levels supported");
  VS_CHECK(B > 0 && S > 0 && Hh > 0 && Q >= 0 && P > 0, "bad sizes");
  VS_CHECK(value && gvalue && shapes && starts && workspace, "null pointer");
  VS_CHECK(Q == 0 || (loc && attw && gout && gloc && gattw), "null pointer");
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");
  Levels lv;
  VS_CHECK(fill_levels(&lv, shapes, starts, L, S), "spatial shapes / level starts inconsistent with S");
  TileGeo tg;
  long long ntiles, taps;
  VS_CHECK(tiled_sizes(shapes, B, Hh, L, Q, P, &tg, &ntiles, &taps), "problem too large for the tiled backward");
  hipStream_t st = (hipStream_t)stream;
  size_t off[6];
  tiled_layout(ntiles, taps, off);
  unsigned char* ws = (unsigned char*)workspace;
  int* ctr = (int*)(ws + off[0]);
  int* local = (int*)(ws + off[1]);
  int* bsum = (int*)(ws + off[2]);
  int* bprefix = (int*)(ws + off[3]);
  int* rec = (int*)(ws + off[4]);
  const int nb = (int)((ntiles + kScanBlock - 1) / kScanBlock);
  VS_HIP(hipMemsetAsync(ctr, 0, (size_t)ntiles * 4, st));
  if (taps > 0) {
    const int tgrid = (int)((taps + 255) / 256);
    hipLaunchKernelGGL(msda_tile_bucket_kernel<false>, dim3(tgrid), dim3(256), 0, st, loc, ctr, (const int*)nullptr,
                       (const int*)nullptr, (int*)nullptr, lv, tg, Hh, Q, L, P, taps);
  }
  hipLaunchKernelGGL(sort_scan_local_kernel, dim3(nb), dim3(256), 0, st, (const int*)ctr, local, bsum, ntiles);
  hipLaunchKernelGGL(sort_scan_blocks_kernel, dim3(1), dim3(1024), 0, st, (const int*)bsum, bprefix, nb);
  if (taps > 0) {
    VS_HIP(hipMemsetAsync(ctr, 0, (size_t)ntiles * 4, st));
    const int tgrid = (int)((taps + 255) / 256);
    hipLaunchKernelGGL(msda_tile_bucket_kernel<true>, dim3(tgrid), dim3(256), 0, st, loc, ctr, (const int*)local,
                       (const int*)bprefix, rec, lv, tg, Hh, Q, L, P, taps);
  }
  const int agrid = (int)((ntiles + 3) / 4);
  if (dtype == VS_BF16)
    hipLaunchKernelGGL(msda_tile_accum_kernel<bf16>, dim3(agrid), dim3(256), 0, st, loc, attw, (const bf16*)gout,
                       (const int*)local, (const int*)bprefix, (const int*)rec, (bf16*)gvalue, lv, tg, S, Hh, Q, L, P,
                       (int)ntiles);
  else
    hipLaunchKernelGGL(msda_tile_accum_kernel<float>, dim3(agrid), dim3(256), 0, st, loc, attw, (const float*)gout,
                       (const int*)local, (const int*)bprefix, (const int*)rec, (float*)gvalue, lv, tg, S, Hh, Q, L,
                       P, (int)ntiles);
  if (Q > 0) launch_geom(dtype, value, loc, attw, gout, gloc, gattw, lv, S, Hh, Q, L, P, (long long)B * Q * Hh, st);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
