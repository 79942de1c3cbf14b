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
// Backward, general queries (decoder cross-attention): one lane per channel (32 lanes =
// one group, 2 groups per wave) so every grad_value atomic wave-instruction is two
// contiguous 128-B row segments (the shape the f32 atomic path runs at full rate,
// MI355X_MICROARCH §Global float atomics); grad_loc / grad_attn are 32-lane shuffle
// reductions, written by lane 0.  That path is atomic-bound: 4 corners x 32 channels
// x 4 B per tap (4.2 GB per pixel-decoder layer at 4x1024^2).
//
// Backward, encoder self-attention (queries ARE the value grid, Q == S): grad_value is
// produced by destination instead.  msda_bwd_band_kernel owns a band of value rows of
// one (image, head, level) in LDS and gathers every tap landing there from the queries
// whose mapped row is within kBandR rows (LDS float atomics, then one plain coalesced
// store per element: no global atomics); the query kernel computes grad_loc /
// grad_attn and atomically adds only the "far" corners (row beyond the margin), which
// the shared integer predicate `near_row` assigns to exactly one of the two kernels.
// Measured on MI355X (4x1024^2, 8 heads, tools/kbench.py): band 7.65 ms + query 1.24 ms
// vs 3.08 ms for the all-atomic path — LDS float atomics (ds_add_f32) on this access
// pattern cost ~6 ms (a non-atomic LDS RMW probe: ~0.2 ms), the latency-bound scan the
// other ~1.3 ms.  The band path is therefore opt-in (encoder=True) until it wins.
#include "common.h"

namespace vs {
namespace {

constexpr int kD = 32;
constexpr int kMaxLevels = 4;

struct Levels {
  int h[kMaxLevels];
  int w[kMaxLevels];
  int start[kMaxLevels];
};


// ---- backward helpers shared by the band and query kernels (must stay identical:
// a corner is accumulated by exactly one of them, decided by `near_row`).
constexpr int kBandR = 4;      // row margin (level-l rows) of the band kernel's query scan; covers the
                               // Deformable-DETR init offsets (|off| <= 4 px); farther taps go atomic
constexpr int kBandMaxRows = 8;     // value rows per band workgroup (fewer if the level is wide)
constexpr int kBandThreads = 1024;  // 32 query slots of 32 channel-lanes
constexpr int kBandUnroll = 4;      // queries in flight per slot (loads hoisted ahead of the LDS adds)

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

// Row of level l (height Hl) onto which query row yq of level lq (height Hq) maps:
// floor(((yq + 0.5) * Hl / Hq) - 0.5), integer arithmetic (exact, no fp ambiguity).
__device__ __forceinline__ int mapped_row(int yq, int Hq, int Hl) {
  const int num = (2 * yq + 1) * Hl - Hq;
  const int den = 2 * Hq;
  return num >= 0 ? num / den : -((-num + den - 1) / den);
}

__device__ __forceinline__ bool near_row(int cy, int m) { return cy >= m - kBandR && cy <= m + kBandR + 1; }

template <typename T>
__global__ void __launch_bounds__(256) msda_fwd_kernel(const T* __restrict__ value,
                                                        const float* __restrict__ loc,
                                                        const float* __restrict__ attw,
                                                        T* __restrict__ out, Levels lv, int S,
                                                        int Hh, int Q, int L, int P,
                                                        long long groups) {
  constexpr int V = Vec16<T>::N;       // channels per lane
  constexpr int LPG = kD / V;          // lanes per group
  long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
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

template <typename T, bool ENC>
__global__ void __launch_bounds__(256) msda_bwd_kernel(
    const T* __restrict__ value, const float* __restrict__ loc, const float* __restrict__ attw,
    const T* __restrict__ gout, float* __restrict__ gvalue, float* __restrict__ gloc,
    float* __restrict__ gattw, Levels lv, int S, int Hh, int Q, int L, int P, long long groups) {
  // lane = channel, 32 lanes per (b, q, head).  ENC: queries are the value grid itself
  // (encoder self-attention, Q == S level-major): near corners are accumulated by
  // msda_bwd_band_kernel, only far corners (|row - mapped row| beyond the margin) are
  // added here with atomics.  !ENC: every corner is an atomic add.
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long grp = gid >> 5;
  const int c = (int)(gid & 31);
  if (grp >= groups) return;  // uniform per 32-lane half-wave
  const int LP = L * P;
  const int h = (int)(grp % Hh);
  const long long bq = grp / Hh;
  const int q = (int)(bq % Q);
  const long long b = bq / Q;
  int lq = 0, yq = 0, Hq = 1;
  if (ENC) {
    while (lq + 1 < L && q >= lv.start[lq + 1]) ++lq;
    yq = (q - lv.start[lq]) / lv.w[lq];
    Hq = lv.h[lq];
  }
  const float* lp = loc + grp * LP * 2;
  const float* wp = attw + grp * LP;
  const size_t rowstride = (size_t)Hh * kD;
  const size_t vbase = ((size_t)b * S * Hh + h) * kD + c;
  const float g = to_f32(gout[grp * kD + c]);
  for (int l = 0; l < L; ++l) {
    const int Hl = lv.h[l], Wl = lv.w[l];
    const size_t lbase = vbase + (size_t)lv.start[l] * rowstride;
    const float fH = (float)Hl, fW = (float)Wl;
    const int m = ENC ? mapped_row(yq, Hq, Hl) : 0;
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
        const bool far0 = !ENC || !near_row(h0, m);
        const bool far1 = !ENC || !near_row(h0 + 1, m);
        if (h0 >= 0 && w0 >= 0) {
          const size_t o = lbase + (size_t)(h0 * Wl + w0) * rowstride;
          v1 = to_f32(value[o]);
          if (far0) atomicAdd(gvalue + o, hh * hw * ga);
        }
        if (h0 >= 0 && w0 + 1 <= Wl - 1) {
          const size_t o = lbase + (size_t)(h0 * Wl + w0 + 1) * rowstride;
          v2 = to_f32(value[o]);
          if (far0) atomicAdd(gvalue + o, hh * lw * ga);
        }
        if (h0 + 1 <= Hl - 1 && w0 >= 0) {
          const size_t o = lbase + (size_t)((h0 + 1) * Wl + w0) * rowstride;
          v3 = to_f32(value[o]);
          if (far1) atomicAdd(gvalue + o, lh * hw * ga);
        }
        if (h0 + 1 <= Hl - 1 && w0 + 1 <= Wl - 1) {
          const size_t o = lbase + (size_t)((h0 + 1) * Wl + w0 + 1) * rowstride;
          v4 = to_f32(value[o]);
          if (far1) atomicAdd(gvalue + o, lh * lw * ga);
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

// Backward, default path: two kernels.
//
// (1) msda_bwd_geom_kernel — grad_attn / grad_loc.  Gather-only, laid out like the
//     forward (a lane owns a 16-B channel slice, 4 (bf16) / 8 (f32) lanes per (b,q,head)),
//     partial dot products reduced over the group's lanes with shuffles.
//
// (2) msda_bwd_scatter_kernel — grad_value, with a register carry.  A half-wave (32
//     lanes = the 32 channels of one head) walks a run of R consecutive queries of one
//     (image, head).  For every tap (level l, point p) it holds the 2x2 block of corners
//     it touched last: 4 per-lane f32 sums and the block's top-left cell.  When the next
//     query's tap lands on a block overlapping the held one (cell offset dx, dy in
//     {-1,0,1}), the shared corners stay in registers and only the corners leaving the
//     block are added to HBM (f32 atomics); a disjoint block flushes all four.  Same sum
//     as one atomic per corner, in a different order.
//
// Why: grad_value is bound by the chip's float-atomic rate (~1.3 TB/s of added bytes,
// MI355X_MICROARCH §Global float atomics): 4 corners x 32 ch x 4 B per tap, 4.2 GB per
// pixel-decoder layer at 4x1024^2.  In the encoder, consecutive queries are horizontally
// adjacent pixels whose (smoothly varying) sampling points move by 1 cell on their own
// level and 1/2, 1/4 cell on coarser ones, so about half the corner adds are shared with
// the previous query (tools/kbench.py "smooth").  Loads and no-return atomics retire in
// order through one counter (vmcnt), so a load issued after an atomic waits for it: the
// scatter kernel therefore stages its run's loc / attn / grad_out in LDS first and its
// query loop issues nothing but LDS reads and atomics.  Unrelated queries (a decoder)
// degrade to one add per corner.
template <typename T>
__global__ void __launch_bounds__(256) msda_bwd_geom_kernel(
    const T* __restrict__ value, const float* __restrict__ loc, const float* __restrict__ attw,
    const T* __restrict__ gout, float* __restrict__ gloc, float* __restrict__ gattw, Levels lv, int S,
    int Hh, int Q, int L, int P, long long groups) {
  constexpr int V = Vec16<T>::N;       // channels per lane
  constexpr int LPG = kD / V;          // lanes per group (4 bf16, 8 f32), a power of two
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long grp = gid / LPG;
  const int sub = (int)(gid % LPG);
  if (grp >= groups) return;           // groups are aligned to LPG lanes: uniform per group
  const int LP = L * P;
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
        gattw[grp * LP + t] = r_w;
        gloc[(grp * LP + t) * 2 + 0] = r_x;
        gloc[(grp * LP + t) * 2 + 1] = r_y;
      }
    }
  }
}

constexpr int kScatterRun = 32;        // queries per half-wave run (LDS staging is sized for it)

template <typename T, int L, int P>
__global__ void __launch_bounds__(256) msda_bwd_scatter_kernel(
    const float* __restrict__ loc, const float* __restrict__ attw, const T* __restrict__ gout,
    float* __restrict__ gvalue, Levels lv, int S, int Hh, int Q, int R, int nrun, long long halfwaves) {
  constexpr int LP = L * P;
  // per half-wave staging: loc [R][LP][2], attn [R][LP], grad_out [R][32] (f32)
  constexpr int kStage = kScatterRun * (LP * 3 + kD);
  __shared__ float stage[8][kStage];
  const int hwl = threadIdx.x >> 5;           // half-wave within the workgroup
  const long long hw_id = (long long)blockIdx.x * 8 + hwl;
  const int c = threadIdx.x & 31;
  if (hw_id >= halfwaves) return;             // uniform per half-wave; no block-wide barrier below
  const int h = (int)(hw_id % Hh);
  const long long br = hw_id / Hh;
  const int run = (int)(br % nrun);
  const long long b = br / nrun;
  const int q0 = run * R;
  const int nq = min(Q, q0 + R) - q0;
  float* sl = stage[hwl];
  float* sw = sl + kScatterRun * LP * 2;
  float* sg = sw + kScatterRun * LP;
  for (int i = 0; i < nq; ++i) {
    const long long grp = ((long long)b * Q + q0 + i) * Hh + h;
    if (c < LP * 2) sl[i * LP * 2 + c] = loc[grp * LP * 2 + c];
    if (c < LP) sw[i * LP + c] = attw[grp * LP + c];
    sg[i * kD + c] = to_f32(gout[grp * kD + c]);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  const size_t rowstride = (size_t)Hh * kD;
  const size_t vbase = ((size_t)b * S * Hh + h) * kD + c;
  int ph[LP], pw[LP];                         // held block's top-left cell per tap
  float acc[LP][4];                           // held corner sums: (0,0) (0,1) (1,0) (1,1)
#pragma unroll
  for (int t = 0; t < LP; ++t) {
    ph[t] = -(1 << 28);
    pw[t] = -(1 << 28);
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[t][k] = 0.f;
  }
  auto flush = [&](int t, int k, int Hl, int Wl, size_t lbase) {
    const int y = ph[t] + (k >> 1), x = pw[t] + (k & 1);
    if (y >= 0 && y < Hl && x >= 0 && x < Wl)
      atomicAdd(gvalue + lbase + (size_t)(y * Wl + x) * rowstride, acc[t][k]);
  };
  for (int i = 0; i < nq; ++i) {
    const float g = sg[i * kD + c];
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const int Hl = lv.h[l], Wl = lv.w[l];
      const size_t lbase = vbase + (size_t)lv.start[l] * rowstride;
#pragma unroll
      for (int p = 0; p < P; ++p) {
        const int t = l * P + p;
        const Tap tg = tap_geom(sl[(i * LP + t) * 2 + 0], sl[(i * LP + t) * 2 + 1], Hl, Wl);
        if (!tg.inside) continue;             // no contribution; the held block stays
        const float ga = g * sw[i * LP + t];
        const int dy = tg.h0 - ph[t], dx = tg.w0 - pw[t];
        // held corner k = (cy, cx) survives iff (cy - dy, cx - dx) lies in the new block
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int ny = (k >> 1) - dy, nx = (k & 1) - dx;
          if (!((unsigned)ny <= 1u && (unsigned)nx <= 1u)) flush(t, k, Hl, Wl, lbase);
        }
        float carried[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int sy = (k >> 1) + dy, sx = (k & 1) + dx;
          const int s = sy * 2 + sx;
          const bool in = (unsigned)sy <= 1u && (unsigned)sx <= 1u;
          carried[k] = !in ? 0.f : s == 0 ? acc[t][0] : s == 1 ? acc[t][1] : s == 2 ? acc[t][2] : acc[t][3];
        }
        // corners outside the level get sums too but are never flushed
        acc[t][0] = carried[0] + tg.hh * tg.hw * ga;
        acc[t][1] = carried[1] + tg.hh * tg.lw * ga;
        acc[t][2] = carried[2] + tg.lh * tg.hw * ga;
        acc[t][3] = carried[3] + tg.lh * tg.lw * ga;
        ph[t] = tg.h0;
        pw[t] = tg.w0;
      }
    }
  }
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const size_t lbase = vbase + (size_t)lv.start[l] * rowstride;
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
      for (int k = 0; k < 4; ++k) flush(l * P + p, k, lv.h[l], lv.w[l], lbase);
  }
}

// grad_value by destination band (encoder mode).  One workgroup = (band of kBandRows
// rows of level lb, head h, image b); the band's [rows][W][32] f32 accumulator lives in
// LDS.  The workgroup scans every query (of every level) whose mapped row on level lb
// lies within kBandR of the band, evaluates its taps on level lb, and adds the corners
// that fall in the band AND are `near` their query (the complement of the query
// kernel's far set) with LDS float atomics; the band is then written with plain
// coalesced stores.  Waves walk queries; lane = channel; 2 queries per wave.
template <typename T>
__global__ void __launch_bounds__(kBandThreads) msda_bwd_band_kernel(
    const float* __restrict__ loc, const float* __restrict__ attw, const T* __restrict__ gout,
    float* __restrict__ gvalue, Levels lv, int S, int Hh, int L, int P, int band_rows) {
  extern __shared__ __attribute__((aligned(16))) float sacc[];
  // decode (level, band) from blockIdx.x
  int bx = blockIdx.x, lb = 0;
  while (lb + 1 < L && bx >= (lv.h[lb] + band_rows - 1) / band_rows) { bx -= (lv.h[lb] + band_rows - 1) / band_rows; ++lb; }
  const int h = blockIdx.y;
  const long long b = blockIdx.z;
  const int Hl = lv.h[lb], Wl = lv.w[lb];
  const int y0 = bx * band_rows;
  const int y1 = min(Hl, y0 + band_rows);  // exclusive
  const int nrows = y1 - y0;
  const int LP = L * P;
  for (int i = threadIdx.x; i < nrows * Wl * kD; i += blockDim.x) sacc[i] = 0.f;
  __syncthreads();
  const int c = threadIdx.x & 31;
  const int slot = threadIdx.x >> 5;          // 16 query slots per workgroup
  constexpr int kSlots = kBandThreads / 32;
  for (int lq = 0; lq < L; ++lq) {
    const int Hq = lv.h[lq], Wq = lv.w[lq];
    // query rows whose mapped row m satisfies y0-R-1 <= m <= y1-1+R (m monotone in yq)
    int ylo = 0, yhi = -1;
    {
      int lo = Hq, hi = -1;
      for (int yq = 0; yq < Hq; ++yq) {
        const int m = mapped_row(yq, Hq, Hl);
        if (m >= y0 - kBandR - 1 && m <= y1 - 1 + kBandR) { lo = min(lo, yq); hi = max(hi, yq); }
      }
      ylo = lo; yhi = hi;
    }
    if (yhi < ylo) continue;
    const int nq = (yhi - ylo + 1) * Wq;
    const int qbase = lv.start[lq] + ylo * Wq;
    for (int q0 = slot * kBandUnroll; q0 < nq; q0 += kSlots * kBandUnroll) {
      float4 la[kBandUnroll], lb4[kBandUnroll], wv[kBandUnroll];
      float gg[kBandUnroll];
      int mm[kBandUnroll];
#pragma unroll
      for (int u = 0; u < kBandUnroll; ++u) {
        const int qi = min(q0 + u, nq - 1);
        const int q = qbase + qi;
        mm[u] = mapped_row(ylo + qi / Wq, Hq, Hl);
        const long long grp = (b * S + q) * Hh + h;
        const float4* lp4 = reinterpret_cast<const float4*>(loc + grp * LP * 2 + lb * P * 2);
        la[u] = lp4[0];
        lb4[u] = lp4[1];
        wv[u] = *reinterpret_cast<const float4*>(attw + grp * LP + lb * P);
        gg[u] = (q0 + u < nq) ? to_f32(gout[grp * kD + c]) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kBandUnroll; ++u) {
        const float xs[4] = {la[u].x, la[u].z, lb4[u].x, lb4[u].z};
        const float ys[4] = {la[u].y, la[u].w, lb4[u].y, lb4[u].w};
        const float ws4[4] = {wv[u].x, wv[u].y, wv[u].z, wv[u].w};
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const Tap t = tap_geom(xs[p], ys[p], Hl, Wl);
          if (!t.inside) continue;
          const float ga = gg[u] * ws4[p];
          const int h0 = t.h0, w0 = t.w0;
#pragma unroll
          for (int dy = 0; dy < 2; ++dy) {
            const int cy = h0 + dy;
            if (cy < y0 || cy >= y1 || cy > Hl - 1 || !near_row(cy, mm[u])) continue;
            const float wy = dy ? t.lh : t.hh;
            float* row = sacc + ((cy - y0) * Wl) * kD + c;
            if (w0 >= 0) atomicAdd(row + w0 * kD, wy * t.hw * ga);
            if (w0 + 1 <= Wl - 1) atomicAdd(row + (w0 + 1) * kD, wy * t.lw * ga);
          }
        }
      }
    }
  }
  __syncthreads();
  const size_t rowstride = (size_t)Hh * kD;
  float* dst = gvalue + ((size_t)b * S * Hh + h) * kD + (size_t)(lv.start[lb] + y0 * Wl) * rowstride;
  for (int i = threadIdx.x; i < nrows * Wl * kD; i += blockDim.x) {
    const int px = i / kD, cc = i - px * kD;
    dst[(size_t)px * rowstride + cc] = sacc[i];
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

extern "C" int vs_msda_forward(int dtype, const void* value, const int64_t* shapes,
                               const int64_t* starts, const float* loc, const float* attw,
                               void* out, int B, int S, int Hh, int D, int L, int Q, int P,
                               void* stream) {
  VS_CHECK(D == kD, "channels per head must be 32");
  VS_CHECK(L >= 1 && L <= kMaxLevels, "1..4 levels supported");
  VS_CHECK(B > 0 && S > 0 && Hh > 0 && Q >= 0 && P > 0, "bad sizes");
  VS_CHECK(value && loc && attw && out && shapes && starts, "null pointer");
  Levels lv;
  VS_CHECK(fill_levels(&lv, shapes, starts, L, S), "spatial shapes / level starts inconsistent with S");
  if (Q == 0) return VS_OK;
  hipStream_t st = (hipStream_t)stream;
  const long long groups = (long long)B * Q * Hh;
  const int block = 256;
  if (dtype == VS_BF16) {
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

static int msda_backward_impl(int dtype, const void* value, const int64_t* shapes, const int64_t* starts,
                              const float* loc, const float* attw, const void* gout, float* gvalue, float* gloc,
                              float* gattw, int B, int S, int Hh, int D, int L, int Q, int P, void* stream,
                              bool encoder) {
  VS_CHECK(D == kD, "channels per head must be 32");
  VS_CHECK(L >= 1 && L <= kMaxLevels, "1..4 levels supported");
  VS_CHECK(B > 0 && S > 0 && Hh > 0 && Q >= 0 && P > 0, "bad sizes");
  VS_CHECK(value && loc && attw && gout && gvalue && gloc && gattw && shapes && starts, "null pointer");
  Levels lv;
  VS_CHECK(fill_levels(&lv, shapes, starts, L, S), "spatial shapes / level starts inconsistent with S");
  VS_CHECK(!encoder || Q == S, "encoder mode needs the queries to be the value grid (Q == S)");
  VS_CHECK(!encoder || P == 4, "encoder-mode backward is specialised for 4 sampling points");
  hipStream_t st = (hipStream_t)stream;
  const long long groups = (long long)B * Q * Hh;
  const int block = 256;
  const long long threads = groups * 32;
  const int grid = (int)((threads + block - 1) / block);
  if (encoder) {
    int maxw = 0, bands = 0;
    for (int l = 0; l < L; ++l) maxw = max(maxw, lv.w[l]);
    const int band_rows = min(kBandMaxRows, (int)((160 * 1024) / ((size_t)maxw * kD * sizeof(float))));
    VS_CHECK(band_rows >= 1, "level too wide for the band kernel");
    for (int l = 0; l < L; ++l) bands += (lv.h[l] + band_rows - 1) / band_rows;
    const size_t lds = (size_t)band_rows * maxw * kD * sizeof(float);
    dim3 bgrid(bands, Hh, B);
    if (dtype == VS_BF16) {
      hipLaunchKernelGGL(msda_bwd_band_kernel<bf16>, bgrid, dim3(kBandThreads), lds, st, loc, attw, (const bf16*)gout,
                         gvalue, lv, S, Hh, L, P, band_rows);
      hipLaunchKernelGGL((msda_bwd_kernel<bf16, true>), dim3(grid), dim3(block), 0, st, (const bf16*)value, loc, attw,
                         (const bf16*)gout, gvalue, gloc, gattw, lv, S, Hh, Q, L, P, groups);
    } else if (dtype == VS_F32) {
      hipLaunchKernelGGL(msda_bwd_band_kernel<float>, bgrid, dim3(kBandThreads), lds, st, loc, attw,
                         (const float*)gout, gvalue, lv, S, Hh, L, P, band_rows);
      hipLaunchKernelGGL((msda_bwd_kernel<float, true>), dim3(grid), dim3(block), 0, st, (const float*)value, loc,
                         attw, (const float*)gout, gvalue, gloc, gattw, lv, S, Hh, Q, L, P, groups);
    } else {
      VS_CHECK(false, "dtype must be VS_F32 or VS_BF16");
    }
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
  VS_HIP(hipMemsetAsync(gvalue, 0, sizeof(float) * (size_t)B * S * Hh * kD, st));
  if (Q == 0) return VS_OK;
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");
  // geom + register-carry scatter when there are enough queries for runs to fill the chip
  // (VS_MSDA_RUN=n forces runs of n <= 32 queries at any size, 0 the single kernel)
  int run = kScatterRun;
  bool split = (long long)B * Q * Hh >= (long long)kScatterRun * 8192;
  if (const char* e = getenv("VS_MSDA_RUN")) {
    run = atoi(e);
    split = run >= 1;
  }
  if (split && P == 4) {
    VS_CHECK(run <= kScatterRun, "VS_MSDA_RUN must be <= 32");
    const int lpg = dtype == VS_BF16 ? 4 : 8;
    const int ggrid = (int)((groups * lpg + block - 1) / block);
    if (dtype == VS_BF16)
      hipLaunchKernelGGL(msda_bwd_geom_kernel<bf16>, dim3(ggrid), dim3(block), 0, st, (const bf16*)value, loc,
                         attw, (const bf16*)gout, gloc, gattw, lv, S, Hh, Q, L, P, groups);
    else
      hipLaunchKernelGGL(msda_bwd_geom_kernel<float>, dim3(ggrid), dim3(block), 0, st, (const float*)value, loc,
                         attw, (const float*)gout, gloc, gattw, lv, S, Hh, Q, L, P, groups);
    const int nrun = (Q + run - 1) / run;
    const long long hws = (long long)B * nrun * Hh;
    const int sgrid = (int)((hws + 7) / 8);
#define VS_SCATTER(TT, LL)                                                                                 \
  hipLaunchKernelGGL((msda_bwd_scatter_kernel<TT, LL, 4>), dim3(sgrid), dim3(block), 0, st, loc, attw,      \
                     (const TT*)gout, gvalue, lv, S, Hh, Q, run, nrun, hws)
#define VS_SCATTER_L(TT)                \
  switch (L) {                          \
    case 1: VS_SCATTER(TT, 1); break;   \
    case 2: VS_SCATTER(TT, 2); break;   \
    case 3: VS_SCATTER(TT, 3); break;   \
    default: VS_SCATTER(TT, 4); break;  \
  }
    if (dtype == VS_BF16) {
      VS_SCATTER_L(bf16)
    } else {
      VS_SCATTER_L(float)
    }
#undef VS_SCATTER_L
#undef VS_SCATTER
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
  if (dtype == VS_BF16) {
    hipLaunchKernelGGL((msda_bwd_kernel<bf16, false>), dim3(grid), dim3(block), 0, st, (const bf16*)value, loc, attw,
                       (const bf16*)gout, gvalue, gloc, gattw, lv, S, Hh, Q, L, P, groups);
  } else if (dtype == VS_F32) {
    hipLaunchKernelGGL((msda_bwd_kernel<float, false>), dim3(grid), dim3(block), 0, st, (const float*)value, loc,
                       attw, (const float*)gout, gvalue, gloc, gattw, lv, S, Hh, Q, L, P, groups);
  } else {
    VS_CHECK(false, "dtype must be VS_F32 or VS_BF16");
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_msda_backward(int dtype, const void* value, const int64_t* shapes, const int64_t* starts,
                                const float* loc, const float* attw, const void* gout, float* gvalue, float* gloc,
                                float* gattw, int B, int S, int Hh, int D, int L, int Q, int P, void* stream) {
  return msda_backward_impl(dtype, value, shapes, starts, loc, attw, gout, gvalue, gloc, gattw, B, S, Hh, D, L, Q,
                            P, stream, false);
}

extern "C" int vs_msda_backward_encoder(int dtype, const void* value, const int64_t* shapes, const int64_t* starts,
                                        const float* loc, const float* attw, const void* gout, float* gvalue,
                                        float* gloc, float* gattw, int B, int S, int Hh, int D, int L, int P,
                                        void* stream) {
  return msda_backward_impl(dtype, value, shapes, starts, loc, attw, gout, gvalue, gloc, gattw, B, S, Hh, D, L, S,
                            P, stream, true);
}
