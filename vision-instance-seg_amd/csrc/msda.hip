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
// Backward, general queries (decoder cross-attention, or whenever the encoder path
// does not apply): grad_loc / grad_attn from a gather kernel (msda_bwd_geom_kernel) and
// grad_value from a scatter kernel with a register carry (msda_bwd_scatter_kernel; see
// there).  Small problems use the single fused kernel (msda_bwd_kernel, one f32 atomic
// per corner).  grad_value is bound by the float-atomic rate (~1.3 TB/s of added bytes,
// MI355X_MICROARCH §Global float atomics).
//
// Backward, encoder self-attention (queries ARE the value grid, Q == S, level-major),
// opt-in (encoder=True): grad_value is first PULLED by destination
// (msda_bwd_pull_kernel): a wave owns a 4x16 block of value cells of one (image, head,
// level l), enumerates the queries of levels not finer than l whose reference point
// maps within R0 cells of the block (an implicit inverse index: the queries are the
// grid), stages their taps and grad_out rows in LDS and accumulates each cell's 32
// channels in registers; every grad_value element is written once with a plain store.
// The carry scatter kernel then adds every other tap (finer query levels, or farther
// than R0 cells) with atomics; pull_tap() assigns each tap to exactly one of the two.
// Measured at 4x1024^2 (tools/msda_probe.py, smooth offsets, R0 = 5): pull 0.9 ms +
// scatter 2.1 ms + geom 0.36 ms, against geom + carry scatter ~2.0 ms for the default
// path — the remaining atomics pile onto the small coarse levels and the per-query level
// decode costs integer divisions — so the model uses the default path.
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


// ---- backward helpers shared by the tile and scatter kernels (must stay identical: a
// tap is accumulated by exactly one of them, decided by `near_tap`).
constexpr int kNearR = 5;           // default near margin R0 of the tile kernel (VS_MSDA_NEAR_R)

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

// Cell of level l (extent nl) onto which query coordinate xq of level lq (extent nq)
// maps: floor((xq + 0.5) * nl / nq - 0.5), integer arithmetic (exact, no fp ambiguity).
__host__ __device__ __forceinline__ int mapped_cell(int xq, int nq, int nl) {
  const int num = (2 * xq + 1) * nl - nq;
  const int den = 2 * nq;
  return num >= 0 ? num / den : -((-num + den - 1) / den);
}

// a tap belongs to the tile kernel ("near") iff it is inside and its top-left cell is
// within R0 cells (both axes) of the query's mapped cell on the tap's level; every other
// tap is added by the scatter kernel
__device__ __forceinline__ bool near_tap(const Tap& t, int mcy, int mcx, int R0) {
  return t.inside && abs(t.h0 - mcy) <= R0 && abs(t.w0 - mcx) <= R0;
}

__device__ __forceinline__ int ceil_div(int a, int b) { return a >= 0 ? (a + b - 1) / b : -((-a) / b); }

// exact range of query coordinates x (level extent nq) whose mapped cell on a level of
// extent nl lies in [lo, hi]:  mapped_cell(x) >= lo  <=>  x >= ceil(((2lo+1)nq - nl) / 2nl)
__device__ __forceinline__ void mapped_range(int lo, int hi, int nq, int nl, int* xa, int* xb) {
  *xa = max(0, ceil_div((2 * lo + 1) * nq - nl, 2 * nl));
  *xb = min(nq - 1, ceil_div((2 * hi + 3) * nq - nl, 2 * nl) - 1);
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

constexpr int kScatterRun = 16;        // queries per half-wave run (LDS staging is sized for it)

// ENC (encoder mode, Q == S level-major): near taps (near_tap) are skipped here; the
// tile kernel has already written every grad_value element.
template <typename T, int L, int P, bool ENC>
__global__ void __launch_bounds__(256) msda_bwd_scatter_kernel(
    const float* __restrict__ loc, const float* __restrict__ attw, const T* __restrict__ gout,
    float* __restrict__ gvalue, Levels lv, int S, int Hh, int Q, int R, int nrun, long long halfwaves, int R0) {
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
    int lq = 0, yq = 0, xq = 0;
    if (ENC) {
      const int q = q0 + i;
      while (lq + 1 < L && q >= lv.start[lq + 1]) ++lq;
      yq = (q - lv.start[lq]) / lv.w[lq];
      xq = (q - lv.start[lq]) % lv.w[lq];
    }
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const int Hl = lv.h[l], Wl = lv.w[l];
      const size_t lbase = vbase + (size_t)lv.start[l] * rowstride;
#pragma unroll
      for (int p = 0; p < P; ++p) {
        const int t = l * P + p;
        const Tap tg = tap_geom(sl[(i * LP + t) * 2 + 0], sl[(i * LP + t) * 2 + 1], Hl, Wl);
        if (!tg.inside) continue;             // no contribution; the held block stays
        if (ENC && near_tap(tg, mapped_cell(yq, lv.h[lq], Hl), mapped_cell(xq, lv.w[lq], Wl), R0)) continue;
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

// grad_value by destination tile (encoder mode; see the header).  Block = (16x16 cell
// tile of level l, head, image); the tile's 256 cells x 32 channels are accumulated in
// LDS (32 KB f32).  For every query level lq the block enumerates the rectangle of
// queries whose mapped cell on level l lies within R0 cells of a corner block touching
// the tile (mapped_range), 16 queries per wave at a time: lane = (query, point) computes
// the tap on level l, keeps it if near_tap() and one of its four corners is in the tile,
// and the kept taps are compacted (wave ballot) into a per-wave list with the query's
// grad_out row staged in LDS.  Then the two half-waves walk the list with lane = channel
// and add weight * grad_out into the tile with LDS float atomics (32 consecutive floats
// per half-wave: conflict-free).  Far taps are left to the scatter kernel.  Finally every
// cell of the tile is stored once (plain f32 stores; the scatter adds on top).
//
// Work per tile grows with the number of queries mapping into its window, so coarse
// levels (whose window holds the finer levels' queries) cost more per tile: the block
// order is tile-major with the coarsest level first (longest jobs start first), and the
// heads of one (tile, image) are consecutive workgroups of one XCD (their loc / grad_out
// rows share cache lines).
constexpr int kTile = 16;

struct TileOrder {
  int level[kMaxLevels];      // levels by ascending cell count (coarsest first)
  int prefix[kMaxLevels + 1]; // tile-slot prefix over that order (slots = tiles x images)
  int slots;                  // total (tile, image) slots
};

template <typename T>
__global__ void __launch_bounds__(256) msda_bwd_tile_kernel(const float* __restrict__ loc,
                                                            const float* __restrict__ attw,
                                                            const T* __restrict__ gout, float* __restrict__ gvalue,
                                                            Levels lv, int S, int Hh, int B, int L, int R0,
                                                            TileOrder to) {
  constexpr int P = 4;
  __shared__ __attribute__((aligned(16))) float sAcc[kTile * kTile * kD];
  __shared__ int4 sCell[4][64];
  __shared__ float4 sWgt[4][64];
  __shared__ int sQ[4][64];
  __shared__ __attribute__((aligned(16))) float sG[4][16][kD];
  // physical id -> (slot, head): workgroup i runs on XCD i % 8; heads of one slot are
  // consecutive workgroups of that XCD, slots advance in order (coarsest level first)
  const int i = blockIdx.x;
  const int xcd = i & 7, j = i >> 3;
  const int h = j % Hh;
  const int slot = (j / Hh) * 8 + xcd;
  if (slot >= to.slots) return;                     // padding (uniform per block)
  int oi = 0;
  while (oi + 1 < L && slot >= to.prefix[oi + 1]) ++oi;
  const int l = to.level[oi];
  const int local = slot - to.prefix[oi];
  const int b = local % B, t = local / B;
  const int Hl = lv.h[l], Wl = lv.w[l];
  const int txn = (Wl + kTile - 1) / kTile;
  const int ty0 = (t / txn) * kTile, tx0 = (t % txn) * kTile;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int LP = L * P;

  for (int k = tid; k < kTile * kTile * kD / 4; k += 256)
    reinterpret_cast<float4*>(sAcc)[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();

  const int half = lane >> 5, c = lane & 31;
  for (int lq = 0; lq < L; ++lq) {
    const int Hq = lv.h[lq], Wq = lv.w[lq];
    // a near tap's top-left cell is within R0 of the query's mapped cell; its corner
    // block touches the tile iff the top-left cell is in [tile0 - 1, tile0 + 15]
    int ya, yb, xa, xb;
    mapped_range(ty0 - 1 - R0, ty0 + kTile - 1 + R0, Hq, Hl, &ya, &yb);
    mapped_range(tx0 - 1 - R0, tx0 + kTile - 1 + R0, Wq, Wl, &xa, &xb);
    if (ya > yb || xa > xb) continue;
    const int nx = xb - xa + 1;
    const int ncand = (yb - ya + 1) * nx;
    for (int base = wave * 16; base < ncand; base += 64) {
      // ---- geometry: lane = (query base + lane/4, point lane%4)
      const int qi = base + (lane >> 2), p = lane & 3;
      int4 cell = make_int4(-1, -1, -1, -1);
      float4 wgt = make_float4(0.f, 0.f, 0.f, 0.f);
      bool keep = false;
      long long grp = 0;
      if (qi < ncand) {
        const int yq = ya + qi / nx, xq = xa + qi % nx;
        grp = ((long long)b * S + lv.start[lq] + yq * Wq + xq) * Hh + h;
        const int mcy = mapped_cell(yq, Hq, Hl), mcx = mapped_cell(xq, Wq, Wl);
        const float2 xy = *reinterpret_cast<const float2*>(loc + (grp * LP + l * P + p) * 2);
        const float a = attw[grp * LP + l * P + p];
        const Tap tg = tap_geom(xy.x, xy.y, Hl, Wl);
        if (near_tap(tg, mcy, mcx, R0)) {
          const int ry0 = tg.h0 - ty0, rx0 = tg.w0 - tx0;
          const bool y0in = (unsigned)ry0 < (unsigned)kTile && tg.h0 >= 0;
          const bool y1in = (unsigned)(ry0 + 1) < (unsigned)kTile && tg.h0 + 1 < Hl;
          const bool x0in = (unsigned)rx0 < (unsigned)kTile && tg.w0 >= 0;
          const bool x1in = (unsigned)(rx0 + 1) < (unsigned)kTile && tg.w0 + 1 < Wl;
          const int base_cell = (ry0 * kTile + rx0) * kD;
          cell.x = y0in && x0in ? base_cell : -1;
          cell.y = y0in && x1in ? base_cell + kD : -1;
          cell.z = y1in && x0in ? base_cell + kTile * kD : -1;
          cell.w = y1in && x1in ? base_cell + (kTile + 1) * kD : -1;
          wgt = make_float4(tg.hh * tg.hw * a, tg.hh * tg.lw * a, tg.lh * tg.hw * a, tg.lh * tg.lw * a);
          keep = cell.x >= 0 || cell.y >= 0 || cell.z >= 0 || cell.w >= 0;
        }
      }
      // ---- grad_out rows of the wave's 16 queries -> LDS (lane = query lane/4, 8 channels)
      {
        const int qg = lane >> 2, c8 = (lane & 3) * 8;
        const int qn = base + qg;
        float gv[8];
        if (qn < ncand) {
          const int yq = ya + qn / nx, xq = xa + qn % nx;
          const long long g2 = ((long long)b * S + lv.start[lq] + yq * Wq + xq) * Hh + h;
          Vec16<T>::load(gout + g2 * kD + c8, gv);
          if constexpr (Vec16<T>::N == 4) Vec16<T>::load(gout + g2 * kD + c8 + 4, gv + 4);
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) gv[k] = 0.f;
        }
        float4* dst = reinterpret_cast<float4*>(&sG[wave][qg][c8]);
        dst[0] = make_float4(gv[0], gv[1], gv[2], gv[3]);
        dst[1] = make_float4(gv[4], gv[5], gv[6], gv[7]);
      }
      // ---- compact the kept taps
      const unsigned long long mask = __ballot(keep);
      const int n = __popcll(mask);
      if (keep) {
        const int pos = __popcll(mask & ((1ull << lane) - 1ull));
        sCell[wave][pos] = cell;
        sWgt[wave][pos] = wgt;
        sQ[wave][pos] = lane >> 2;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // ---- add: half-wave per list entry, lane = channel
      for (int e = half; e < n; e += 2) {
        const int4 ce = sCell[wave][e];
        const float4 we = sWgt[wave][e];
        const float g = sG[wave][sQ[wave][e]][c];
        if (ce.x >= 0) atomicAdd(&sAcc[ce.x + c], we.x * g);
        if (ce.y >= 0) atomicAdd(&sAcc[ce.y + c], we.y * g);
        if (ce.z >= 0) atomicAdd(&sAcc[ce.z + c], we.z * g);
        if (ce.w >= 0) atomicAdd(&sAcc[ce.w + c], we.w * g);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  __syncthreads();
  // ---- store the tile: 8 consecutive lanes per cell (128 B), every cell once
  const size_t rowstride = (size_t)Hh * kD;
  float* gl = gvalue + (((size_t)b * S + lv.start[l]) * Hh + h) * kD;
  for (int k = tid; k < kTile * kTile * 8; k += 256) {
    const int cl = k >> 3, part = k & 7;
    const int cy = ty0 + cl / kTile, cx = tx0 + cl % kTile;
    if (cy < Hl && cx < Wl)
      *reinterpret_cast<float4*>(gl + (size_t)(cy * Wl + cx) * rowstride + part * 4) =
          reinterpret_cast<const float4*>(sAcc)[k];
  }
}

// ---------------------------------------------------------------------------------
// grad_value by destination after a counting sort of the corner contributions (no float
// atomics).  key(b, cell, h) = (b * S + cell) * Hh + h: the grad_value row of that
// head, so keys in order are the output in order.
//   count:  per valid corner of every tap, count[key] += 1 (int atomics)
//   scan:   offset(key) = exclusive prefix of count (1024-key blocks + block prefix)
//   fill:   slot = offset(key) + (atomicSub(count[key], 1) - 1): record {query, weight}
//           (count returns to 0)
//   pull:   a group of lanes per key sums weight * grad_out[b, query, h, :] over its
//           records in f32 and writes the row once, in the value dtype
// The contributions reaching one row come from the queries whose taps land next to it;
// their grad_out rows are re-read from L2 / MALL, not HBM.
constexpr int kScanBlock = 1024;

__device__ __forceinline__ void corner_keys(const Tap& tg, int Wl, int Hl, long long rowbase, int Hh, long long* key,
                                            float* wk) {
  const int h0 = tg.h0, w0 = tg.w0;
  const bool ok[4] = {h0 >= 0 && w0 >= 0, h0 >= 0 && w0 + 1 <= Wl - 1, h0 + 1 <= Hl - 1 && w0 >= 0,
                      h0 + 1 <= Hl - 1 && w0 + 1 <= Wl - 1};
  const int off[4] = {h0 * Wl + w0, h0 * Wl + w0 + 1, (h0 + 1) * Wl + w0, (h0 + 1) * Wl + w0 + 1};
  wk[0] = tg.hh * tg.hw;
  wk[1] = tg.hh * tg.lw;
  wk[2] = tg.lh * tg.hw;
  wk[3] = tg.lh * tg.lw;
#pragma unroll
  for (int k = 0; k < 4; ++k) key[k] = ok[k] ? (rowbase + off[k]) * Hh : -1;
}

// one thread per tap (b, q, h, l, p); FILL = false: count, true: write records
template <bool FILL>
__global__ void __launch_bounds__(256) msda_sort_kernel(const float* __restrict__ loc, const float* __restrict__ attw,
                                                        int* __restrict__ count, const int* __restrict__ local,
                                                        const int* __restrict__ bprefix, int2* __restrict__ rec,
                                                        Levels lv, int S, int Hh, int Q, int L, int P, long long taps) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= taps) return;
  const int LP = L * P;
  const int t = (int)(i % LP);
  const long long grp = i / LP;
  const int h = (int)(grp % Hh);
  const long long bq = grp / Hh;
  const int q = (int)(bq % Q);
  const long long b = bq / Q;
  const int l = t / P;
  const int Hl = lv.h[l], Wl = lv.w[l];
  const float2 xy = reinterpret_cast<const float2*>(loc)[i];
  const Tap tg = tap_geom(xy.x, xy.y, Hl, Wl);
  if (!tg.inside) return;
  long long key[4];
  float wk[4];
  corner_keys(tg, Wl, Hl, b * S + lv.start[l], Hh, key, wk);
  if (!FILL) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (key[k] >= 0) atomicAdd(count + key[k] + h, 1);
  } else {
    const float a = attw[i];
    int slot[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) slot[k] = key[k] >= 0 ? atomicSub(count + key[k] + h, 1) - 1 : 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (key[k] >= 0) {
        const long long kk = key[k] + h;
        rec[local[kk] + bprefix[kk / kScanBlock] + slot[k]] = make_int2(q, __float_as_int(a * wk[k]));
      }
  }
}

// block-local exclusive scan of count (kScanBlock keys per block) + block totals
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
template <typename T>
__global__ void __launch_bounds__(256) msda_pull_sorted_kernel(const int* __restrict__ local,
                                                               const int* __restrict__ bprefix,
                                                               const int2* __restrict__ rec, const T* __restrict__ gout,
                                                               T* __restrict__ gvalue, int S, int Hh, int Q,
                                                               long long nkeys) {
  constexpr int V = Vec16<T>::N;
  constexpr int LPG = kD / V;
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long key = gid / LPG;
  const int sub = (int)(gid % LPG);
  if (key >= nkeys) return;
  const int r0 = local[key] + bprefix[key / kScanBlock];
  const int r1 = key + 1 < nkeys ? local[key + 1] + bprefix[(key + 1) / kScanBlock] : bprefix[(nkeys - 1) / kScanBlock + 1];
  const int h = (int)(key % Hh);
  const long long b = key / Hh / S;
  const T* gb = gout + ((size_t)b * Q * Hh + h) * kD + sub * V;
  const size_t qstride = (size_t)Hh * kD;
  float acc[V];
#pragma unroll
  for (int c = 0; c < V; ++c) acc[c] = 0.f;
  int r = r0;
  for (; r + 4 <= r1; r += 4) {            // 4 records' gathers in flight
    int2 e[4];
    float g[4][V];
#pragma unroll
    for (int u = 0; u < 4; ++u) e[u] = rec[r + u];
#pragma unroll
    for (int u = 0; u < 4; ++u) Vec16<T>::load(gb + (size_t)e[u].x * qstride, g[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float w = __int_as_float(e[u].y);
#pragma unroll
      for (int c = 0; c < V; ++c) acc[c] = __fmaf_rn(w, g[u][c], acc[c]);
    }
  }
  for (; r < r1; ++r) {
    const int2 e = rec[r];
    float g[V];
    Vec16<T>::load(gb + (size_t)e.x * qstride, g);
    const float w = __int_as_float(e.y);
#pragma unroll
    for (int c = 0; c < V; ++c) acc[c] = __fmaf_rn(w, g[c], acc[c]);
  }
  Vec16<T>::store(gvalue + key * kD + sub * V, acc);
}

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

// workspace: count [nkeys] | local [nkeys] | bsum [nb] | bprefix [nb + 1] | records
void sorted_layout(long long nkeys, long long maxrec, size_t* off) {
  const long long nb = (nkeys + kScanBlock - 1) / kScanBlock;
  off[0] = 0;
  off[1] = align256(off[0] + nkeys * 4);
  off[2] = align256(off[1] + nkeys * 4);
  off[3] = align256(off[2] + nb * 4);
  off[4] = align256(off[3] + (nb + 1) * 4);
  off[5] = align256(off[4] + (size_t)maxrec * 8);
}


// ---------------------------------------------------------------------------------
// grad_value by QUERY tiles with a per-wave LDS window (Q == S and P == 4; default for
// the pixel-decoder layers).
//
// A one-wave workgroup owns a tile of 16 queries of one (image, head, channel half): a
// 4 x 4 block of one level when the queries are the value grid (level-major, mode 1),
// else 16 consecutive queries (mode 0).  Per value level l the wave takes the bounding
// box of the corners its 64 taps touch, clipped to kWinCells cells, as an f32 window in
// LDS (cell x 16 channels, rows padded so the two corner rows use disjoint banks), and
// walks the taps in order with lanes = 4 corner quadrants x 16 channels: every corner
// is one plain LDS read-modify-write (a single wave: LDS ops retire in order, the four
// quadrants of a tap are distinct cells, so no atomics and no races).  Then every
// touched window cell is added to grad_value once (f32 atomics: neighbouring tiles'
// windows overlap), and corners outside the clipped window are added directly.
// Smoothly varying encoder offsets put a tile's taps of one level into a few dozen
// cells, so the global atomics fall several-fold against one per corner per tap
// (measured: pixel-decoder layer backward 1.74 -> 1.10 ms at C2).
#ifndef VS_MSDA_WIN_CELLS
#define VS_MSDA_WIN_CELLS 96
#endif
constexpr int kWinCells = VS_MSDA_WIN_CELLS;   // LDS window capacity (cells x 16 ch f32 = 6 KB)
#ifndef VS_MSDA_TX
#define VS_MSDA_TX 4
#endif
#ifndef VS_MSDA_TY
#define VS_MSDA_TY 4
#endif
constexpr int kTX = VS_MSDA_TX, kTY = VS_MSDA_TY;   // query tile width / height (grid mode)
constexpr int kTQ = kTX * kTY;                      // queries per tile (a power of two <= 64)
static_assert((kTQ & (kTQ - 1)) == 0 && kTQ >= 4 && kTQ <= 64, "query tile must hold 4..64 queries, a power of 2");
constexpr int kWinC = 16;                // channels per workgroup (a head's 32 split over two)

struct QueryTiles {
  int mode;                              // 1: 4x4 grid tiles per level, 0: runs of 16
  int prefix[kMaxLevels + 1];            // grid mode: tile-index prefix per query level
  int ntx[kMaxLevels];
  int per_image;                         // tiles per image
};

__device__ __forceinline__ int tile_query(const QueryTiles& qt, const Levels& lv, int L, int tile, int idx, int Q) {
  if (idx >= kTQ) return -1;
  if (qt.mode == 0) {
    const int q = tile * kTQ + idx;
    return q < Q ? q : -1;
  }
  int lq = 0;
  while (lq + 1 < L && tile >= qt.prefix[lq + 1]) ++lq;
  const int t = tile - qt.prefix[lq];
  const int y = (t / qt.ntx[lq]) * kTY + idx / kTX, x = (t % qt.ntx[lq]) * kTX + idx % kTX;
  return (y < lv.h[lq] && x < lv.w[lq]) ? lv.start[lq] + y * lv.w[lq] + x : -1;
}

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

template <typename T>
__global__ void __launch_bounds__(64)
#ifdef VS_MSDA_WIN_WPE
__attribute__((amdgpu_waves_per_eu(VS_MSDA_WIN_WPE)))
#endif
msda_bwd_window_kernel(const float* __restrict__ loc,
                                                             const float* __restrict__ attw,
                                                             const T* __restrict__ gout, float* __restrict__ gvalue,
                                                             Levels lv, QueryTiles qt, int S, int Hh, int Q, int L,
                                                             int nblk, int dbg) {
  constexpr int P = 4;
  constexpr int kWinFloats = kWinCells * kWinC + 32;   // + the row-pitch pad
  __shared__ float win[kWinFloats + 64];               // + one trash slot per lane
  __shared__ float sg[kTQ * kWinC];
  __shared__ float rec[kTQ * 4 * 8];                     // [query][point][quadrant] {weight, target}
  const int blk = xcd_swizzle(blockIdx.x, nblk);
  const int chalf = blk & 1;
  const int h = (blk >> 1) % Hh;
  const int tile = ((blk >> 1) / Hh) % qt.per_image;
  const int b = (blk >> 1) / Hh / qt.per_image;
  const int lane = threadIdx.x;
  const int LP = L * P;
  const int myq = tile_query(qt, lv, L, tile, lane, Q);
  const long long mygrp = ((long long)b * Q + (myq < 0 ? 0 : myq)) * Hh + h;
  {
    const int c = lane & 15, sub = lane >> 4;       // grad_out: 16 channels of 4 queries per pass
    for (int r = 0; r < kTQ / 4; ++r) {
      const int idx = 4 * r + sub;
      const int q = __shfl(myq, idx, 64);
      sg[idx * kWinC + c] = q >= 0 ? to_f32(gout[(((long long)b * Q + q) * Hh + h) * kD + chalf * kWinC + c]) : 0.f;
    }
  }
  for (int i = lane; i < kWinFloats + 64; i += 64) win[i] = 0.f;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  // walk layout: lane = corner quadrant (qy, qx) x 16 channels
  const int quad = lane >> 4, ch = lane & 15;
  const size_t rowstride = (size_t)Hh * kD;
  const size_t vbase = ((size_t)b * S * Hh + h) * kD + chalf * kWinC + ch;
  for (int l = 0; l < L; ++l) {
    const int Hl = lv.h[l], Wl = lv.w[l];
    const size_t lbase = vbase + (size_t)lv.start[l] * rowstride;
    // lane = query: its 4 taps on level l, and the bounding box of their valid corners
    int th[P], tw[P];
    float tlh[P], tlw[P], ta[P];
    bool tv[P];
    int ylo = 1 << 30, xlo = 1 << 30, yhi = -1, xhi = -1;
    {
      float4 xy0 = make_float4(0.f, 0.f, 0.f, 0.f), xy1 = xy0, aw = xy0;
      if (myq >= 0) {
        const float4* lp = reinterpret_cast<const float4*>(loc + (mygrp * LP + l * P) * 2);
        xy0 = lp[0];
        xy1 = lp[1];
        aw = *reinterpret_cast<const float4*>(attw + mygrp * LP + l * P);
      }
      const float xs[P] = {xy0.x, xy0.z, xy1.x, xy1.z}, ys[P] = {xy0.y, xy0.w, xy1.y, xy1.w};
      const float as[P] = {aw.x, aw.y, aw.z, aw.w};
#pragma unroll
      for (int p = 0; p < P; ++p) {
        const Tap t = tap_geom(xs[p], ys[p], Hl, Wl);
        tv[p] = myq >= 0 && t.inside;
        th[p] = t.h0;
        tw[p] = t.w0;
        tlh[p] = t.lh;
        tlw[p] = t.lw;
        ta[p] = as[p];
        if (tv[p]) {
          ylo = min(ylo, max(t.h0, 0));
          yhi = max(yhi, min(t.h0 + 1, Hl - 1));
          xlo = min(xlo, max(t.w0, 0));
          xhi = max(xhi, min(t.w0 + 1, Wl - 1));
        }
      }
    }
    unsigned long long vm[P];
#pragma unroll
    for (int p = 0; p < P; ++p) vm[p] = __ballot(tv[p]);
    if ((vm[0] | vm[1] | vm[2] | vm[3]) == 0ull) continue;
    const int oy = wave_min(ylo), ox = wave_min(xlo);
    int WX = min(wave_max(xhi) - ox + 1, kWinCells);
    // row pitch = 32 (mod 64) floats: the two corner rows of a tap use disjoint LDS banks
    const int RP = WX * kWinC + ((32 - (WX * kWinC) % 64) + 64) % 64;
    const int WY = min(wave_max(yhi) - oy + 1, kWinFloats / RP);
    // Tap records: lane = query writes, per tap p and corner quadrant k, {weight, target}
    // where target >= 0 is the corner's window offset (the trash slot for an invalid
    // tap or corner outside the level, weight 0) and target < 0 encodes -(level cell + 1)
    // for a valid corner outside the clipped window (direct atomic).
#pragma unroll
    for (int p = 0; p < P; ++p) {
      float2 r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int y = th[p] + (k >> 1), x = tw[p] + (k & 1);
        const bool ok = tv[p] && y >= 0 && y < Hl && x >= 0 && x < Wl;
        const bool in = ok && (unsigned)(y - oy) < (unsigned)WY && (unsigned)(x - ox) < (unsigned)WX;
        const float wy = (k >> 1) ? tlh[p] : 1.f - tlh[p], wx = (k & 1) ? tlw[p] : 1.f - tlw[p];
        const int tgt = in ? (y - oy) * RP + (x - ox) * kWinC : ok ? -(y * Wl + x + 1) : kWinFloats;
        r[k] = make_float2(ok ? wy * wx * ta[p] : 0.f, __int_as_float(tgt));
      }
      float4* dst = reinterpret_cast<float4*>(rec + ((lane & (kTQ - 1)) * P + p) * 8);
      if (lane < kTQ) dst[0] = make_float4(r[0].x, r[0].y, r[1].x, r[1].y);
      if (lane < kTQ) dst[1] = make_float4(r[2].x, r[2].y, r[3].x, r[3].y);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // walk: lane = corner quadrant x 16 channels; each tap is one record read (hoisted,
    // independent of the window) and one LDS read-modify-write per lane
    const int trash = kWinFloats + lane;
    float2 rn[P];
    float gn = sg[ch];
#pragma unroll
    for (int p = 0; p < P; ++p) rn[p] = *reinterpret_cast<const float2*>(rec + p * 8 + quad * 2);
    for (int q = 0; q < ((dbg & 1) ? 0 : kTQ); ++q) {
      float2 r[P];
#pragma unroll
      for (int p = 0; p < P; ++p) r[p] = rn[p];
      const float g = gn;
      const int qn = (q + 1) & (kTQ - 1);        // prefetch the next query's records
      gn = sg[qn * kWinC + ch];
#pragma unroll
      for (int p = 0; p < P; ++p) rn[p] = *reinterpret_cast<const float2*>(rec + (qn * P + p) * 8 + quad * 2);
#pragma unroll
      for (int p = 0; p < P; ++p) {
        const int tgt = __float_as_int(r[p].y);
        const float d = r[p].x * g;
        const int a = tgt >= 0 ? tgt + ch : trash;
        win[a] += d;
        if (tgt < 0 && !(dbg & 8)) atomicAdd(gvalue + lbase + (size_t)(-tgt - 1) * rowstride, d);
      }
    }
    // add the window to grad_value once per touched cell, and clear it for the next level
    const int ncell = WY * WX;
    for (int i = quad; i < ncell; i += 4) {
      const int cy = i / WX, cx = i - cy * WX;
      float* pw = win + cy * RP + cx * kWinC + ch;
      const float v = *pw;
      *pw = 0.f;
      if (v != 0.f && !(dbg & 2))
        atomicAdd(gvalue + lbase + (size_t)((oy + cy) * Wl + ox + cx) * rowstride, v);
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

template <bool ENC>
static void launch_scatter(int dtype, const float* loc, const float* attw, const void* gout, float* gvalue,
                           const Levels& lv, int B, int S, int Hh, int Q, int L, int run, int R0, hipStream_t st) {
  const int nrun = (Q + run - 1) / run;
  const long long hws = (long long)B * nrun * Hh;
  const int sgrid = (int)((hws + 7) / 8);
#define VS_SCATTER(TT, LL)                                                                                   \
  hipLaunchKernelGGL((msda_bwd_scatter_kernel<TT, LL, 4, ENC>), dim3(sgrid), dim3(256), 0, st, loc, attw,     \
                     (const TT*)gout, gvalue, lv, S, Hh, Q, run, nrun, hws, R0)
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
}

static int msda_backward_impl(int dtype, const void* value, const int64_t* shapes, const int64_t* starts,
                              const float* loc, const float* attw, const void* gout, float* gvalue, float* gloc,
                              float* gattw, int B, int S, int Hh, int D, int L, int Q, int P, void* stream,
                              bool encoder) {
  VS_CHECK(D == kD, "channels per head must be 32");
  VS_CHECK(L >= 1 && L <= kMaxLevels, "1..4 levels supported");
  VS_CHECK(B > 0 && S > 0 && Hh > 0 && Q >= 0 && P > 0, "bad sizes");
  VS_CHECK(value && loc && attw && gout && gvalue && gloc && gattw && shapes && starts, "null pointer");
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype must be VS_F32 or VS_BF16");
  Levels lv;
  VS_CHECK(fill_levels(&lv, shapes, starts, L, S), "spatial shapes / level starts inconsistent with S");
  VS_CHECK(!encoder || Q == S, "encoder mode needs the queries to be the value grid (Q == S)");
  VS_CHECK(!encoder || P == 4, "encoder-mode backward is specialised for 4 sampling points");
  hipStream_t st = (hipStream_t)stream;
  const long long groups = (long long)B * Q * Hh;
  if (encoder) {
    // tile kernel (plain stores of every grad_value element: all near taps, LDS
    // accumulation), then the carry scatter adds the far taps, and the geom kernel
    // computes grad_loc / grad_attn
    int R0 = kNearR;
    if (const char* e = getenv("VS_MSDA_NEAR_R")) R0 = atoi(e);
    VS_CHECK(R0 >= 0 && R0 <= 64, "VS_MSDA_NEAR_R out of range");
    TileOrder to;
    int ord[kMaxLevels];
    for (int l = 0; l < L; ++l) ord[l] = l;
    for (int a = 0; a < L; ++a)                 // ascending cell count (stable)
      for (int c2 = a + 1; c2 < L; ++c2)
        if ((long long)lv.h[ord[c2]] * lv.w[ord[c2]] < (long long)lv.h[ord[a]] * lv.w[ord[a]]) {
          const int tmp = ord[a];
          ord[a] = ord[c2];
          ord[c2] = tmp;
        }
    to.prefix[0] = 0;
    for (int k = 0; k < kMaxLevels; ++k) to.level[k] = k < L ? ord[k] : 0;
    for (int k = 0; k < L; ++k) {
      const int l = ord[k];
      const int tiles = ((lv.h[l] + kTile - 1) / kTile) * ((lv.w[l] + kTile - 1) / kTile);
      to.prefix[k + 1] = to.prefix[k] + tiles * B;
    }
    for (int k = L; k < kMaxLevels; ++k) to.prefix[k + 1] = to.prefix[L];
    to.slots = to.prefix[L];
    const long long nblk = (long long)((to.slots + 7) / 8) * 8 * Hh;
    VS_CHECK(nblk < (1LL << 31), "too many tiles");
    // VS_MSDA_SKIP (profiling only): bit 0 skips the tile kernel, bit 1 the scatter, bit 2 geom
    int skip = 0;
    if (const char* e = getenv("VS_MSDA_SKIP")) skip = atoi(e);
    if (!(skip & 1)) {
      if (dtype == VS_BF16)
        hipLaunchKernelGGL(msda_bwd_tile_kernel<bf16>, dim3((unsigned)nblk), dim3(256), 0, st, loc, attw,
                           (const bf16*)gout, gvalue, lv, S, Hh, B, L, R0, to);
      else
        hipLaunchKernelGGL(msda_bwd_tile_kernel<float>, dim3((unsigned)nblk), dim3(256), 0, st, loc, attw,
                           (const float*)gout, gvalue, lv, S, Hh, B, L, R0, to);
    }
    if (!(skip & 2)) launch_scatter<true>(dtype, loc, attw, gout, gvalue, lv, B, S, Hh, Q, L, kScatterRun, R0, st);
    if (!(skip & 4)) launch_geom(dtype, value, loc, attw, gout, gloc, gattw, lv, S, Hh, Q, L, P, groups, st);
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
  VS_HIP(hipMemsetAsync(gvalue, 0, sizeof(float) * (size_t)B * S * Hh * kD, st));
  if (Q == 0) return VS_OK;
  // geom + register-carry scatter when there are enough queries for runs to fill the chip
  // (VS_MSDA_RUN=n forces runs of n <= kScatterRun queries at any size, 0 the single kernel)
  int run = kScatterRun;
  bool split = (long long)B * Q * Hh >= (long long)kScatterRun * 8192;
  if (const char* e = getenv("VS_MSDA_RUN")) {
    run = atoi(e);
    split = run >= 1;
  }
  // query-tile LDS-window scatter (VS_MSDA_WIN=0 selects the register-carry scatter)
  bool win = split && P == 4;
  if (const char* e = getenv("VS_MSDA_WIN")) win = win && atoi(e) != 0;
  if (win) {
    QueryTiles qt;
    qt.mode = Q == S ? 1 : 0;
    qt.prefix[0] = 0;
    for (int l = 0; l < kMaxLevels; ++l) {
      const bool on = qt.mode == 1 && l < L;
      qt.ntx[l] = on ? (lv.w[l] + kTX - 1) / kTX : 1;
      qt.prefix[l + 1] = qt.prefix[l] + (on ? ((lv.h[l] + kTY - 1) / kTY) * qt.ntx[l] : 0);
    }
    qt.per_image = qt.mode == 1 ? qt.prefix[L] : (Q + kTQ - 1) / kTQ;
    const long long nblk = 2LL * B * qt.per_image * Hh;
    VS_CHECK(nblk < (1LL << 31), "too many query tiles");
    int dbg = 0;                           // VS_MSDA_WIN_DBG (profiling only): 1 skips the walk, 2 the flush atomics
    if (const char* e = getenv("VS_MSDA_WIN_DBG")) dbg = atoi(e);
    launch_geom(dtype, value, loc, attw, gout, gloc, gattw, lv, S, Hh, Q, L, P, groups, st);
    if (dtype == VS_BF16)
      hipLaunchKernelGGL(msda_bwd_window_kernel<bf16>, dim3((unsigned)nblk), dim3(64), 0, st, loc, attw,
                         (const bf16*)gout, gvalue, lv, qt, S, Hh, Q, L, (int)nblk, dbg);
    else
      hipLaunchKernelGGL(msda_bwd_window_kernel<float>, dim3((unsigned)nblk), dim3(64), 0, st, loc, attw,
                         (const float*)gout, gvalue, lv, qt, S, Hh, Q, L, (int)nblk, dbg);
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
  if (split && P == 4) {
    VS_CHECK(run <= kScatterRun, "VS_MSDA_RUN must not exceed the LDS-staged run (16)");
    launch_geom(dtype, value, loc, attw, gout, gloc, gattw, lv, S, Hh, Q, L, P, groups, st);
    launch_scatter<false>(dtype, loc, attw, gout, gvalue, lv, B, S, Hh, Q, L, run, 0, st);
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
                            P, stream, false);
}

extern "C" int vs_msda_backward_encoder(int dtype, const void* value, const int64_t* shapes, const int64_t* starts,
                                        const float* loc, const float* attw, const void* gout, float* gvalue,
                                        float* gloc, float* gattw, int B, int S, int Hh, int D, int L, int P,
                                        void* stream) {
  return msda_backward_impl(dtype, value, shapes, starts, loc, attw, gout, gvalue, gloc, gattw, B, S, Hh, D, L, S,
                            P, stream, true);
}

extern "C" long long vs_msda_backward_sorted_workspace_bytes(int B, int S, int Hh, int Q, int L, int P) {
  size_t off[6];
  sorted_layout((long long)B * S * Hh, 4LL * B * Q * Hh * L * P, off);
  return (long long)off[5];
}

extern "C" int vs_msda_backward_sorted(int dtype, const void* value, const int64_t* shapes, const int64_t* starts,
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
  const long long nkeys = (long long)B * S * Hh;
  const long long taps = (long long)B * Q * Hh * L * P;
  VS_CHECK(4 * taps < (1LL << 31), "too many corner contributions for 32-bit record offsets");
  hipStream_t st = (hipStream_t)stream;
  size_t off[6];
  sorted_layout(nkeys, 4 * taps, off);
  char* ws = (char*)workspace;
  int* count = (int*)(ws + off[0]);
  int* local = (int*)(ws + off[1]);
  int* bsum = (int*)(ws + off[2]);
  int* bprefix = (int*)(ws + off[3]);
  int2* rec = (int2*)(ws + off[4]);
  const int nb = (int)((nkeys + kScanBlock - 1) / kScanBlock);
  VS_HIP(hipMemsetAsync(count, 0, (size_t)nkeys * 4, st));
  if (Q > 0) {
    const int tgrid = (int)((taps + 255) / 256);
    hipLaunchKernelGGL(msda_sort_kernel<false>, dim3(tgrid), dim3(256), 0, st, loc, attw, count, local, bprefix, rec,
                       lv, S, Hh, Q, L, P, taps);
  }
  hipLaunchKernelGGL(sort_scan_local_kernel, dim3(nb), dim3(256), 0, st, count, local, bsum, nkeys);
  hipLaunchKernelGGL(sort_scan_blocks_kernel, dim3(1), dim3(1024), 0, st, bsum, bprefix, nb);
  if (Q > 0) {
    const int tgrid = (int)((taps + 255) / 256);
    hipLaunchKernelGGL(msda_sort_kernel<true>, dim3(tgrid), dim3(256), 0, st, loc, attw, count, local, bprefix, rec,
                       lv, S, Hh, Q, L, P, taps);
  }
  const int lpg = dtype == VS_BF16 ? 4 : 8;
  const int pgrid = (int)((nkeys * lpg + 255) / 256);
  if (dtype == VS_BF16)
    hipLaunchKernelGGL(msda_pull_sorted_kernel<bf16>, dim3(pgrid), dim3(256), 0, st, local, bprefix, rec,
                       (const bf16*)gout, (bf16*)gvalue, S, Hh, Q, nkeys);
  else
    hipLaunchKernelGGL(msda_pull_sorted_kernel<float>, dim3(pgrid), dim3(256), 0, st, local, bprefix, rec,
                       (const float*)gout, (float*)gvalue, S, Hh, Q, nkeys);
  if (Q > 0) launch_geom(dtype, value, loc, attw, gout, gloc, gattw, lv, S, Hh, Q, L, P, (long long)B * Q * Hh, st);
  VS_LAUNCH_CHECK();
  return VS_OK;
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
