// Swin (shifted-)window attention core, forward + backward.
//
// Semantics (HF:swin:373-398 eager_attention_forward, HF:swin:418-468, mask
// HF:swin:584-607, bias HF:swin:329-370):
//   S_ij = (q_i . k_j) * scale + table[rel(i,j), h] + (shift && region_i != region_j ? -100 : 0)
//   O_i  = softmax_j(S_i) V          (f32 softmax)
// where rel(i,j) = (ty_i - ty_j + ws-1)(2ws-1) + (tx_i - tx_j + ws-1) and the region id of
// a token is computed from its padded-grid position (the HF mask is built on the
// un-rolled grid: thresholds Hp-ws and Hp-shift).  Neither the [nW,N,N] mask nor the
// [heads,N,N] bias is ever materialised: both are derived per (i,j) from integer
// coordinates and a (2ws-1)^2 LDS copy of the table column.
//
// Layout: qkv [Bw, N, 3, heads, 32] (the fused q;k;v Linear output, N = ws^2),
// out [Bw, N, heads*32], lse f32 [Bw, heads, N].
//
// Structure (first correct HIP path): one workgroup per (window, head); K and V of the
// window staged in LDS as f32; one lane per query row (64*ceil(N/64) lanes), rows read
// K/V rows by LDS broadcast.  Two passes over keys (max, then exp-sum + PV) keep the
// softmax identical to the reference's max-subtract form.  Backward: lane-per-row pass
// for dQ and the bias gradient (LDS float atomics into (2ws-1)^2 bins), lane-per-column
// pass for dK/dV, recomputing P from the saved log-sum-exp.  The per-window bias
// gradient partials are written to [Bw, heads, (2ws-1)^2] and summed by the caller
// (deterministic, no cross-workgroup atomics on a 169-entry table).
#include "lds_dma.h"
#include "mfma_util.h"
#include "mx_util.h"

namespace vs {
namespace {

constexpr int kD = 32;

struct WinGeom {
  int heads, ws, shift, nWh, nWw, N, T2;  // T2 = (2ws-1)^2
  float scale;
  int H, W, nat;                           // nat: out / grad_out in the image layout [B, H, W, C]
  // division by multiply-high (check_geom): a window's token / ws for t < 2^16 / ws, and the
  // window index / (nWh nWw) and / nWw (exact while the dividend times the divisor < 2^32).
  // Each integer division was ~30 VALU, and the index arithmetic of the staging and of the
  // image-layout rows had grown to about half of the backward kernels' VALU instructions
  unsigned m_ws, m_nw, m_nWw;
};

__device__ __forceinline__ int div_ws(const WinGeom& g, int t) { return (int)(__umul24((unsigned)t, g.m_ws) >> 16); }
__device__ __forceinline__ int div_nw(const WinGeom& g, int bw) {
  return g.m_nw ? (int)__umulhi((unsigned)bw, g.m_nw) : bw;            // m 0: divisor 1
}
__device__ __forceinline__ int div_nWw(const WinGeom& g, int wl) {
  return g.m_nWw ? (int)__umulhi((unsigned)wl, g.m_nWw) : wl;
}

// Row of window token t of window bw in the output / output-gradient layout: the window
// layout (bw N + t), or -- nat, the window reverse folded into the kernel -- the token's
// pixel in [B, H, W] (the partition's roll undone; -1 for a token of the zero padding,
// which the reverse crops: its output is not stored and its output gradient is zero)
__device__ __forceinline__ long long out_row(const WinGeom& g, int bw, int t) {
  if (!g.nat) return (long long)bw * g.N + t;
  const int nw = g.nWh * g.nWw, b = div_nw(g, bw), wl = bw - b * nw;
  const int wy = div_nWw(g, wl), wx = wl - wy * g.nWw;
  const int ty = div_ws(g, t), tx = t - ty * g.ws;
  int y = wy * g.ws + ty + g.shift, x = wx * g.ws + tx + g.shift;
  if (y >= g.nWh * g.ws) y -= g.nWh * g.ws;
  if (x >= g.nWw * g.ws) x -= g.nWw * g.ws;
  if (y >= g.H || x >= g.W) return -1;
  return ((long long)b * g.H + y) * g.W + x;
}

__device__ __forceinline__ int region_of(int p, int Pp, int ws, int shift) {
  return (p >= Pp - ws) + (p >= Pp - shift);
}

template <typename T>
__device__ __forceinline__ void load_row32(const T* src, float* dst) {
  constexpr int V = Vec16<T>::N;
#pragma unroll
  for (int c = 0; c < kD; c += V) Vec16<T>::load(src + c, dst + c);
}

template <typename T>
__device__ __forceinline__ void store_row32(T* dst, const float* src) {
  constexpr int V = Vec16<T>::N;
#pragma unroll
  for (int c = 0; c < kD; c += V) Vec16<T>::store(dst + c, src + c);
}

// Cooperative copy of one head's 32-channel rows of part `s` (0 q, 1 k, 2 v) into LDS f32.
template <typename T>
__device__ __forceinline__ void stage_rows(const T* qkv_win, int s, int C3, int h, int N, float* lds) {
  constexpr int V = Vec16<T>::N;
  constexpr int CH = kD / V;  // 16-B chunks per row
  for (int idx = threadIdx.x; idx < N * CH; idx += blockDim.x) {
    const int t = idx / CH, c = (idx % CH) * V;
    float tmp[V];
    Vec16<T>::load(qkv_win + (size_t)t * C3 + s * (C3 / 3) + h * kD + c, tmp);
#pragma unroll
    for (int i = 0; i < V; ++i) lds[t * kD + c + i] = tmp[i];
  }
}

__device__ __forceinline__ float dot32(const float* a, const float* __restrict__ b_lds) {
  float s = 0.f;
  const float4* b4 = reinterpret_cast<const float4*>(b_lds);
#pragma unroll
  for (int c = 0; c < kD / 4; ++c) {
    const float4 b = b4[c];
    s = fmaf(a[4 * c + 0], b.x, s);
    s = fmaf(a[4 * c + 1], b.y, s);
    s = fmaf(a[4 * c + 2], b.z, s);
    s = fmaf(a[4 * c + 3], b.w, s);
  }
  return s;
}

template <typename T>
__global__ void __launch_bounds__(256) win_attn_fwd_kernel(const T* __restrict__ qkv,
                                                           const float* __restrict__ table,
                                                           T* __restrict__ out, float* __restrict__ lse,
                                                           WinGeom g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int N = g.N, ws = g.ws, T2 = g.T2, tw = 2 * ws - 1;
  const int bw = blockIdx.x, h = blockIdx.y;
  const int C = g.heads * kD, C3 = 3 * C;
  float* sk = smem;
  float* sv = sk + N * kD;
  float* sb = sv + N * kD;
  const T* win = qkv + (size_t)bw * N * C3;
  stage_rows(win, 1, C3, h, N, sk);
  stage_rows(win, 2, C3, h, N, sv);
  for (int t = threadIdx.x; t < T2; t += blockDim.x) sb[t] = table[t * g.heads + h];
  __syncthreads();
  const int i = threadIdx.x;
  if (i >= N) return;
  const int wl = bw % (g.nWh * g.nWw);
  const int wy = wl / g.nWw, wx = wl % g.nWw;
  const int Hp = g.nWh * ws, Wp = g.nWw * ws;
  const int tyi = i / ws, txi = i % ws;
  const bool shifted = g.shift > 0;
  const int ri = shifted ? region_of(wy * ws + tyi, Hp, ws, g.shift) * 3 + region_of(wx * ws + txi, Wp, ws, g.shift) : 0;
  float q[kD];
  load_row32(win + (size_t)i * C3 + h * kD, q);
  // pass 1: row max
  float m = -INFINITY;
  for (int j = 0, tyj = 0, txj = 0; j < N; ++j) {
    float s = dot32(q, sk + j * kD) * g.scale + sb[(tyi - tyj + ws - 1) * tw + (txi - txj + ws - 1)];
    if (shifted) {
      const int rj = region_of(wy * ws + tyj, Hp, ws, g.shift) * 3 + region_of(wx * ws + txj, Wp, ws, g.shift);
      if (rj != ri) s += -100.f;
    }
    m = fmaxf(m, s);
    if (++txj == ws) { txj = 0; ++tyj; }
  }
  // pass 2: exp-sum and P.V
  float o[kD];
#pragma unroll
  for (int c = 0; c < kD; ++c) o[c] = 0.f;
  float l = 0.f;
  for (int j = 0, tyj = 0, txj = 0; j < N; ++j) {
    float s = dot32(q, sk + j * kD) * g.scale + sb[(tyi - tyj + ws - 1) * tw + (txi - txj + ws - 1)];
    if (shifted) {
      const int rj = region_of(wy * ws + tyj, Hp, ws, g.shift) * 3 + region_of(wx * ws + txj, Wp, ws, g.shift);
      if (rj != ri) s += -100.f;
    }
    const float p = __expf(s - m);
    l += p;
    const float4* v4 = reinterpret_cast<const float4*>(sv + j * kD);
#pragma unroll
    for (int c = 0; c < kD / 4; ++c) {
      const float4 v = v4[c];
      o[4 * c + 0] = fmaf(p, v.x, o[4 * c + 0]);
      o[4 * c + 1] = fmaf(p, v.y, o[4 * c + 1]);
      o[4 * c + 2] = fmaf(p, v.z, o[4 * c + 2]);
      o[4 * c + 3] = fmaf(p, v.w, o[4 * c + 3]);
    }
    if (++txj == ws) { txj = 0; ++tyj; }
  }
  const float inv = 1.f / l;
#pragma unroll
  for (int c = 0; c < kD; ++c) o[c] *= inv;
  store_row32(out + ((size_t)bw * N + i) * C + h * kD, o);
  lse[((size_t)bw * g.heads + h) * N + i] = m + __logf(l);
}

template <typename T>
__global__ void __launch_bounds__(256) win_attn_bwd_kernel(
    const T* __restrict__ qkv, const float* __restrict__ table, const T* __restrict__ out,
    const float* __restrict__ lse, const T* __restrict__ gout, T* __restrict__ gqkv,
    float* __restrict__ gtable_part, WinGeom g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int N = g.N, ws = g.ws, T2 = g.T2, tw = 2 * ws - 1;
  const int bw = blockIdx.x, h = blockIdx.y;
  const int C = g.heads * kD, C3 = 3 * C;
  float* sq = smem;
  float* sk = sq + N * kD;
  float* sv = sk + N * kD;
  float* sdo = sv + N * kD;
  float* slse = sdo + N * kD;
  float* sdd = slse + N;
  float* sb = sdd + N;
  float* sbins = sb + T2;
  const T* win = qkv + (size_t)bw * N * C3;
  stage_rows(win, 0, C3, h, N, sq);
  stage_rows(win, 1, C3, h, N, sk);
  stage_rows(win, 2, C3, h, N, sv);
  {
    constexpr int V = Vec16<T>::N;
    constexpr int CH = kD / V;
    const T* go = gout + (size_t)bw * N * C + h * kD;
    for (int idx = threadIdx.x; idx < N * CH; idx += blockDim.x) {
      const int t = idx / CH, c = (idx % CH) * V;
      float tmp[V];
      Vec16<T>::load(go + (size_t)t * C + c, tmp);
#pragma unroll
      for (int e = 0; e < V; ++e) sdo[t * kD + c + e] = tmp[e];
    }
  }
  for (int t = threadIdx.x; t < T2; t += blockDim.x) {
    sb[t] = table[t * g.heads + h];
    sbins[t] = 0.f;
  }
  const int i = threadIdx.x;
  if (i < N) {
    float o[kD], d[kD];
    load_row32(out + ((size_t)bw * N + i) * C + h * kD, o);
    load_row32(gout + ((size_t)bw * N + i) * C + h * kD, d);
    float D = 0.f;
#pragma unroll
    for (int c = 0; c < kD; ++c) D = fmaf(o[c], d[c], D);
    sdd[i] = D;
    slse[i] = lse[((size_t)bw * g.heads + h) * N + i];
  }
  __syncthreads();
  const int wl = bw % (g.nWh * g.nWw);
  const int wy = wl / g.nWw, wx = wl % g.nWw;
  const int Hp = g.nWh * ws, Wp = g.nWw * ws;
  const bool shifted = g.shift > 0;
  T* gwin = gqkv + (size_t)bw * N * C3;
  if (i < N) {
    // ---- phase A: lane = query row i -> dQ_i and bias-gradient bins
    const int tyi = i / ws, txi = i % ws;
    const int ri = shifted ? region_of(wy * ws + tyi, Hp, ws, g.shift) * 3 + region_of(wx * ws + txi, Wp, ws, g.shift) : 0;
    float q[kD], dO[kD], dq[kD];
#pragma unroll
    for (int c = 0; c < kD; ++c) { q[c] = sq[i * kD + c]; dO[c] = sdo[i * kD + c]; dq[c] = 0.f; }
    const float Li = slse[i], Di = sdd[i];
    for (int j = 0, tyj = 0, txj = 0; j < N; ++j) {
      const int bidx = (tyi - tyj + ws - 1) * tw + (txi - txj + ws - 1);
      float s = dot32(q, sk + j * kD) * g.scale + sb[bidx];
      if (shifted) {
        const int rj = region_of(wy * ws + tyj, Hp, ws, g.shift) * 3 + region_of(wx * ws + txj, Wp, ws, g.shift);
        if (rj != ri) s += -100.f;
      }
      const float p = __expf(s - Li);
      const float dp = dot32(dO, sv + j * kD);
      const float ds = p * (dp - Di);
      atomicAdd(&sbins[bidx], ds);
      const float4* k4 = reinterpret_cast<const float4*>(sk + j * kD);
#pragma unroll
      for (int c = 0; c < kD / 4; ++c) {
        const float4 k = k4[c];
        dq[4 * c + 0] = fmaf(ds, k.x, dq[4 * c + 0]);
        dq[4 * c + 1] = fmaf(ds, k.y, dq[4 * c + 1]);
        dq[4 * c + 2] = fmaf(ds, k.z, dq[4 * c + 2]);
        dq[4 * c + 3] = fmaf(ds, k.w, dq[4 * c + 3]);
      }
      if (++txj == ws) { txj = 0; ++tyj; }
    }
#pragma unroll
    for (int c = 0; c < kD; ++c) dq[c] *= g.scale;
    store_row32(gwin + (size_t)i * C3 + 0 * C + h * kD, dq);
  }
  if (i < N) {
    // ---- phase B: lane = key column j -> dK_j, dV_j
    const int j = i;
    const int tyj = j / ws, txj = j % ws;
    const int rj = shifted ? region_of(wy * ws + tyj, Hp, ws, g.shift) * 3 + region_of(wx * ws + txj, Wp, ws, g.shift) : 0;
    float k[kD], v[kD], dk[kD], dv[kD];
#pragma unroll
    for (int c = 0; c < kD; ++c) { k[c] = sk[j * kD + c]; v[c] = sv[j * kD + c]; dk[c] = 0.f; dv[c] = 0.f; }
    for (int ii = 0, tyi = 0, txi = 0; ii < N; ++ii) {
      float s = dot32(k, sq + ii * kD) * g.scale + sb[(tyi - tyj + ws - 1) * tw + (txi - txj + ws - 1)];
      if (shifted) {
        const int ri = region_of(wy * ws + tyi, Hp, ws, g.shift) * 3 + region_of(wx * ws + txi, Wp, ws, g.shift);
        if (ri != rj) s += -100.f;
      }
      const float p = __expf(s - slse[ii]);
      const float dp = dot32(v, sdo + ii * kD);
      const float ds = p * (dp - sdd[ii]);
      const float4* q4 = reinterpret_cast<const float4*>(sq + ii * kD);
      const float4* d4 = reinterpret_cast<const float4*>(sdo + ii * kD);
#pragma unroll
      for (int c = 0; c < kD / 4; ++c) {
        const float4 qq = q4[c];
        const float4 dd = d4[c];
        dk[4 * c + 0] = fmaf(ds, qq.x, dk[4 * c + 0]);
        dk[4 * c + 1] = fmaf(ds, qq.y, dk[4 * c + 1]);
        dk[4 * c + 2] = fmaf(ds, qq.z, dk[4 * c + 2]);
        dk[4 * c + 3] = fmaf(ds, qq.w, dk[4 * c + 3]);
        dv[4 * c + 0] = fmaf(p, dd.x, dv[4 * c + 0]);
        dv[4 * c + 1] = fmaf(p, dd.y, dv[4 * c + 1]);
        dv[4 * c + 2] = fmaf(p, dd.z, dv[4 * c + 2]);
        dv[4 * c + 3] = fmaf(p, dd.w, dv[4 * c + 3]);
      }
      if (++txi == ws) { txi = 0; ++tyi; }
    }
#pragma unroll
    for (int c = 0; c < kD; ++c) dk[c] *= g.scale;
    store_row32(gwin + (size_t)j * C3 + 1 * C + h * kD, dk);
    store_row32(gwin + (size_t)j * C3 + 2 * C + h * kD, dv);
  }
  __syncthreads();
  float* gp = gtable_part + ((size_t)bw * g.heads + h) * T2;
  for (int t = threadIdx.x; t < T2; t += blockDim.x) gp[t] = sbins[t];
}

// ---------------------------------------------------------------------------------------
// bf16 MFMA path (windows of N <= 64 tokens, e.g. Swin ws = 7; N <= 160 below): one wave per (window,
// head).  v_mfma_f32_32x32x16_bf16 fragments (lane l: r = l & 31, hh = l >> 5):
//   A: row r, k = 8hh + j;  B: col r, k = 8hh + j;  C/D: col r, row (i&3) + 8(i>>2) + 4hh.
// Forward: S^T = K Q^T (keys on rows, 2x2 tiles over the 64-padded window), so a lane
// holds 32 keys of ONE query: the softmax is in-register plus one lane^32 exchange.  Then
// O^T = V^T P^T takes P^T straight from the accumulators: the MFMA's k index is mapped to
// keys in the C layout's row order (k = 8hh + j  <->  key 16t + (j&3) + 8(j>>2) + 4hh) and
// the A operand (V^T, staged in LDS) is read in that same order, so P never leaves
// registers.  Backward: win_attn_bwd_fa below (two phases, any N <= 160).

constexpr int kMaxT2 = 225;       // (2*8-1)^2
constexpr int kZoneSmall = 7 * 16 + 1;   // bias_zone for ws <= 8
constexpr int kPadK = 72;         // LDS row pitch (shorts) of the 64-token operands

// Token metadata of the window: tok[t] = kk << 16 | region with kk = ty (2ws-1) + tx, so
// the relative-position index of a (query, key) pair is kk_q - kk_k + (ws-1) 2ws
// (HF:swin:350-365: (ty_q - ty_k + ws-1)(2ws-1) + tx_q - tx_k + ws-1) -- one subtract per
// logit, no integer multiply.  Region ids as HF:swin:584-607 (padded-grid position).
// A padded token (t >= N) gets kk = rel_c0 - T2: every pair it forms with a real token
// then indexes one of the two -inf zones staged around the bias table (stage_bias), so
// padded keys drop out of the softmax with no per-logit test.
__device__ __forceinline__ int rel_c0(const WinGeom& g) { return (g.ws - 1) * 2 * g.ws; }

__device__ __forceinline__ int token_meta(const WinGeom& g, int bw, int t) {
  if (t >= g.N) return (int)((unsigned)(rel_c0(g) - g.T2) << 16);
  const int ws = g.ws;
  const int wl = bw - div_nw(g, bw) * (g.nWh * g.nWw);
  const int wy = div_nWw(g, wl), wx = wl - wy * g.nWw;
  const int ty = div_ws(g, t), tx = t - ty * ws;
  const int reg = g.shift > 0 ? region_of(wy * ws + ty, g.nWh * ws, ws, g.shift) * 3 +
                                    region_of(wx * ws + tx, g.nWw * ws, ws, g.shift)
                              : 0;
  return (int)((unsigned)(ty * (2 * ws - 1) + tx) << 16) | reg;
}

// Only windows of the last window row / column of a shifted block mix regions (the roll
// wraps there); every other window skips the mask with a uniform branch.
__device__ __forceinline__ bool window_mixed(const WinGeom& g, int bw) {
  const int wl = bw - div_nw(g, bw) * (g.nWh * g.nWw);
  const int wy = div_nWw(g, wl);
  return g.shift > 0 && (wy == g.nWh - 1 || wl - wy * g.nWw == g.nWw - 1);
}

__device__ __forceinline__ void window_tokens(const WinGeom& g, int bw, int lane, int* tok) {
  tok[lane] = token_meta(g, bw, lane);
}

// Logits in log2 units (softmax through exp2): S2 = (q.k) scale log2e + table log2e
// (+ mask -100 log2e).  The staged bias is [zone | table column | zone], zone = rel_c0 + 1
// entries of -inf (the reach of a padded token's kk); `bias` points at the table.
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kMaskLog2 = -100.f * kLog2e;

__device__ __forceinline__ int bias_zone(const WinGeom& g) { return rel_c0(g) + 1; }

__device__ __forceinline__ float* stage_bias(float* sb, const float* table, const WinGeom& g, int h, int tid,
                                             int nthr) {
  const int z = bias_zone(g), n = g.T2 + 2 * z;
  for (int t = tid; t < n; t += nthr) {
    const int k = t - z;
    sb[t] = (k >= 0 && k < g.T2) ? table[k * g.heads + h] * kLog2e : -INFINITY;
  }
  return sb + z;
}

// Scaled logits + bias of an S^T tile (rows = keys 32 kt + crow(i, hh) in the registers,
// column = query q on the lane), padded keys -inf through the zones.  rel[i] receives each
// logit's bias index (the backward bins dS with it).  tok must be 16-B aligned.
__device__ __forceinline__ void logits_kq(f32x16_t& s, const WinGeom& g, float scale2, const int* tok,
                                          const float* bias, int kt, int q, int hh, int* rel) {
  const int qo = (tok[q] >> 16) + rel_c0(g);
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const int kb = 32 * kt + 8 * g4 + 4 * hh;
    const int4 t4 = *reinterpret_cast<const int4*>(tok + kb);
    const int tk[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = 4 * g4 + e;
      const int rl = qo - (tk[e] >> 16);
      rel[i] = rl;
      s[i] = fmaf(s[i], scale2, bias[rl]);
    }
  }
}

// the shift mask of the same tile (mixed windows only)
__device__ __forceinline__ void mask_kq(f32x16_t& s, const int* tok, int kt, int q, int hh) {
  const int rq = tok[q] & 0xffff;
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const int4 t4 = *reinterpret_cast<const int4*>(tok + 32 * kt + 8 * g4 + 4 * hh);
    const int tk[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if ((tk[e] & 0xffff) != rq) s[4 * g4 + e] += kMaskLog2;
  }
}

__device__ __forceinline__ void logits_tile(f32x16_t& s, const WinGeom& g, float scale2, bool mixed, const int* tok,
                                            const float* bias, int kt, int qt, int r, int hh) {
  int rel[16];
  logits_kq(s, g, scale2, tok, bias, kt, 32 * qt + r, hh, rel);
  if (mixed) mask_kq(s, tok, kt, 32 * qt + r, hh);
}

// The same logits for an S tile (rows = queries 32 qt + crow(i, hh), column = key on the
// lane): identical values to logits_kq for every (query, key) pair; a padded query row or
// padded key column is -inf through the zones.
__device__ __forceinline__ void logits_qk(f32x16_t& s, const WinGeom& g, float scale2, bool mixed, const int* tok,
                                          const float* bias, int qt, int key, int hh) {
  const int tk = tok[key];
  const int ko = (tk >> 16) - rel_c0(g), rk = tk & 0xffff;
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const int4 t4 = *reinterpret_cast<const int4*>(tok + 32 * qt + 8 * g4 + 4 * hh);
    const int tq[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) s[4 * g4 + e] = fmaf(s[4 * g4 + e], scale2, bias[(tq[e] >> 16) - ko]);
  }
  if (mixed) {
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int4 t4 = *reinterpret_cast<const int4*>(tok + 32 * qt + 8 * g4 + 4 * hh);
      const int tq[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if ((tq[e] & 0xffff) != rk) s[4 * g4 + e] += kMaskLog2;
    }
  }
}

__device__ __forceinline__ float exp2_fast(float x) { return __builtin_amdgcn_exp2f(x); }

constexpr int kFwdWaves = 4;

__global__ void __launch_bounds__(64 * kFwdWaves, 3) win_attn_fwd_mfma(const bf16* __restrict__ qkv,
                                                                    const float* __restrict__ table,
                                                                    bf16* __restrict__ out, float* __restrict__ lse,
                                                                    WinGeom g, int items) {
  __shared__ __attribute__((aligned(16))) short sVt[kFwdWaves][32 * kPadK];   // V^T [d][key]
  __shared__ float sBias[kFwdWaves][kMaxT2 + 2 * kZoneSmall];
  __shared__ __attribute__((aligned(16))) int sTok[kFwdWaves][64];
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int item = blockIdx.x * kFwdWaves + wave;
  if (item >= items) return;                  // wave-uniform; only wave-level syncs below
  const int h = item % g.heads, bw = item / g.heads;
  const int N = g.N, C = g.heads * kD, C3 = 3 * C;
  const bf16* win = qkv + (size_t)bw * N * C3;
  short* vt = sVt[wave];
  int* tok = sTok[wave];
  window_tokens(g, bw, l, tok);
  const float* bias = stage_bias(sBias[wave], table, g, h, l, 64);
  const bool mixed = window_mixed(g, bw);
  const float scale2 = g.scale * kLog2e;
  {  // V^T: lane = key
    const int key = l;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      bf16x8_t v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (key < N) v = ld8(win + (size_t)key * C3 + 2 * C + h * kD + 8 * c);
#pragma unroll
      for (int j = 0; j < 8; ++j) vt[(8 * c + j) * kPadK + key] = v[j];
    }
  }
  // S^T = K Q^T
  f32x16_t acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    bf16x8_t ka[2], qb[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int row = 32 * t + r;
      const bf16x8_t z = {0, 0, 0, 0, 0, 0, 0, 0};
      ka[t] = row < N ? ld8(win + (size_t)row * C3 + C + h * kD + 16 * st + 8 * hh) : z;
      qb[t] = row < N ? ld8(win + (size_t)row * C3 + h * kD + 16 * st + 8 * hh) : z;
    }
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
        acc[kt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka[kt], qb[qt], acc[kt][qt], 0, 0, 0);
  }
  wave_sync();                                // tok / bias / V^T visible to the whole wave
  float inv[2], lq[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    logits_tile(acc[0][qt], g, scale2, mixed, tok, bias, 0, qt, r, hh);
    logits_tile(acc[1][qt], g, scale2, mixed, tok, bias, 1, qt, r, hh);
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) m = fmaxf(m, fmaxf(acc[0][qt][i], acc[1][qt][i]));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      acc[0][qt][i] = exp2_fast(acc[0][qt][i] - m);
      acc[1][qt][i] = exp2_fast(acc[1][qt][i] - m);
      sum += acc[0][qt][i] + acc[1][qt][i];
    }
    sum += __shfl_xor(sum, 32, 64);
    inv[qt] = 1.f / sum;
    lq[qt] = (m + __log2f(sum)) * (1.f / kLog2e);
  }
  // O^T = V^T P^T
  f32x16_t o[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[qt][i] = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int kt = t >> 1, th = t & 1;
    const bf16x8_t a = ld_perm(vt + r * kPadK, 32 * kt + 16 * th + 4 * hh);
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
      o[qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, pack8(acc[kt][qt], 8 * th), o[qt], 0, 0, 0);
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = 32 * qt + r;
    const long long orow = q < N ? out_row(g, bw, q) : -1;
    if (q < N && hh == 0) lse[((size_t)bw * g.heads + h) * N + q] = lq[qt];
    if (orow >= 0) {
      bf16* dst = out + orow * C + h * kD;
#pragma unroll
      for (int grp = 0; grp < 4; ++grp) {
        bf16x4_t v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = bf16_bits(o[qt][4 * grp + e] * inv[qt]);
        *reinterpret_cast<bf16x4_t*>(dst + 8 * grp + 4 * hh) = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// bf16 MFMA path for windows of 64 < N <= 32*NT tokens (Swin-B/L ws = 12: N = 144, NT = 5).
// One workgroup per (window, head), one wave per 32-query tile; fragments as above.
// Forward: K (natural [key][d]) and V^T ([d][key]) of the window staged once in LDS; a
// wave forms S^T for all NT key tiles of its queries (NT accumulators), softmax in
// registers, and O^T = V^T P^T with P^T straight from the accumulators (permuted k).
// Backward: a wave forms S^T and dP^T for its queries (2 NT accumulators) and writes P^T
// to a shared [key][q] LDS tile (which aliases the K/V staging); after a block barrier
// wave w computes dV of key tile w over all queries; the tile is then overwritten with
// dS^T for dK of key tile w; dQ^T of the wave's queries comes from registers as above.
constexpr int kMaxT2Big = 529;    // (2*12-1)^2
constexpr int kZoneBig = 11 * 24 + 1;    // bias_zone for ws <= 12

// ---- fp8 (OCP e4m3, gfx950) window attention, config C5 ------------------------------
// F8 = true runs the forward's logits S^T = K Q^T and O^T = V^T P^T on the BLOCK-SCALED MX
// MFMA v_mfma_scale_f32_32x32x64_f8f6f4 with e4m3 operands: 2x the bf16 MFMA rate per clock
// on gfx950 (MI355X_MICROARCH.md §Matrix cores), the dequantisation fused into the
// instruction.  Operand layout, as measured on the box (tools/micro/mfma_scale_probe.hip,
// profiles/r3_mfma_scale_probe.txt): K = 64 is two 32-deep scale blocks; lane l (row /
// column l&31, half hh = l>>5) holds 16 elements of block 0 in its dwords 0-3 and 16 of
// block 1 in dwords 4-7 (the two lanes of a row hold all 32 of each block; any k order
// works as long as A and B agree), and its e8m0 scale byte (2^(e-127)) is the scale of
// block hh of its row / column.
//   * logits: the head dimension (32) is block 0 (block 1 is zero): lane half hh carries
//     channels 16hh..16hh+15, so every q and k TOKEN gets its own power-of-two scale (amax
//     over its 32 channels);
//   * P V: 64 keys per instruction, block 0 = key tile 2b, block 1 = tile 2b+1; lane half
//     hh takes its own accumulator rows (crow(., hh)) of both tiles, so P comes straight
//     from the registers, at one fixed scale (mx_pfixed); V has one scale per (window, head).
// Operands stay bf16 in HBM; the backward recomputes S from the same e4m3 values,
// dequantised exactly to bf16 (the logits agree to f32 rounding, so exp(S - lse) is the
// forward's P), and forms every gradient product in bf16 from the bf16 operands
// (straight-through quantisation).
// MX helpers (i32x8_t, mfma_mx, e4m3 conversions, amax / scale exponents): mx_util.h

// a token's channels 16hh..16hh+15 (two 16-B bf16 chunks) -> its logit operand: block 0 =
// the token (scale from all 32 channels), block 1 zero.  Returns the lane's scale byte.
__device__ __forceinline__ int mx_token(bf16x8_t c0, bf16x8_t c1, int hh, i32x8_t& q) {
  const unsigned am = xhalf_max_bits(max(amax8_bits(c0), amax8_bits(c1)));
  const int k = mx_exp_bits(am);
  const float inv = __builtin_ldexpf(1.f, -k);
  const uint4 u0 = bits128(c0), u1 = bits128(c1);
  q[0] = e4m3x4(u0.x, u0.y, inv);
  q[1] = e4m3x4(u0.z, u0.w, inv);
  q[2] = e4m3x4(u1.x, u1.y, inv);
  q[3] = e4m3x4(u1.z, u1.w, inv);
  q[4] = q[5] = q[6] = q[7] = 0;
  return hh == 0 ? 127 - k : 127;
}

__device__ __forceinline__ int mx_token_gmem(const bf16* row, int hh, bool valid, i32x8_t& q) {
  const bf16x8_t c0 = valid ? ld8(row + 16 * hh) : zero8();
  const bf16x8_t c1 = valid ? ld8(row + 16 * hh + 8) : zero8();
  return mx_token(c0, c1, hh, q);
}

// P = exp(S - max) <= 1 as an MX operand with ONE fixed scale: e4m3(256 P), scale byte
// 127 - 8.  A per-block scale would pick 2^8 too for every block holding its row's maximum
// and differs only below 2^-14 (subnormal e4m3 here), so no amax is needed; `at(j)` yields
// this lane's element j (16 of K-block 0, then 16 of block 1)
constexpr int kPScaleByte = 127 - 8;
template <typename F>
__device__ __forceinline__ void mx_pfixed(F at, i32x8_t& q) {
  constexpr float inv = 1.f / 256.f;
#pragma unroll
  for (int w = 0; w < 8; ++w) {
    s16x2_t r = {0, 0};
    r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(r, at(4 * w), at(4 * w + 1), inv, false);
    r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(r, at(4 * w + 2), at(4 * w + 3), inv, true);
    q[w] = __builtin_bit_cast(int, r);
  }
}

// Staging-time quantisation of a token held as 4 lanes x 8 channels (lane & 3 = chunk):
// the token's amax over its 32 channels (two shuffles), its e4m3 bytes (x 2^k, the same
// bytes mx_token makes from the same values) and its scale byte.
__device__ __forceinline__ uint2 mx_chunk8(bf16x8_t c, int* scale_byte) {
  const unsigned am = umax_xor(umax_xor(amax8_bits(c), 1), 2);
  const int k = mx_exp_bits(am);
  const float inv = __builtin_ldexpf(1.f, -k);
  const uint4 u = bits128(c);
  *scale_byte = 127 - k;
  return make_uint2((unsigned)e4m3x4(u.x, u.y, inv), (unsigned)e4m3x4(u.z, u.w, inv));
}

// a token's logit operand from its staged e4m3 row (32 bytes at `row8`): lane half hh
// takes bytes 16hh..16hh+15 as K-block 0, block 1 zero; scale byte of block hh
__device__ __forceinline__ int mx_token_lds8(const unsigned char* row8, int scale_byte, int hh, i32x8_t& q) {
  const uint4 v = *reinterpret_cast<const uint4*>(row8 + 16 * hh);
  q[0] = (int)v.x; q[1] = (int)v.y; q[2] = (int)v.z; q[3] = (int)v.w;
  q[4] = q[5] = q[6] = q[7] = 0;
  return hh == 0 ? scale_byte : 127;
}

// e4m3 round trip of 8 bf16 values at scale 2^k, back in bf16 (exact: e4m3 values carry 4
// significant bits): the dequantised operand the fp8 logits were formed from
__device__ __forceinline__ bf16x8_t fp8_roundtrip8(bf16x8_t c, int k) {
  const float inv = __builtin_ldexpf(1.f, -k);
  const uint4 u = bits128(c);
  const unsigned in[4] = {u.x, u.y, u.z, u.w};
  unsigned o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const s16x2_t r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(s16x2_t{0, 0}, __builtin_bit_cast(bf16x2v_t, in[j]),
                                                                inv, false);
    o[j] = __builtin_bit_cast(unsigned,
                              __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(__builtin_bit_cast(unsigned, r), inv, false));
  }
  return __builtin_bit_cast(bf16x8_t, make_uint4(o[0], o[1], o[2], o[3]));
}

// a staged token chunk (4 lanes x 8 channels) rounded through e4m3 at its token scale
__device__ __forceinline__ bf16x8_t fp8_token_chunk(bf16x8_t c) {
  return fp8_roundtrip8(c, mx_exp_bits(umax_xor(umax_xor(amax8_bits(c), 1), 2)));
}

// this lane's half-token (two chunks) rounded through e4m3 at the token's scale
__device__ __forceinline__ void fp8_token_lane(bf16x8_t* c) {
  const int k = mx_exp_bits(xhalf_max_bits(max(amax8_bits(c[0]), amax8_bits(c[1]))));
  c[0] = fp8_roundtrip8(c[0], k);
  c[1] = fp8_roundtrip8(c[1], k);
}

// (window, head) of a one-workgroup-per-(window, head) kernel.  1-D launches (the default):
// the heads of a window are consecutive logical workgroups on ONE XCD (xcd_swizzle): a
// head's slice of a qkv / out / grad row is 64 B, half a 128-B line, so a window's heads
// share every line they read or write and meet in that XCD's L2 instead of each pulling
// (and, for the gradients, partially writing back) whole lines on different XCDs at
// different times.  2-D launches (gridDim.y = heads): blockIdx as is.
__device__ __forceinline__ void win_block(const WinGeom& g, int& bw, int& h) {
  if (gridDim.y > 1) {
    bw = blockIdx.x;
    h = blockIdx.y;
    return;
  }
  const int lg = xcd_swizzle(blockIdx.x, gridDim.x);
  bw = lg / g.heads;
  h = lg - bw * g.heads;
}

template <int NT>
__device__ __forceinline__ void window_tokens_blk(const WinGeom& g, int bw, int* tok) {
  for (int t = threadIdx.x; t < 32 * NT; t += blockDim.x) tok[t] = token_meta(g, bw, t);
}

// Forward for 64 < N <= 160 (one workgroup per (window, head)) with an ONLINE softmax: a wave
// walks its key tiles keeping one S^T tile, the running max / sum and the O^T accumulator live
// (rescaled by exp2(m_old - m_new) per tile): 80 VGPRs instead of 120 for the two-pass form
// (all NT S^T tiles live; removed in round 6).  The kernel is latency-bound (SQ counters at C5,
// profiles/r3_win_pmc.txt: waves parked at waitcnt / barrier ~45-50 % of their cycles with 3
// workgroups per CU), so the registers buy resident workgroups: 4 per CU at NT = 5 (6 waves /
// SIMD) instead of 3 (C5 forward 0.88 -> 0.79 ms).  The tile loop stays rolled: unrolled, the
// scheduler hoists every tile's QK^T MFMAs and all S^T tiles are live again.
template <int NT>
__global__ void __launch_bounds__(64 * NT) __attribute__((amdgpu_waves_per_eu(6))) win_attn_fwd_online(const bf16* __restrict__ qkv,
                                                                   const float* __restrict__ table,
                                                                   bf16* __restrict__ out, float* __restrict__ lse,
                                                                   WinGeom g) {
  constexpr int NP = 32 * NT, PT = NP + 8, PK = 40;
  __shared__ __attribute__((aligned(16))) short sK[NP * PK];   // K [key][d]
  __shared__ __attribute__((aligned(16))) short sVt[32 * PT];  // V^T [d][key]
  __shared__ float sBias[kMaxT2Big + 2 * kZoneBig];
  __shared__ __attribute__((aligned(16))) int sTok[NP];
  int bw, h;
  win_block(g, bw, h);
  const int qt = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int N = g.N, C = g.heads * kD, C3 = 3 * C;
  const bf16* win = qkv + (size_t)bw * N * C3;
  bf16x8_t qb[2];
  {
    bf16x8_t ck[2], cv[2];
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int p = threadIdx.x + it * 64 * NT, t = p >> 2, c = p & 3;
      const bf16* row = win + (size_t)t * C3 + h * kD + 8 * c;
      ck[it] = t < N ? ld8(row + C) : zero8();
      cv[it] = t < N ? ld8(row + 2 * C) : zero8();
    }
    const int qrow = 32 * qt + r;
#pragma unroll
    for (int st = 0; st < 2; ++st)
      qb[st] = qrow < N ? ld8(win + (size_t)qrow * C3 + h * kD + 16 * st + 8 * hh) : zero8();
    window_tokens_blk<NT>(g, bw, sTok);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int p = threadIdx.x + it * 64 * NT, t = p >> 2, c = p & 3;
      *reinterpret_cast<bf16x8_t*>(sK + t * PK + 8 * c) = ck[it];
#pragma unroll
      for (int j = 0; j < 8; ++j) sVt[(8 * c + j) * PT + t] = cv[it][j];
    }
  }
  const float* bias = stage_bias(sBias, table, g, h, threadIdx.x, blockDim.x);
  const bool mixed = window_mixed(g, bw);
  const float scale2 = g.scale * kLog2e;
  __syncthreads();
  float m = -INFINITY, sum = 0.f;
  f32x16_t o;
  zero16(o);
#pragma unroll 1
  for (int kt = 0; kt < NT; ++kt) {            // not unrolled: the scheduler would hoist every
    f32x16_t s;                                // tile's QK^T MFMAs and keep all S^T tiles live
    zero16(s);
#pragma unroll
    for (int st = 0; st < 2; ++st)
      s = mfma16(*reinterpret_cast<const bf16x8_t*>(sK + (32 * kt + r) * PK + 16 * st + 8 * hh), qb[st], s);
    logits_tile(s, g, scale2, mixed, sTok, bias, kt, qt, r, hh);
    float tm = s[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) tm = fmaxf(tm, s[i]);
    tm = fmaxf(tm, __shfl_xor(tm, 32, 64));
    const float mn = fmaxf(m, tm);            // finite: every tile of a real query holds a real key
    if (kt > 0) {                             // (tile 0 always does; padded query lanes are never stored)
      const float alpha = exp2_fast(m - mn);
      sum *= alpha;
#pragma unroll
      for (int i = 0; i < 16; ++i) o[i] *= alpha;
    }
    m = mn;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      s[i] = exp2_fast(s[i] - mn);
      sum += s[i];
    }
#pragma unroll
    for (int th = 0; th < 2; ++th)
      o = mfma16(ld_perm(sVt + r * PT, 32 * kt + 16 * th + 4 * hh), pack8(s, 8 * th), o);
  }
  sum += __shfl_xor(sum, 32, 64);
  const int q = 32 * qt + r;
  const long long orow = q < N ? out_row(g, bw, q) : -1;
  if (q < N && hh == 0) lse[((size_t)bw * g.heads + h) * N + q] = (m + __log2f(sum)) * (1.f / kLog2e);
  if (orow >= 0) {
    const float inv = 1.f / sum;
    bf16* dst = out + orow * C + h * kD;
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) {
      bf16x4_t v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = bf16_bits(o[4 * grp + e] * inv);
      *reinterpret_cast<bf16x4_t*>(dst + 8 * grp + 4 * hh) = v;
    }
  }
}

// fp8 forward (C5): K and V are quantised ONCE per workgroup while staged -- K per token
// (e4m3 rows + a scale byte each), V with one power-of-two scale for the (window, head),
// stored transposed as bytes -- so every wave reads ready MX operands from LDS (half the
// bytes of the bf16 staging) and only quantises its own query and its P tiles (per
// (query, 32-key tile) scale, in registers).
template <int NT, bool ONLINE>
__global__ void __launch_bounds__(64 * NT) __attribute__((amdgpu_waves_per_eu(ONLINE ? 5 : NT == 5 ? 4 : 1))) win_attn_fwd_mx(const bf16* __restrict__ qkv, const float* __restrict__ table,
                                                           bf16* __restrict__ out, float* __restrict__ lse, WinGeom g) {
  constexpr int NP = 32 * NT, PK8 = 48, PV8 = NP + 16;      // bytes per K row / V^T row
  __shared__ __attribute__((aligned(16))) unsigned char sK8[NP * PK8];
  __shared__ __attribute__((aligned(16))) unsigned char sV8[32 * PV8];
  __shared__ int sKs[NP];
  __shared__ unsigned sVam[NT];
  __shared__ float sBias[kMaxT2Big + 2 * kZoneBig];
  __shared__ __attribute__((aligned(16))) int sTok[NP];
  int bw, h;
  win_block(g, bw, h);
  const int qt = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int N = g.N, C = g.heads * kD, C3 = 3 * C;
  const bf16* win = qkv + (size_t)bw * N * C3;
  bf16x8_t ck[2], cv[2];
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int p = threadIdx.x + it * 64 * NT, t = p >> 2, c = p & 3;
    const bf16* row = win + (size_t)t * C3 + h * kD + 8 * c;
    ck[it] = t < N ? ld8(row + C) : zero8();
    cv[it] = t < N ? ld8(row + 2 * C) : zero8();
  }
  const int qrow = 32 * qt + r;
  i32x8_t qm;
  const int qs = mx_token_gmem(win + (size_t)qrow * C3 + h * kD, hh, qrow < N, qm);
  window_tokens_blk<NT>(g, bw, sTok);
  const float* bias = stage_bias(sBias, table, g, h, threadIdx.x, blockDim.x);
  const bool mixed = window_mixed(g, bw);
  const float scale2 = g.scale * kLog2e;
  unsigned vam = 0;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int p = threadIdx.x + it * 64 * NT, t = p >> 2, c = p & 3;
    int sb;
    *reinterpret_cast<uint2*>(sK8 + t * PK8 + 8 * c) = mx_chunk8(ck[it], &sb);
    if (c == 0) sKs[t] = sb;
    vam = max(vam, amax8_bits(cv[it]));
  }
#pragma unroll
  for (int sft = 32; sft >= 1; sft >>= 1) vam = umax_xor(vam, sft);
  if (l == 0) sVam[qt] = vam;
  __syncthreads();
  unsigned va = 0;
#pragma unroll
  for (int w = 0; w < NT; ++w) va = max(va, sVam[w]);
  const int kv = mx_exp_bits(va);
  const float vinv = __builtin_ldexpf(1.f, -kv);
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int p = threadIdx.x + it * 64 * NT, t = p >> 2, c = p & 3;
    const uint4 u = bits128(cv[it]);
    const int w0 = e4m3x4(u.x, u.y, vinv), w1 = e4m3x4(u.z, u.w, vinv);
#pragma unroll
    for (int j = 0; j < 8; ++j) sV8[(8 * c + j) * PV8 + t] = (unsigned char)(((j < 4 ? w0 : w1) >> (8 * (j & 3))) & 0xff);
  }
  __syncthreads();
  if constexpr (ONLINE) {
    // online softmax over key-tile PAIRS (one MX P V instruction each): two S^T tiles, the
    // running max / sum and O^T live (see win_attn_fwd_online)
    float m = -INFINITY, sum = 0.f;
    f32x16_t o;
    zero16(o);
    const int vsb = 127 - kv;
#pragma unroll 1
    for (int b2 = 0; b2 < (NT + 1) / 2; ++b2) {
      const int k0 = 2 * b2, k1 = 2 * b2 + 1;
      const bool has1 = k1 < NT;
      f32x16_t s0, s1;
      zero16(s0);
      zero16(s1);
      {
        i32x8_t km;
        const int key = 32 * k0 + r;
        const int ks = mx_token_lds8(sK8 + key * PK8, sKs[key], hh, km);
        s0 = mfma_mx(km, ks, qm, qs, s0);
      }
      logits_tile(s0, g, scale2, mixed, sTok, bias, k0, qt, r, hh);
      if (has1) {
        i32x8_t km;
        const int key = 32 * k1 + r;
        const int ks = mx_token_lds8(sK8 + key * PK8, sKs[key], hh, km);
        s1 = mfma_mx(km, ks, qm, qs, s1);
        logits_tile(s1, g, scale2, mixed, sTok, bias, k1, qt, r, hh);
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) s1[i] = -INFINITY;
      }
      float tm = fmaxf(s0[0], s1[0]);
#pragma unroll
      for (int i = 1; i < 16; ++i) tm = fmaxf(tm, fmaxf(s0[i], s1[i]));
      tm = fmaxf(tm, __shfl_xor(tm, 32, 64));
      const float mn = fmaxf(m, tm);
      if (b2 > 0) {
        const float alpha = exp2_fast(m - mn);
        sum *= alpha;
#pragma unroll
        for (int i = 0; i < 16; ++i) o[i] *= alpha;
      }
      m = mn;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        s0[i] = exp2_fast(s0[i] - mn);
        s1[i] = exp2_fast(s1[i] - mn);
        sum += s0[i] + s1[i];
      }
      i32x8_t vm, pm;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4)
          vm[4 * u + g4] = (u == 0 || has1)
                               ? *reinterpret_cast<const int*>(sV8 + r * PV8 + 32 * (u ? k1 : k0) + 8 * g4 + 4 * hh)
                               : 0;
      mx_pfixed([&](int j) { return j < 16 ? s0[j] : s1[j - 16]; }, pm);
      o = mfma_mx(vm, vsb, pm, kPScaleByte, o);
    }
    sum += __shfl_xor(sum, 32, 64);
    const long long orow = qrow < N ? out_row(g, bw, qrow) : -1;
    if (qrow < N && hh == 0) lse[((size_t)bw * g.heads + h) * N + qrow] = (m + __log2f(sum)) * (1.f / kLog2e);
    if (orow >= 0) {
      const float inv = 1.f / sum;
      bf16* dst = out + orow * C + h * kD;
#pragma unroll
      for (int grp = 0; grp < 4; ++grp) {
        bf16x4_t v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = bf16_bits(o[4 * grp + e] * inv);
        *reinterpret_cast<bf16x4_t*>(dst + 8 * grp + 4 * hh) = v;
      }
    }
    return;
  }
  // S^T = K Q^T: the staged key rows straight into the MX MFMA
  f32x16_t acc[NT];
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    zero16(acc[kt]);
    i32x8_t km;
    const int key = 32 * kt + r;
    const int ks = mx_token_lds8(sK8 + key * PK8, sKs[key], hh, km);
    acc[kt] = mfma_mx(km, ks, qm, qs, acc[kt]);
  }
  float m = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    logits_tile(acc[kt], g, scale2, mixed, sTok, bias, kt, qt, r, hh);
#pragma unroll
    for (int i = 0; i < 16; ++i) m = fmaxf(m, acc[kt][i]);
  }
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int kt = 0; kt < NT; ++kt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      acc[kt][i] = exp2_fast(acc[kt][i] - m);
      sum += acc[kt][i];
    }
  sum += __shfl_xor(sum, 32, 64);
  const float lq = (m + __log2f(sum)) * (1.f / kLog2e);
  const float inv = 1.f / sum;
  // O^T = V^T P^T, 64 keys (tiles 2 b2, 2 b2 + 1) per instruction; lane half hh takes the
  // keys of its accumulator rows crow(., hh): 4 consecutive keys = one V^T dword
  f32x16_t o;
  zero16(o);
  const int vsb = 127 - kv;
#pragma unroll
  for (int b2 = 0; b2 < (NT + 1) / 2; ++b2) {
    constexpr int kLast = NT - 1;
    const int k0 = 2 * b2, k1 = 2 * b2 + 1 < NT ? 2 * b2 + 1 : kLast;
    const bool has1 = 2 * b2 + 1 < NT;
    i32x8_t vm, pm;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        vm[4 * u + g4] = (u == 0 || has1)
                             ? *reinterpret_cast<const int*>(sV8 + r * PV8 + 32 * (u ? k1 : k0) + 8 * g4 + 4 * hh)
                             : 0;
    mx_pfixed([&](int j) { return j < 16 ? acc[k0][j] : (has1 ? acc[k1][j - 16] : 0.f); }, pm);
    o = mfma_mx(vm, vsb, pm, kPScaleByte, o);
  }
  const long long orow = qrow < N ? out_row(g, bw, qrow) : -1;
  if (qrow < N && hh == 0) lse[((size_t)bw * g.heads + h) * N + qrow] = lq;
  if (orow >= 0) {
    bf16* dst = out + orow * C + h * kD;
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) {
      bf16x4_t v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = bf16_bits(o[4 * grp + e] * inv);
      *reinterpret_cast<bf16x4_t*>(dst + 8 * grp + 4 * hh) = v;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Backward, flash-attention-2 split in two phases of ONE workgroup per (window, head),
// NT = ceil(N / 32) waves, any N <= 160 (Swin-T ws 7: NT = 2; Swin-B/L ws 12: NT = 5).
// The earlier kernels kept a whole query tile's S^T / dP^T rows in registers and a
// [key][query] P^T / dS^T tile in LDS: 203 VGPR + 128 AGPR (1 wave/SIMD) for N <= 64 and
// 89 KB of LDS (1 workgroup/CU) for N = 144.  Here each wave streams over 32-token tiles
// with only the current tile's S and dP (2 x 16 f32) and its output accumulators live:
//   phase 1 (wave = query tile qt):  for each key tile kt: S^T = K Q^T, dP^T = V dO^T,
//     P = exp(S - lse), dS = P (dP - D); dQ^T += K^T dS^T (dS^T straight from registers,
//     K^T read in the permuted key order); the bias gradient binned in the wave's own LDS
//     bins (for one register and one lane half the 32 queries of a key have 32 distinct
//     offsets, so the halves take turns and every update is a plain read-modify-write);
//   phase 2 (wave = key tile kw, after the staging is swapped): for each query tile qt:
//     S = Q K^T, dP = dO V^T (query rows, key columns), P, dS as above;
//     dV^T += dO^T P and dK^T += Q^T dS (P, dS straight from registers, dO^T / Q^T read
//     in the permuted query order).
// S and dP are formed twice (the MFMA units idle in this kernel); LDS peaks at ~47 KB for
// N = 144 (3 workgroups/CU).  F8: the logits on the forward's fp8 operands and scales.
// DBG: the parts switched off in the round-5 timing split (profiles/r5_win_bwd_ab.txt; 1 no bias
// binning, 2 no phase 2, 4 no phase-1 tile loop, 8 no bias gather); only DBG = 0 is instantiated
template <int NT, bool F8, int DBG = 0>
__global__ void __launch_bounds__(64 * NT, NT == 5 ? 4 : NT == 2 ? 3 : 1) win_attn_bwd_fa(
    const bf16* __restrict__ qkv, const float* __restrict__ table, const bf16* __restrict__ out,
    const float* __restrict__ lse, const bf16* __restrict__ gout, bf16* __restrict__ gqkv,
    float* __restrict__ gtable_part, WinGeom g) {
  constexpr int NP = 32 * NT, PT = NP + 8, PK = 40;
  constexpr int kNat = NP * PK, kTr = 32 * PT;
  constexpr int kT2 = NT <= 2 ? 225 : NT == 3 ? 289 : NT == 4 ? 441 : 529;   // (2 ws_max - 1)^2
  // NT <= 2 (Swin-T ws 7): each lane half has its own bins, so the halves need not take turns
  // (2 wave barriers per tile fewer); the 1.8 KB more LDS costs no occupancy at 128 threads.
  // Larger windows keep one set per wave (more LDS there lowers the workgroups per CU)
  constexpr bool kHalfBins = NT <= 2;
  constexpr int kBinW = kT2 * (kHalfBins ? 2 : 1);            // f32 bias-gradient bins per wave
  constexpr int kP1 = 2 * kNat + kTr + NT * kBinW * 2;        // K, V, K^T, f32 bins (in shorts)
  constexpr int kP2 = 2 * kNat + 2 * kTr;                     // Q, dO, Q^T, dO^T
  __shared__ __attribute__((aligned(16))) short sU[kP1 > kP2 ? kP1 : kP2];
  __shared__ float sBias[kMaxT2Big + 2 * kZoneBig];
  __shared__ __attribute__((aligned(16))) int sTok[NP];
  __shared__ float sL[NP], sD[NP];
  int bw, h;
  win_block(g, bw, h);
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int N = g.N, C = g.heads * kD, C3 = 3 * C;
  const bf16* win = qkv + (size_t)bw * N * C3 + h * kD;
  const bf16* gwo = gout + h * kD;            // rows through out_row (window or image layout)
  const bf16* owin = out + h * kD;
  bf16* gw = gqkv + (size_t)bw * N * C3 + h * kD;
  const float* lrow = lse + ((size_t)bw * g.heads + h) * N;
  // Every global operand of a phase is requested before any is used (one round trip per
  // phase): the staging chunks -- exactly two 16-B chunks per thread and tensor (NP x 4
  // chunks, 64 NT threads) --, this lane's query row slices (phase 1: Q, dO, O for
  // D = rowsum(dO * O), lse) or key row slices (phase 2: K, V).  Loading phase 2's operands
  // up front as well, or giving each lane half its own bias bins, measured 1.5x slower at
  // N = 144 (registers / LDS cost occupancy; tools/winbench.py).
  const int qt = wv, kw = wv;
  const int q = 32 * qt + r, key = 32 * kw + r;
  bf16x8_t ck[2], cv[2], cq[2], cd[2];
  auto load_p2 = [&]() {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int p = threadIdx.x + it * 64 * NT, t = p >> 2, c = p & 3;
      cq[it] = t < N ? ld8(win + (size_t)t * C3 + 8 * c) : zero8();
      const long long orow = t < N ? out_row(g, bw, t) : -1;
      cd[it] = orow >= 0 ? ld8(gwo + orow * C + 8 * c) : zero8();
    }
  };
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int p = threadIdx.x + it * 64 * NT, t = p >> 2, c = p & 3;
    const bool in = t < N;
    const bf16* row = win + (size_t)t * C3 + 8 * c;
    ck[it] = in ? ld8(row + C) : zero8();
    cv[it] = in ? ld8(row + 2 * C) : zero8();
  }
  bf16x8_t qb[2], db[2], ob[2], kb[2], vb[2];
  auto load_kv = [&]() {
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int off = 16 * st + 8 * hh;
      kb[st] = key < N ? ld8(win + (size_t)key * C3 + C + off) : zero8();
      vb[st] = key < N ? ld8(win + (size_t)key * C3 + 2 * C + off) : zero8();
    }
  };
  const long long qorow = q < N ? out_row(g, bw, q) : -1;
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    const int off = 16 * st + 8 * hh;
    qb[st] = q < N ? ld8(win + (size_t)q * C3 + off) : zero8();
    db[st] = qorow >= 0 ? ld8(gwo + qorow * C + off) : zero8();
    ob[st] = qorow >= 0 ? ld8(owin + qorow * C + off) : zero8();
  }

  const float Lq = q < N ? lrow[q] * kLog2e : 0.f;      // log2 units
  window_tokens_blk<NT>(g, bw, sTok);
  const float* bias = stage_bias(sBias, table, g, h, threadIdx.x, blockDim.x);
  const bool mixed = window_mixed(g, bw);
  const float scale2 = g.scale * kLog2e;
  // ---- phase 1 staging: K, V natural, K^T; D, lse; bins zeroed
  short* sKn = sU;
  short* sVn = sU + kNat;
  short* sKT = sU + 2 * kNat;
  float* sBins = reinterpret_cast<float*>(sU + 2 * kNat + kTr);
  // F8: natural-order K (read only by the logits) staged as the forward's e4m3 values
  // (per-token scale), dequantised back to bf16 exactly; the gradients use raw K (sKT)
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int p = threadIdx.x + it * 64 * NT, t = p >> 2, c = p & 3;
    *reinterpret_cast<bf16x8_t*>(sKn + t * PK + 8 * c) = F8 ? fp8_token_chunk(ck[it]) : ck[it];
    *reinterpret_cast<bf16x8_t*>(sVn + t * PK + 8 * c) = cv[it];
#pragma unroll
    for (int j = 0; j < 8; ++j) sKT[(8 * c + j) * PT + t] = ck[it][j];
  }
  float Dq = 0.f;
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      Dq += bf16_bits_to_f32((unsigned short)ob[st][j]) * bf16_bits_to_f32((unsigned short)db[st][j]);
  Dq += __shfl_xor(Dq, 32, 64);
  if (hh == 0) {
    sD[q] = Dq;
    sL[q] = Lq;
  }
  for (int t = threadIdx.x; t < NT * kBinW; t += blockDim.x) sBins[t] = 0.f;
  __syncthreads();
  const WinGeom& gl = g;
  bf16x8_t qs8[2] = {qb[0], qb[1]};          // F8: this lane's query as the forward's e4m3 values
  if (F8) fp8_token_lane(qs8);
  float* bins = sBins + qt * kBinW + (kHalfBins ? hh * kT2 : 0);
  f32x16_t dq;
  zero16(dq);
  for (int kt = 0; kt < ((DBG & 4) ? 0 : NT); ++kt) {
    f32x16_t s, dp;
    zero16(s);
    zero16(dp);
    // F8: the forward's logits from the same e4m3 values (dequantised exactly), summed in
    // another order: S agrees to f32 rounding, so exp(S - lse) is the forward's P
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int o = (32 * kt + r) * PK + 16 * st + 8 * hh;
      s = mfma16(*reinterpret_cast<const bf16x8_t*>(sKn + o), qs8[st], s);
      dp = mfma16(*reinterpret_cast<const bf16x8_t*>(sVn + o), db[st], dp);
    }
    int rel[16];
    if (DBG & 8) {
      for (int i = 0; i < 16; ++i) { s[i] *= scale2; rel[i] = 16 * kt + i; }
    } else {
      logits_kq(s, gl, scale2, sTok, bias, kt, q, hh, rel);
    }
    if (mixed) mask_kq(s, sTok, kt, q, hh);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = q < N ? exp2_fast(s[i] - Lq) : 0.f;
      dp[i] = p * (dp[i] - Dq);
    }
    // dQ^T += K^T dS^T
#pragma unroll
    for (int th = 0; th < 2; ++th) {
      const bf16x8_t a = ld_perm(sKT + r * PT, 32 * kt + 16 * th + 4 * hh);
      dq = mfma16(a, pack8(dp, 8 * th), dq);
    }
    // relative-position bias gradient: for one register the 32 lanes of a half hold one
    // key and 32 queries, i.e. 32 distinct bins, so with the halves taking turns every
    // update is a plain LDS read-modify-write (ds_add_f32 is slow on gfx950).  Padded
    // query lanes index the zone below the table and are masked off; a padded key row
    // (dS = 0 on every lane: P = exp2(-inf)) indexes the zone above it and is clamped onto
    // the last bin, where its whole instruction adds zero
    if (DBG & 1) {
    } else if (kHalfBins) {
      // one lane half, one register: 32 queries x one key = 32 distinct bins; LDS accesses
      // of a wave stay in program order, so the registers' read-modify-writes chain safely
      if (q < N) {
#pragma unroll
        for (int i = 0; i < 16; ++i) bins[min(rel[i], g.T2 - 1)] += dp[i];
      }
    } else {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        if (hh == half && q < N) {
#pragma unroll
          for (int i = 0; i < 16; ++i) bins[min(rel[i], g.T2 - 1)] += dp[i];
        }
        wave_sync();
      }
    }
  }
  if (q < N) {
    bf16* dst = gw + (size_t)q * C3;
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) {
      bf16x4_t v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = bf16_bits(dq[4 * grp + e] * g.scale);
      *reinterpret_cast<bf16x4_t*>(dst + 8 * grp + 4 * hh) = v;
    }
  }
  __syncthreads();                            // bins complete; phase-1 staging dead after this
  {
    float* gp = gtable_part + ((size_t)bw * g.heads + h) * g.T2;
    for (int t = threadIdx.x; t < g.T2; t += blockDim.x) {
      float a = 0.f;
#pragma unroll
      for (int w = 0; w < NT; ++w) {
        a += sBins[w * kBinW + t];
        if (kHalfBins) a += sBins[w * kBinW + kT2 + t];
      }
      gp[t] = a;
    }
  }
  if (DBG & 2) return;
  __syncthreads();
  // ---- phase 2 staging: Q, dO natural; Q^T, dO^T
  load_p2();
  load_kv();
  short* sQn = sU;
  short* sDn = sU + kNat;
  short* sQT = sU + 2 * kNat;
  short* sDT = sU + 2 * kNat + kTr;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int p = threadIdx.x + it * 64 * NT, t = p >> 2, c = p & 3;
    // F8: natural-order Q (read only by the logits) as its e4m3 values
    *reinterpret_cast<bf16x8_t*>(sQn + t * PK + 8 * c) = F8 ? fp8_token_chunk(cq[it]) : cq[it];
    *reinterpret_cast<bf16x8_t*>(sDn + t * PK + 8 * c) = cd[it];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sQT[(8 * c + j) * PT + t] = cq[it][j];
      sDT[(8 * c + j) * PT + t] = cd[it][j];
    }
  }
  bf16x8_t ks8[2] = {kb[0], kb[1]};          // F8: this lane's key as the forward's e4m3 values
  if (F8) fp8_token_lane(ks8);
  __syncthreads();
  f32x16_t dv, dk;
  zero16(dv);
  zero16(dk);
  for (int qq = 0; qq < NT; ++qq) {
    f32x16_t s, dp;
    zero16(s);
    zero16(dp);
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int o = (32 * qq + r) * PK + 16 * st + 8 * hh;
      s = mfma16(*reinterpret_cast<const bf16x8_t*>(sQn + o), ks8[st], s);
      dp = mfma16(*reinterpret_cast<const bf16x8_t*>(sDn + o), vb[st], dp);
    }
    if (DBG & 8) {
      for (int i = 0; i < 16; ++i) s[i] *= scale2;
    } else {
      logits_qk(s, gl, scale2, mixed, sTok, bias, qq, key, hh);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qi = 32 * qq + crow(i, hh);
      const float p = exp2_fast(s[i] - sL[qi]);
      s[i] = p;
      dp[i] = p * (dp[i] - sD[qi]);
    }
#pragma unroll
    for (int th = 0; th < 2; ++th) {
      const int base = 32 * qq + 16 * th + 4 * hh;
      dv = mfma16(ld_perm(sDT + r * PT, base), pack8(s, 8 * th), dv);
      dk = mfma16(ld_perm(sQT + r * PT, base), pack8(dp, 8 * th), dk);
    }
  }
  if (key < N) {
    bf16* dst = gw + (size_t)key * C3;
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) {
      bf16x4_t a, b;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[e] = bf16_bits(dk[4 * grp + e] * g.scale);
        b[e] = bf16_bits(dv[4 * grp + e]);
      }
      *reinterpret_cast<bf16x4_t*>(dst + C + 8 * grp + 4 * hh) = a;
      *reinterpret_cast<bf16x4_t*>(dst + 2 * C + 8 * grp + 4 * hh) = b;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Backward, round 5 (win_attn_bwd_fb): the same two phases as win_attn_bwd_fa with
//  * every operand staged ONCE in its natural [token][32] layout with 64-B rows, the 16-B
//    chunks XOR-swizzled by (token >> 2) & 3 (a row-major 16-lane read of one chunk column
//    and a 4-row ds_read_b64_tr_b16 read both cover all 64 banks): the transposed operands
//    (K^T for dQ, dO^T for dV, Q^T for dK) come from the transposed LDS read in the permuted
//    key / query order, so no [channel][token] copy is written (the fa kernel wrote it with
//    16 two-byte stores per chunk, a third of its LDS cycles were bank conflicts);
//  * the relative-position bias gradient accumulated as FIXED-POINT integers with no-return
//    ds_add_u32 into the wave's bins (integer LDS atomics run at ~12 lane-ops/clk/CU on
//    gfx950, f32 ones at 0.33; tools/micro/lds_atomic_bench.hip).  No lane halves taking
//    turns, no read-modify-write chains.  The wave's quantum is a power of two set from a
//    bound on what any of its bins can reach:
//      |dS_qk| = P_qk |dP_qk - D_q| <= P_qk (|dO_q| |V_k| + |dO_q| |O_q|) <= 2 P_qk |dO_q| Vmax
//    (|O_q| <= Vmax: O_q is a convex combination of V rows); a bin takes one key per query,
//    so |bin| <= 2 Vmax sum_{q of the wave} |dO_q| =: B, and the quantum 2^(e - 31) with
//    B < 2^e / 1.02 keeps every partial sum inside int32 (the 2 % covers the rounding of the
//    <= 160 terms).  Each term is rounded once, to 2^-32 B: the bins agree with f32 sums to
//    a few 1e-6 of the gradient's range (tests/test_gpu_ops.py).
__device__ __forceinline__ float sumsq8(bf16x8_t c) {
  float a = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = bf16_bits_to_f32((unsigned short)c[j]);
    a = fmaf(x, x, a);
  }
  return a;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// round half up to an integer (one instruction; __float2int_rn is two)
__device__ __forceinline__ int cvt_rpi(float x) {
  int r;
  asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// Per-logit work of the fb kernel, in VALU terms (the fa kernel spent ~290 VALU per 32x32
// tile of phase 1, the tile's 6 MFMAs ~190 cycles):
//  * the token metadata hold 4 kk (a byte offset) in the high half, so one subtract gives
//    the bias AND the bin byte offset; the bias table sits at a compile-time LDS address
//    (zone size fixed per NT), folded into the ds_read offset;
//  * dS is formed already scaled by the bins' inverse quantum 2^(31-e): the same products
//    (p (dp - D) scaled by a power of two is exact), so it feeds both the dQ MFMA (dQ is
//    scaled back at the store, exactly) and v_cvt_rpi_i32_f32 for the bin;
//  * a padded query has lse = +inf (P = 0 with no select).
//  * bias and bins are PITCHED: relative offset (dy, dx) at (dy + ws-1) P + dx + ws-1 with
//    P = ws + 32 (P = ws mod 32, so a token's pitched position y P + x is its raster index t
//    mod 32): the 32 lanes of a half-wave (32 consecutive query or key tokens) hit 32 distinct
//    banks in every bias read and every bin atomic (with rows of 2 ws - 1 they collided up to
//    3-way, ~40 % of the LDS-busy cycles were conflicts, profiles/r5_win_bwd_sq_c5.txt).
//    Columns 2 ws - 1 .. P-1 of a row are -inf in the bias: a padded KEY sits at x = -ws, so
//    every (real query, padded key) pair lands there (P = 0 with no zone rows);
// Padded queries / keys (dS = 0) index bins outside the wave's [0, T2): the bins of the
// neighbouring waves or the margins around them, where adding 0 changes nothing.
// DBG: the parts switched off in the round-5 timing split (1 no bins, 2 no phase 2, 4 no phase-1
// tile loop); only DBG = 0 is instantiated.  WPE 3 (3 waves / SIMD) measured 1.44 vs 1.21 ms at C5
template <int NT, bool F8, int WPE = F8 ? 3 : 4, int DBG = 0>
__global__ void __launch_bounds__(64 * NT) __attribute__((amdgpu_waves_per_eu(WPE))) win_attn_bwd_fb(
    const bf16* __restrict__ qkv, const float* __restrict__ table, const bf16* __restrict__ out,
    const float* __restrict__ lse, const bf16* __restrict__ gout, bf16* __restrict__ gqkv,
    float* __restrict__ gtable_part, WinGeom g) {
  constexpr int NP = 32 * NT, kImg = NP * 32;
  constexpr int kWs = NT <= 2 ? 8 : NT == 3 ? 9 : NT == 4 ? 11 : 12;           // ws_max
  constexpr int kBinW = (2 * kWs - 1) * (kWs + 32);                           // pitched bins
  constexpr int kZ = 16;                                                      // >= ws margin
  // phase 1: K (raw, for K^T), V [, K through e4m3 for the logits]; phase 2: Q, dO [, Q e4m3]
  __shared__ __attribute__((aligned(16))) short sU[(F8 ? 3 : 2) * kImg];
  __shared__ float sBias[kBinW + kZ];
  __shared__ int sBins[NT * kBinW + kZ];
  __shared__ __attribute__((aligned(16))) int sTok[NP];
  __shared__ float sL[NP], sD[NP];
  __shared__ float sVmax[NT], sQuant[NT];
  int bw, h;
  win_block(g, bw, h);
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int N = g.N, C = g.heads * kD, C3 = 3 * C;
  const bf16* win = qkv + (size_t)bw * N * C3 + h * kD;
  const bf16* gwo = gout + h * kD;
  const bf16* owin = out + h * kD;
  bf16* gw = gqkv + (size_t)bw * N * C3 + h * kD;
  const float* lrow = lse + ((size_t)bw * g.heads + h) * N;
  const int qt = wv, kw = wv;
  const int q = 32 * qt + r, key = 32 * kw + r;
  bf16x8_t ck[2], cv[2], cq[2], cd[2];
  auto load_p2 = [&]() {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int p = threadIdx.x + it * 64 * NT, t = p >> 2, c = p & 3;
      cq[it] = t < N ? ld8(win + (size_t)t * C3 + 8 * c) : zero8();
      const long long orow = t < N ? out_row(g, bw, t) : -1;
      cd[it] = orow >= 0 ? ld8(gwo + orow * C + 8 * c) : zero8();
    }
  };
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int p = threadIdx.x + it * 64 * NT, t = p >> 2, c = p & 3;
    const bool in = t < N;
    const bf16* row = win + (size_t)t * C3 + 8 * c;
    ck[it] = in ? ld8(row + C) : zero8();
    cv[it] = in ? ld8(row + 2 * C) : zero8();
  }
  bf16x8_t qb[2], db[2], ob[2], kb[2], vb[2];
  auto load_kv = [&]() {
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int off = 16 * st + 8 * hh;
      kb[st] = key < N ? ld8(win + (size_t)key * C3 + C + off) : zero8();
      vb[st] = key < N ? ld8(win + (size_t)key * C3 + 2 * C + off) : zero8();
    }
  };
  const long long qorow = q < N ? out_row(g, bw, q) : -1;
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    const int off = 16 * st + 8 * hh;
    qb[st] = q < N ? ld8(win + (size_t)q * C3 + off) : zero8();
    db[st] = qorow >= 0 ? ld8(gwo + qorow * C + off) : zero8();
    ob[st] = qorow >= 0 ? ld8(owin + qorow * C + off) : zero8();
  }

  const float Lq = q < N ? lrow[q] * kLog2e : INFINITY;      // log2 units; padded: P = 0
  // token metadata: 4 (y P + x) << 16 | region; a padded token at (0, -ws)
  const int ws = g.ws, P = ws + 32, R = 2 * ws - 1;
  for (int t = threadIdx.x; t < NP; t += blockDim.x) {
    const int m = token_meta(g, bw, t);
    const int ty = t / ws, kk = t < N ? ty * P + (t - ty * ws) : -ws;
    sTok[t] = (int)((unsigned)(4 * kk) << 16) | (m & 0xffff);
  }
  // [margin | (2ws-1) rows of P: table row (log2 units), -inf gap], margin -inf
  for (int t = threadIdx.x; t < kBinW + kZ; t += blockDim.x) {
    const int k = t - kZ, a = k / P, b = k - a * P;
    sBias[t] = (k >= 0 && a < R && b < R) ? table[(a * R + b) * g.heads + h] * kLog2e : -INFINITY;
  }
  const char* biasb = reinterpret_cast<const char*>(sBias + kZ);   // + 4 rel
  const bool mixed = window_mixed(g, bw);
  const float scale2 = g.scale * kLog2e;
  const int c04 = 4 * (ws - 1) * (P + 1);
  // ---- phase 1 staging: K, V natural (swizzled); D, lse; bins zeroed; the bound's maxima
  short* sK = sU;
  short* sV = sU + kImg;
  short* sKq = sU + 2 * kImg;
  float vmax2 = 0.f;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int p = threadIdx.x + it * 64 * NT, t = p >> 2, c = p & 3;
    *reinterpret_cast<bf16x8_t*>(sK + swz64(t, c)) = ck[it];
    *reinterpret_cast<bf16x8_t*>(sV + swz64(t, c)) = cv[it];
    if (F8) *reinterpret_cast<bf16x8_t*>(sKq + swz64(t, c)) = fp8_token_chunk(ck[it]);
    float v2 = sumsq8(cv[it]);                 // the token's 4 chunks sit on 4 adjacent lanes
    v2 += __shfl_xor(v2, 1, 64);
    v2 += __shfl_xor(v2, 2, 64);
    vmax2 = fmaxf(vmax2, v2);
  }
  float Dq = 0.f;
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      Dq += bf16_bits_to_f32((unsigned short)ob[st][j]) * bf16_bits_to_f32((unsigned short)db[st][j]);
  Dq += __shfl_xor(Dq, 32, 64);
  float dn = sumsq8(db[0]) + sumsq8(db[1]);
  dn = sqrtf(dn + __shfl_xor(dn, 32, 64));   // |dO_q| (0 for a padded query)
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) dn += __shfl_xor(dn, o, 64);   // sum over the wave's queries
  vmax2 = wave_max(vmax2);
  if (l == 0) sVmax[wv] = vmax2;
  if (hh == 0) {
    sD[q] = Dq;
    sL[q] = Lq;
  }
  for (int t = threadIdx.x; t < NT * kBinW + kZ; t += blockDim.x) sBins[t] = 0;
  __syncthreads();
  float vm = 0.f;
#pragma unroll
  for (int w = 0; w < NT; ++w) vm = fmaxf(vm, sVmax[w]);
  const float bound = 2.04f * sqrtf(vm) * dn;
  int e = -96;                                // keeps 2^(31 - e) a normal f32
  if (bound > 0.f && bound < INFINITY) {
    (void)frexpf(bound, &e);                  // bound < 2^e
    e = max(e, -96);
  }
  const float inv_q = __builtin_ldexpf(1.f, 31 - e), quantum = __builtin_ldexpf(1.f, e - 31);
  if (l == 0) sQuant[wv] = quantum;
  const float nDq = -Dq * inv_q;
  char* binsb = reinterpret_cast<char*>(sBins + kZ + wv * kBinW);   // + 4 rel
  bf16x8_t qs8[2] = {qb[0], qb[1]};
  if (F8) fp8_token_lane(qs8);
  const short* sKl = F8 ? sKq : sK;           // the logits' K
  const int qo4 = (sTok[q] >> 16) + c04;
  f32x16_t dq;
  zero16(dq);
  for (int kt = 0; kt < ((DBG & 4) ? 0 : NT); ++kt) {
    f32x16_t s, dp;
    zero16(s);
    zero16(dp);
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int t = 32 * kt + r, c = 2 * st + hh;
      s = mfma16(*reinterpret_cast<const bf16x8_t*>(sKl + swz64(t, c)), qs8[st], s);
      dp = mfma16(*reinterpret_cast<const bf16x8_t*>(sV + swz64(t, c)), db[st], dp);
    }
    int rel4[16];
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int4 t4 = *reinterpret_cast<const int4*>(sTok + 32 * kt + 8 * g4 + 4 * hh);
      const int tk[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        const int i = 4 * g4 + e4;
        rel4[i] = qo4 - (tk[e4] >> 16);
        s[i] = fmaf(s[i], scale2, *reinterpret_cast<const float*>(biasb + rel4[i]));
      }
    }
    if (mixed) mask_kq(s, sTok, kt, q, hh);
#pragma unroll
    for (int i = 0; i < 16; ++i) dp[i] = exp2_fast(s[i] - Lq) * fmaf(dp[i], inv_q, nDq);   // dS / quantum
#pragma unroll
    for (int th = 0; th < 2; ++th) dq = mfma16(tr_perm64(sK, 32 * kt + 16 * th, l), pack8(dp, 8 * th), dq);
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (!(DBG & 1))
        __hip_atomic_fetch_add(reinterpret_cast<int*>(binsb + rel4[i]), cvt_rpi(dp[i]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  if (q < N) {
    bf16* dst = gw + (size_t)q * C3;
    const float sc = quantum * g.scale;
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) {
      bf16x4_t v;
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) v[e4] = bf16_bits(dq[4 * grp + e4] * sc);
      *reinterpret_cast<bf16x4_t*>(dst + 8 * grp + 4 * hh) = v;
    }
  }
  load_p2();
  load_kv();
  __syncthreads();                            // bins complete; phase-1 staging dead after this
  {
    float* gp = gtable_part + ((size_t)bw * g.heads + h) * g.T2;
    for (int t = threadIdx.x; t < g.T2; t += blockDim.x) {
      const int ra = t / R, pb = kZ + ra * P + (t - ra * R);
      float a = 0.f;
#pragma unroll
      for (int w = 0; w < NT; ++w) a += (float)sBins[pb + w * kBinW] * sQuant[w];
      gp[t] = a;
    }
  }
  if (DBG & 2) return;
  // ---- phase 2 staging: Q, dO natural (swizzled)
  short* sQ = sU;
  short* sDo = sU + kImg;
  short* sQq = sU + 2 * kImg;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int p = threadIdx.x + it * 64 * NT, t = p >> 2, c = p & 3;
    *reinterpret_cast<bf16x8_t*>(sQ + swz64(t, c)) = cq[it];
    *reinterpret_cast<bf16x8_t*>(sDo + swz64(t, c)) = cd[it];
    if (F8) *reinterpret_cast<bf16x8_t*>(sQq + swz64(t, c)) = fp8_token_chunk(cq[it]);
  }
  bf16x8_t ks8[2] = {kb[0], kb[1]};
  if (F8) fp8_token_lane(ks8);
  const short* sQl = F8 ? sQq : sQ;
  const int tkey = sTok[key];
  const int ko4 = (tkey >> 16) - c04, rk = tkey & 0xffff;
  __syncthreads();
  f32x16_t dv, dk;
  zero16(dv);
  zero16(dk);
  for (int qq = 0; qq < NT; ++qq) {
    f32x16_t s, dp;
    zero16(s);
    zero16(dp);
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int t = 32 * qq + r, c = 2 * st + hh;
      s = mfma16(*reinterpret_cast<const bf16x8_t*>(sQl + swz64(t, c)), ks8[st], s);
      dp = mfma16(*reinterpret_cast<const bf16x8_t*>(sDo + swz64(t, c)), vb[st], dp);
    }
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int4 t4 = *reinterpret_cast<const int4*>(sTok + 32 * qq + 8 * g4 + 4 * hh);
      const int tq[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4)
        s[4 * g4 + e4] = fmaf(s[4 * g4 + e4], scale2, *reinterpret_cast<const float*>(biasb + ((tq[e4] >> 16) - ko4)));
    }
    if (mixed) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int4 t4 = *reinterpret_cast<const int4*>(sTok + 32 * qq + 8 * g4 + 4 * hh);
        const int tq[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4)
          if ((tq[e4] & 0xffff) != rk) s[4 * g4 + e4] += kMaskLog2;
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qi = 32 * qq + crow(i, hh);
      const float p = exp2_fast(s[i] - sL[qi]);
      s[i] = p;
      dp[i] = p * (dp[i] - sD[qi]);
    }
#pragma unroll
    for (int th = 0; th < 2; ++th) {
      const int base = 32 * qq + 16 * th;
      dv = mfma16(tr_perm64(sDo, base, l), pack8(s, 8 * th), dv);
      dk = mfma16(tr_perm64(sQ, base, l), pack8(dp, 8 * th), dk);
    }
  }
  if (key < N) {
    bf16* dst = gw + (size_t)key * C3;
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) {
      bf16x4_t a, b;
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        a[e4] = bf16_bits(dk[4 * grp + e4] * g.scale);
        b[e4] = bf16_bits(dv[4 * grp + e4]);
      }
      *reinterpret_cast<bf16x4_t*>(dst + C + 8 * grp + 4 * hh) = a;
      *reinterpret_cast<bf16x4_t*>(dst + 2 * C + 8 * grp + 4 * hh) = b;
    }
  }
}

int check_geom(WinGeom& g, int Bw, int heads, int ws, int shift, int nWh, int nWw, float scale) {
  g.heads = heads; g.ws = ws; g.shift = shift; g.nWh = nWh; g.nWw = nWw; g.scale = scale;
  g.N = ws * ws;
  g.T2 = (2 * ws - 1) * (2 * ws - 1);
  g.H = nWh * ws; g.W = nWw * ws; g.nat = 0;
  g.m_ws = ws > 0 ? (65536u + (unsigned)ws - 1u) / (unsigned)ws : 0u;
  const unsigned long long nw = (unsigned long long)nWh * (unsigned long long)nWw;
  g.m_nw = nw > 1 ? (unsigned)(((1ull << 32) + nw - 1) / nw) : 0u;     // 1: see div_nw
  g.m_nWw = nWw > 1 ? (unsigned)(((1ull << 32) + (unsigned long long)nWw - 1) / (unsigned long long)nWw) : 0u;
  return Bw > 0 && heads > 0 && ws > 0 && ws <= 16 && shift >= 0 && shift < ws && nWh > 0 && nWw > 0 &&
         Bw % (nWh * nWw) == 0 && (unsigned long long)Bw * nw < (1ull << 32);
}

}  // namespace
}  // namespace vs

using namespace vs;

// VS_WIN_ATTN_SCALAR=1 selects the scalar-FMA kernels for bf16 too (A/B and debugging)
static bool use_mfma() {
  const char* e = getenv("VS_WIN_ATTN_SCALAR");
  return !(e && atoi(e) != 0);
}

// (window, head) workgroups as one XCD-grouped 1-D grid: a window's heads share L2 lines (round 4:
// C5 backward -6.6 %, forward -16 %, C2 backward -12 % against the 2-D grid, profiles/r4_winbench_xcd.txt)
static dim3 blk_grid(dim3 g2) { return dim3(g2.x * g2.y); }

#define VS_NT_SWITCH(nt, M)            \
  switch (nt) {                        \
    case 1: case 2: M(2); break;       \
    case 3: M(3); break;               \
    case 4: M(4); break;               \
    default: M(5); break;              \
  }

template <bool F8>
static void launch_fwd_blk(const WinGeom& g, dim3 grid, hipStream_t st, const void* qkv, const float* table,
                           void* out, float* lse) {
  grid = blk_grid(grid);
#define VS_FWD_BLK(NT_)                                                                                     \
  if (F8)                                                                                                   \
    hipLaunchKernelGGL((win_attn_fwd_mx<NT_, true>), grid, dim3(64 * NT_), 0, st, (const bf16*)qkv, table,   \
                       (bf16*)out, lse, g);                                                                 \
  else                                                                                                      \
    hipLaunchKernelGGL((win_attn_fwd_online<NT_>), grid, dim3(64 * NT_), 0, st, (const bf16*)qkv, table,     \
                       (bf16*)out, lse, g)
  VS_NT_SWITCH((g.N + 31) / 32, VS_FWD_BLK)
#undef VS_FWD_BLK
}

// The round-5 backward (win_attn_bwd_fb) runs the bf16 windows of 64 < N <= 160 (Swin-B/L ws 12,
// C3 / C5): -12 % at C5 (profiles/r5_win_bwd_ab.txt).  At N <= 64 (Swin-T ws 7, C2) and on the
// fp8 path (a third staged image costs a workgroup per CU) the round-4 kernel stays faster.
// VS_WIN_BWD_FB=0: the round-4 kernel everywhere; 2: the round-5 one everywhere (A/B)
static bool bwd_fb(bool f8, int N) {
  const char* e = getenv("VS_WIN_BWD_FB");
  const int v = e ? atoi(e) : 1;
  return v == 2 || (v == 1 && !f8 && N > 64);
}

template <bool F8>
static void launch_bwd_fa(const WinGeom& g, dim3 grid, hipStream_t st, const void* qkv, const float* table,
                          const void* out, const float* lse, const void* grad_out, void* grad_qkv, float* gpart) {
  grid = blk_grid(grid);
#define VS_BWD_FA(NT_)                                                                                      \
  hipLaunchKernelGGL((win_attn_bwd_fa<NT_, F8>), grid, dim3(64 * NT_), 0, st, (const bf16*)qkv, table,       \
                     (const bf16*)out, lse, (const bf16*)grad_out, (bf16*)grad_qkv, gpart, g)
  if (bwd_fb(F8, g.N)) {
#define VS_BWD_FB(NT_)                                                                                      \
  hipLaunchKernelGGL((win_attn_bwd_fb<NT_, F8>), grid, dim3(64 * NT_), 0, st, (const bf16*)qkv, table,       \
                     (const bf16*)out, lse, (const bf16*)grad_out, (bf16*)grad_qkv, gpart, g)
    VS_NT_SWITCH((g.N + 31) / 32, VS_BWD_FB)
#undef VS_BWD_FB
    return;
  }
  VS_NT_SWITCH((g.N + 31) / 32, VS_BWD_FA)
#undef VS_BWD_FA
}

extern "C" int vs_window_attn_forward(int dtype, const void* qkv, const float* table, void* out,
                                      float* lse, int Bw, int heads, int ws, int shift, int nWh,
                                      int nWw, float scale, void* stream) {
  WinGeom g;
  VS_CHECK(check_geom(g, Bw, heads, ws, shift, nWh, nWw, scale), "bad window geometry");
  VS_CHECK(qkv && table && out && lse, "null pointer");
  const int threads = ((g.N + 63) / 64) * 64;
  VS_CHECK(threads <= 256, "window too large (N > 256)");
  const size_t lds = sizeof(float) * (2 * g.N * kD + g.T2);
  dim3 grid(Bw, heads);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VS_BF16 && g.N <= 64 && use_mfma()) {
    const int items = Bw * heads;
    hipLaunchKernelGGL(win_attn_fwd_mfma, dim3((items + kFwdWaves - 1) / kFwdWaves), dim3(64 * kFwdWaves), 0, st,
                       (const bf16*)qkv, table, (bf16*)out, lse, g, items);
  } else if (dtype == VS_BF16 && g.N <= 160 && use_mfma()) {
    launch_fwd_blk<false>(g, grid, st, qkv, table, out, lse);
  } else if (dtype == VS_BF16) {
    hipLaunchKernelGGL(win_attn_fwd_kernel<bf16>, grid, dim3(threads), lds, st, (const bf16*)qkv, table,
                       (bf16*)out, lse, g);
  } else if (dtype == VS_F32) {
    hipLaunchKernelGGL(win_attn_fwd_kernel<float>, grid, dim3(threads), lds, st, (const float*)qkv, table,
                       (float*)out, lse, g);
  } else {
    VS_CHECK(false, "dtype must be VS_F32 or VS_BF16");
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_window_attn_backward(int dtype, const void* qkv, const float* table, const void* out,
                                       const float* lse, const void* grad_out, void* grad_qkv,
                                       float* grad_table_partial, int Bw, int heads, int ws, int shift,
                                       int nWh, int nWw, float scale, void* stream) {
  WinGeom g;
  VS_CHECK(check_geom(g, Bw, heads, ws, shift, nWh, nWw, scale), "bad window geometry");
  VS_CHECK(qkv && table && out && lse && grad_out && grad_qkv && grad_table_partial, "null pointer");
  const int threads = ((g.N + 63) / 64) * 64;
  VS_CHECK(threads <= 256, "window too large (N > 256)");
  const size_t lds = sizeof(float) * (4 * g.N * kD + 2 * g.N + 2 * g.T2);
  VS_CHECK(lds <= 160 * 1024, "window too large for LDS");
  dim3 grid(Bw, heads);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VS_BF16 && g.N <= 160 && use_mfma()) {
    launch_bwd_fa<false>(g, grid, st, qkv, table, out, lse, grad_out, grad_qkv, grad_table_partial);
  } else if (dtype == VS_BF16) {
    hipLaunchKernelGGL(win_attn_bwd_kernel<bf16>, grid, dim3(threads), lds, st, (const bf16*)qkv, table,
                       (const bf16*)out, lse, (const bf16*)grad_out, (bf16*)grad_qkv, grad_table_partial, g);
  } else if (dtype == VS_F32) {
    hipLaunchKernelGGL(win_attn_bwd_kernel<float>, grid, dim3(threads), lds, st, (const float*)qkv, table,
                       (const float*)out, lse, (const float*)grad_out, (float*)grad_qkv, grad_table_partial, g);
  } else {
    VS_CHECK(false, "dtype must be VS_F32 or VS_BF16");
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}

// fp8 (e4m3) window attention (config C5): bf16 storage, fp8 MFMA for the logits and
// P.V (see "fp8 window attention" above); N <= 160 (ws <= 12).
extern "C" int vs_window_attn_forward_fp8(const void* qkv, const float* table, void* out, float* lse, int Bw,
                                          int heads, int ws, int shift, int nWh, int nWw, float scale,
                                          void* stream) {
  WinGeom g;
  VS_CHECK(check_geom(g, Bw, heads, ws, shift, nWh, nWw, scale), "bad window geometry");
  VS_CHECK(qkv && table && out && lse, "null pointer");
  VS_CHECK(g.N <= 160, "fp8 window attention needs window^2 <= 160");
  launch_fwd_blk<true>(g, dim3(Bw, heads), (hipStream_t)stream, qkv, table, out, lse);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_window_attn_backward_fp8(const void* qkv, const float* table, const void* out, const float* lse,
                                           const void* grad_out, void* grad_qkv, float* grad_table_partial, int Bw,
                                           int heads, int ws, int shift, int nWh, int nWw, float scale,
                                           void* stream) {
  WinGeom g;
  VS_CHECK(check_geom(g, Bw, heads, ws, shift, nWh, nWw, scale), "bad window geometry");
  VS_CHECK(qkv && table && out && lse && grad_out && grad_qkv && grad_table_partial, "null pointer");
  VS_CHECK(g.N <= 160, "fp8 window attention needs window^2 <= 160");
  launch_bwd_fa<true>(g, dim3(Bw, heads), (hipStream_t)stream, qkv, table, out, lse, grad_out, grad_qkv,
                      grad_table_partial);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

// Image-layout variants (the window reverse folded into the attention kernels): out /
// grad_out are [B, height, width, heads*32] in the un-shifted, un-padded image layout
// (what vs_window_reverse would make of the window-layout output), qkv / grad_qkv / lse /
// the table partials keep the window layout.  bf16 MFMA / fp8 MX kernels only.
static int image_geom(WinGeom& g, int dtype, int Bw, int heads, int ws, int shift, int nWh, int nWw, int height,
                      int width, float scale) {
  if (!check_geom(g, Bw, heads, ws, shift, nWh, nWw, scale)) return 0;
  g.H = height;
  g.W = width;
  g.nat = 1;
  return dtype == VS_BF16 && use_mfma() && g.N <= 160 && height > (nWh - 1) * ws && height <= nWh * ws &&
         width > (nWw - 1) * ws && width <= nWw * ws;
}

extern "C" int vs_window_attn_forward_image(int dtype, int fp8, const void* qkv, const float* table, void* out,
                                            float* lse, int Bw, int heads, int ws, int shift, int nWh, int nWw,
                                            int height, int width, float scale, void* stream) {
  WinGeom g;
  VS_CHECK(image_geom(g, dtype, Bw, heads, ws, shift, nWh, nWw, height, width, scale),
           "bad window / image geometry (image layout: bf16, window^2 <= 160, nwin x window covering the image)");
  VS_CHECK(qkv && table && out && lse, "null pointer");
  hipStream_t st = (hipStream_t)stream;
  if (fp8) {
    launch_fwd_blk<true>(g, dim3(Bw, heads), st, qkv, table, out, lse);
  } else if (g.N <= 64) {
    const int items = Bw * heads;
    hipLaunchKernelGGL(win_attn_fwd_mfma, dim3((items + kFwdWaves - 1) / kFwdWaves), dim3(64 * kFwdWaves), 0, st,
                       (const bf16*)qkv, table, (bf16*)out, lse, g, items);
  } else {
    launch_fwd_blk<false>(g, dim3(Bw, heads), st, qkv, table, out, lse);
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_window_attn_backward_image(int dtype, int fp8, const void* qkv, const float* table,
                                             const void* out, const float* lse, const void* grad_out, void* grad_qkv,
                                             float* grad_table_partial, int Bw, int heads, int ws, int shift,
                                             int nWh, int nWw, int height, int width, float scale, void* stream) {
  WinGeom g;
  VS_CHECK(image_geom(g, dtype, Bw, heads, ws, shift, nWh, nWw, height, width, scale),
           "bad window / image geometry (image layout: bf16, window^2 <= 160, nwin x window covering the image)");
  VS_CHECK(qkv && table && out && lse && grad_out && grad_qkv && grad_table_partial, "null pointer");
  if (fp8)
    launch_bwd_fa<true>(g, dim3(Bw, heads), (hipStream_t)stream, qkv, table, out, lse, grad_out, grad_qkv,
                        grad_table_partial);
  else
    launch_bwd_fa<false>(g, dim3(Bw, heads), (hipStream_t)stream, qkv, table, out, lse, grad_out, grad_qkv,
                         grad_table_partial);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
