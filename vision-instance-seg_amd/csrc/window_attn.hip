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
#include "mfma_util.h"

namespace vs {
namespace {

constexpr int kD = 32;

struct WinGeom {
  int heads, ws, shift, nWh, nWw, N, T2;  // T2 = (2ws-1)^2
  float scale;
};

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
// registers.  Backward: dP^T = V dO^T (same layout), dV = P^T dO and dK = dS^T Q through
// one LDS copy of P^T / dS^T, dQ^T = K^T dS^T again straight from registers; the bias
// gradient is binned per window in LDS (as the scalar path).
// Relative-position bias gradient of one (window, head) from its dS^T tile in LDS
// ([key][query] bf16, row pitch `pitch`): bin t = (dy, dx) gets the sum of dS over the
// pairs with ty_q - ty_k = dy, tx_q - tx_k = dx (HF:swin:350-365 index), each bin
// summed by one thread in a fixed order (deterministic).  Threads `tid` of `nthreads`.
__device__ __forceinline__ void bias_grad_bins(const short* dst, int pitch, const WinGeom& g, int tid, int nthreads,
                                               float* out) {
  const int ws = g.ws, tw = 2 * ws - 1;
  for (int t = tid; t < g.T2; t += nthreads) {
    const int dy = t / tw - (ws - 1), dx = t % tw - (ws - 1);
    const int qy0 = dy > 0 ? dy : 0, qy1 = dy < 0 ? ws + dy : ws;
    const int qx0 = dx > 0 ? dx : 0, qx1 = dx < 0 ? ws + dx : ws;
    float acc = 0.f;
    for (int qy = qy0; qy < qy1; ++qy)
      for (int qx = qx0; qx < qx1; ++qx) {
        const int q = qy * ws + qx, k = (qy - dy) * ws + (qx - dx);
        acc += bf16_bits_to_f32((unsigned short)dst[k * pitch + q]);
      }
    out[t] = acc;
  }
}

constexpr int kMaxT2 = 225;       // (2*8-1)^2
constexpr int kPadK = 72;         // LDS row pitch (shorts) of the 64-token operands

// token metadata of the window: ty | tx << 8 | region << 16
__device__ __forceinline__ void window_tokens(const WinGeom& g, int bw, int lane, int* tok) {
  const int ws = g.ws;
  const int wl = bw % (g.nWh * g.nWw);
  const int wy = wl / g.nWw, wx = wl % g.nWw;
  const int Hp = g.nWh * ws, Wp = g.nWw * ws;
  const int t = lane;
  if (t < g.N) {
    const int ty = t / ws, tx = t % ws;
    const int reg = g.shift > 0 ? region_of(wy * ws + ty, Hp, ws, g.shift) * 3 + region_of(wx * ws + tx, Wp, ws, g.shift) : 0;
    tok[t] = ty | (tx << 8) | (reg << 16);
  } else {
    tok[t] = 0;
  }
}

// scaled logits + bias + shift mask for the S^T accumulators of one (kt, qt) tile
__device__ __forceinline__ void logits_tile(f32x16_t& s, const WinGeom& g, const int* tok, const float* bias, int kt,
                                            int qt, int r, int hh) {
  const int q = 32 * qt + r;
  const int tq = tok[q];
  const int tyq = tq & 255, txq = (tq >> 8) & 255, rq = tq >> 16;
  const int tw = 2 * g.ws - 1;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int k = 32 * kt + (i & 3) + 8 * (i >> 2) + 4 * hh;
    if (k < g.N) {
      const int tk = tok[k];
      const int rel = (tyq - (tk & 255) + g.ws - 1) * tw + (txq - ((tk >> 8) & 255) + g.ws - 1);
      float v = s[i] * g.scale + bias[rel];
      if ((tk >> 16) != rq) v += -100.f;
      s[i] = v;
    } else {
      s[i] = -INFINITY;
    }
  }
}

constexpr int kFwdWaves = 4;

__global__ void __launch_bounds__(64 * kFwdWaves) win_attn_fwd_mfma(const bf16* __restrict__ qkv,
                                                                    const float* __restrict__ table,
                                                                    bf16* __restrict__ out, float* __restrict__ lse,
                                                                    WinGeom g, int items) {
  __shared__ __attribute__((aligned(16))) short sVt[kFwdWaves][32 * kPadK];   // V^T [d][key]
  __shared__ float sBias[kFwdWaves][kMaxT2];
  __shared__ int sTok[kFwdWaves][64];
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int item = blockIdx.x * kFwdWaves + wave;
  if (item >= items) return;                  // wave-uniform; only wave-level syncs below
  const int h = item % g.heads, bw = item / g.heads;
  const int N = g.N, C = g.heads * kD, C3 = 3 * C;
  const bf16* win = qkv + (size_t)bw * N * C3;
  short* vt = sVt[wave];
  float* bias = sBias[wave];
  int* tok = sTok[wave];
  window_tokens(g, bw, l, tok);
  for (int t = l; t < g.T2; t += 64) bias[t] = table[t * g.heads + h];
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
    logits_tile(acc[0][qt], g, tok, bias, 0, qt, r, hh);
    logits_tile(acc[1][qt], g, tok, bias, 1, qt, r, hh);
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) m = fmaxf(m, fmaxf(acc[0][qt][i], acc[1][qt][i]));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      acc[0][qt][i] = __expf(acc[0][qt][i] - m);
      acc[1][qt][i] = __expf(acc[1][qt][i] - m);
      sum += acc[0][qt][i] + acc[1][qt][i];
    }
    sum += __shfl_xor(sum, 32, 64);
    inv[qt] = 1.f / sum;
    lq[qt] = m + __logf(sum);
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
    if (q < N) {
      bf16* dst = out + ((size_t)bw * N + q) * C + h * kD;
#pragma unroll
      for (int grp = 0; grp < 4; ++grp) {
        bf16x4_t v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = bf16_bits(o[qt][4 * grp + e] * inv[qt]);
        *reinterpret_cast<bf16x4_t*>(dst + 8 * grp + 4 * hh) = v;
      }
      if (hh == 0) lse[((size_t)bw * g.heads + h) * N + q] = lq[qt];
    }
  }
}

constexpr int kBwdWaves = 2;

__global__ void __launch_bounds__(64 * kBwdWaves) win_attn_bwd_mfma(
    const bf16* __restrict__ qkv, const float* __restrict__ table, const bf16* __restrict__ out,
    const float* __restrict__ lse, const bf16* __restrict__ gout, bf16* __restrict__ gqkv,
    float* __restrict__ gtable_part, WinGeom g, int items) {
  __shared__ __attribute__((aligned(16))) short sT[kBwdWaves][64 * kPadK];    // P^T, then dS^T [key][q]
  __shared__ __attribute__((aligned(16))) short sDoT[kBwdWaves][32 * kPadK];  // dO^T [d][q]
  __shared__ __attribute__((aligned(16))) short sQT[kBwdWaves][32 * kPadK];   // Q^T [d][q]
  __shared__ __attribute__((aligned(16))) short sKT[kBwdWaves][32 * kPadK];   // K^T [d][key]
  __shared__ float sBias[kBwdWaves][kMaxT2];
  __shared__ int sTok[kBwdWaves][64];
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int item = blockIdx.x * kBwdWaves + wave;
  if (item >= items) return;
  const int h = item % g.heads, bw = item / g.heads;
  const int N = g.N, C = g.heads * kD, C3 = 3 * C;
  const bf16* win = qkv + (size_t)bw * N * C3;
  const bf16* gwin_o = gout + (size_t)bw * N * C + h * kD;
  short* pt = sT[wave];
  short* dot_ = sDoT[wave];
  short* qt_ = sQT[wave];
  short* kt_ = sKT[wave];
  float* bias = sBias[wave];
  int* tok = sTok[wave];
  window_tokens(g, bw, l, tok);
  for (int t = l; t < g.T2; t += 64) bias[t] = table[t * g.heads + h];
  {  // transposed copies, lane = token
    const int t = l;
    const bf16x8_t z = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bf16x8_t q = t < N ? ld8(win + (size_t)t * C3 + h * kD + 8 * c) : z;
      const bf16x8_t k = t < N ? ld8(win + (size_t)t * C3 + C + h * kD + 8 * c) : z;
      const bf16x8_t d = t < N ? ld8(gwin_o + (size_t)t * C + 8 * c) : z;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        qt_[(8 * c + j) * kPadK + t] = q[j];
        kt_[(8 * c + j) * kPadK + t] = k[j];
        dot_[(8 * c + j) * kPadK + t] = d[j];
      }
    }
  }
  // S^T = K Q^T and dP^T = V dO^T
  f32x16_t sacc[2][2], dacc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) sacc[a][b][i] = dacc[a][b][i] = 0.f;
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    bf16x8_t ka[2], va[2], qb[2], db[2];
    const bf16x8_t z = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int row = 32 * t + r;
      const int off = 16 * st + 8 * hh;
      ka[t] = row < N ? ld8(win + (size_t)row * C3 + C + h * kD + off) : z;
      va[t] = row < N ? ld8(win + (size_t)row * C3 + 2 * C + h * kD + off) : z;
      qb[t] = row < N ? ld8(win + (size_t)row * C3 + h * kD + off) : z;
      db[t] = row < N ? ld8(gwin_o + (size_t)row * C + off) : z;
    }
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        sacc[kt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka[kt], qb[qt], sacc[kt][qt], 0, 0, 0);
        dacc[kt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va[kt], db[qt], dacc[kt][qt], 0, 0, 0);
      }
  }
  // D_q = dO_q . O_q  and the saved log-sum-exp, per query column
  float Dq[2], Lq[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = 32 * qt + r;
    float d = 0.f;
    Lq[qt] = 0.f;
    if (q < N) {
      const bf16* orow = out + ((size_t)bw * N + q) * C + h * kD + 16 * hh;
      const bf16* grow = gwin_o + (size_t)q * C + 16 * hh;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const bf16x8_t ov = ld8(orow + 8 * c), gv = ld8(grow + 8 * c);
#pragma unroll
        for (int j = 0; j < 8; ++j) d += bf16_bits_to_f32((unsigned short)ov[j]) * bf16_bits_to_f32((unsigned short)gv[j]);
      }
      Lq[qt] = lse[((size_t)bw * g.heads + h) * N + q];
    }
    Dq[qt] = d + __shfl_xor(d, 32, 64);
  }
  wave_sync();
  // P^T = exp(logits - lse); P^T -> LDS [key][q] (bf16)
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      logits_tile(sacc[kt][qt], g, tok, bias, kt, qt, r, hh);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = (32 * qt + r) < N ? __expf(sacc[kt][qt][i] - Lq[qt]) : 0.f;
        sacc[kt][qt][i] = p;
        pt[(32 * kt + (i & 3) + 8 * (i >> 2) + 4 * hh) * kPadK + 32 * qt + r] = bf16_bits(p);
      }
    }
  wave_sync();
  // dV = P^T dO  (rows = keys, cols = d; k over queries)
  f32x16_t dv[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int i = 0; i < 16; ++i) dv[kt][i] = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(dot_ + r * kPadK + 16 * t + 8 * hh);
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(pt + (32 * kt + r) * kPadK + 16 * t + 8 * hh);
      dv[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, dv[kt], 0, 0, 0);
    }
  }
  bf16* gw = gqkv + (size_t)bw * N * C3 + h * kD;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = 32 * kt + (i & 3) + 8 * (i >> 2) + 4 * hh;
      if (key < N) gw[(size_t)key * C3 + 2 * C + r] = __float2bfloat16(dv[kt][i]);
    }
  // dS^T = P^T (dP^T - D_q)
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float ds = sacc[kt][qt][i] * (dacc[kt][qt][i] - Dq[qt]);
        dacc[kt][qt][i] = ds;
      }
  }
  wave_sync();                                // every lane has read P^T for dV
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i)
        pt[(32 * kt + (i & 3) + 8 * (i >> 2) + 4 * hh) * kPadK + 32 * qt + r] = bf16_bits(dacc[kt][qt][i]);
  wave_sync();
  // dK = scale * dS^T Q
  f32x16_t dk[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int i = 0; i < 16; ++i) dk[kt][i] = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(qt_ + r * kPadK + 16 * t + 8 * hh);
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(pt + (32 * kt + r) * kPadK + 16 * t + 8 * hh);
      dk[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, dk[kt], 0, 0, 0);
    }
  }
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = 32 * kt + (i & 3) + 8 * (i >> 2) + 4 * hh;
      if (key < N) gw[(size_t)key * C3 + C + r] = __float2bfloat16(dk[kt][i] * g.scale);
    }
  // dQ^T = scale * K^T dS^T  (dS^T straight from registers, K^T read in the permuted key order)
  f32x16_t dq[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int i = 0; i < 16; ++i) dq[qt][i] = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int kt = t >> 1, th = t & 1;
    const bf16x8_t a = ld_perm(kt_ + r * kPadK, 32 * kt + 16 * th + 4 * hh);
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
      dq[qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, pack8(dacc[kt][qt], 8 * th), dq[qt], 0, 0, 0);
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = 32 * qt + r;
    if (q < N) {
      bf16* dst = gw + (size_t)q * C3;
#pragma unroll
      for (int grp = 0; grp < 4; ++grp) {
        bf16x4_t v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = bf16_bits(dq[qt][4 * grp + e] * g.scale);
        *reinterpret_cast<bf16x4_t*>(dst + 8 * grp + 4 * hh) = v;
      }
    }
  }
  wave_sync();
  // bias gradient: bin (dy, dx) sums dS over the query/key pairs at that offset, read
  // back from the dS^T tile (no LDS float atomics: ~0.33 lane-ops/clk/CU on gfx950)
  bias_grad_bins(pt, kPadK, g, l, 64, gtable_part + ((size_t)bw * g.heads + h) * g.T2);
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

// ---- fp8 (OCP e4m3, gfx950) window attention, config C5 ------------------------------
// F8 = true selects v_mfma_f32_32x32x16_fp8_fp8 for S^T = K Q^T (forward and the
// backward's recompute) and for O^T = V^T P^T (forward).  Operands stay bf16 in HBM and
// LDS; each wave quantises its MFMA fragments on the fly with per-(window, head)
// power-of-two scales s = 2^floor(log2(448 / amax)) of q, k and v (amax over the window's
// N x 32 values; exact descale), and P (in [0, 1] before normalisation) with s = 256.
// The backward recomputes S with the same fp8 operands and scales (identical logits, so
// exp(S - lse) is the forward's P) and forms every gradient product in bf16 from the
// bf16 operands (straight-through quantisation).  Non-scaled fp8 MFMA issues at the bf16
// rate on gfx950 (MI355X_MICROARCH §Matrix cores): this is a numerics mode of the same
// latency/LDS-bound kernel, not a throughput change.
typedef long fp8x8_t;

__device__ __forceinline__ fp8x8_t fp8_pack8(const float* f) {
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
  return (fp8x8_t)(((unsigned long)(unsigned)hi << 32) | (unsigned)lo);
}

// bf16 fragment x s -> e4m3 fragment (element j in byte j)
__device__ __forceinline__ fp8x8_t fp8_frag(bf16x8_t v, float s) {
  float f[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = bf16_bits_to_f32((unsigned short)v[j]) * s;
  return fp8_pack8(f);
}

// 8 consecutive accumulator registers x s -> e4m3 fragment (permuted k, as pack8)
__device__ __forceinline__ fp8x8_t fp8_acc8(const f32x16_t& a, int base, float s) {
  float f[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = a[base + j] * s;
  return fp8_pack8(f);
}

__device__ __forceinline__ f32x16_t mfma_fp8(fp8x8_t a, fp8x8_t b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float amax8(bf16x8_t v, float m) {
#pragma unroll
  for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(bf16_bits_to_f32((unsigned short)v[j])));
  return m;
}

// e4m3 scale of a block: largest power of two with amax * s <= 448 (1 for an all-zero block)
__device__ __forceinline__ float fp8_scale(float amax) {
  return amax > 0.f ? exp2f(floorf(log2f(448.f / amax))) : 1.f;
}

constexpr float kP8Scale = 256.f;

// block-wide max of NV per-thread values through `red` [waves][NV] (one __syncthreads
// supplied by the caller between the write and the read)
template <int NV>
__device__ __forceinline__ void wave_amax_store(float* v, float* red) {
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float m = v[i];
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) m = fmaxf(m, __shfl_xor(m, s, 64));
    if ((threadIdx.x & 63) == 0) red[(threadIdx.x >> 6) * NV + i] = m;
  }
}

template <int NV>
__device__ __forceinline__ void block_amax_load(float* v, const float* red, int waves) {
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float m = 0.f;
    for (int w = 0; w < waves; ++w) m = fmaxf(m, red[w * NV + i]);
    v[i] = m;
  }
}

template <int NT>
__device__ __forceinline__ void window_tokens_blk(const WinGeom& g, int bw, int* tok) {
  const int ws = g.ws;
  const int wl = bw % (g.nWh * g.nWw);
  const int wy = wl / g.nWw, wx = wl % g.nWw;
  const int Hp = g.nWh * ws, Wp = g.nWw * ws;
  for (int t = threadIdx.x; t < 32 * NT; t += blockDim.x) {
    if (t < g.N) {
      const int ty = t / ws, tx = t % ws;
      const int reg = g.shift > 0 ? region_of(wy * ws + ty, Hp, ws, g.shift) * 3 + region_of(wx * ws + tx, Wp, ws, g.shift) : 0;
      tok[t] = ty | (tx << 8) | (reg << 16);
    } else {
      tok[t] = 0;
    }
  }
}

template <int NT, bool F8>
__global__ void __launch_bounds__(64 * NT) win_attn_fwd_mfma_big(const bf16* __restrict__ qkv,
                                                                 const float* __restrict__ table,
                                                                 bf16* __restrict__ out, float* __restrict__ lse,
                                                                 WinGeom g) {
  constexpr int NP = 32 * NT, PT = NP + 8, PK = 40;
  __shared__ __attribute__((aligned(16))) short sK[NP * PK];   // K [key][d]
  __shared__ __attribute__((aligned(16))) short sVt[32 * PT];  // V^T [d][key]
  __shared__ float sBias[kMaxT2Big];
  __shared__ int sTok[NP];
  __shared__ float sRed[F8 ? NT * 3 : 1];
  const int bw = blockIdx.x, h = blockIdx.y;
  const int qt = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int N = g.N, C = g.heads * kD, C3 = 3 * C;
  const bf16* win = qkv + (size_t)bw * N * C3;
  window_tokens_blk<NT>(g, bw, sTok);
  for (int t = threadIdx.x; t < g.T2; t += blockDim.x) sBias[t] = table[t * g.heads + h];
  float am[3] = {0.f, 0.f, 0.f};              // |q|, |k|, |v| maxima (F8)
  for (int p = threadIdx.x; p < NP * 4; p += blockDim.x) {
    const int t = p >> 2, c = p & 3;
    bf16x8_t k = zero8(), v = zero8();
    if (t < N) {
      k = ld8(win + (size_t)t * C3 + C + h * kD + 8 * c);
      v = ld8(win + (size_t)t * C3 + 2 * C + h * kD + 8 * c);
      if (F8) {
        am[0] = amax8(ld8(win + (size_t)t * C3 + h * kD + 8 * c), am[0]);
        am[1] = amax8(k, am[1]);
        am[2] = amax8(v, am[2]);
      }
    }
    *reinterpret_cast<bf16x8_t*>(sK + t * PK + 8 * c) = k;
#pragma unroll
    for (int j = 0; j < 8; ++j) sVt[(8 * c + j) * PT + t] = v[j];
  }
  if (F8) wave_amax_store<3>(am, sRed);
  bf16x8_t qb[2];
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    const int row = 32 * qt + r;
    qb[st] = row < N ? ld8(win + (size_t)row * C3 + h * kD + 16 * st + 8 * hh) : zero8();
  }
  __syncthreads();
  float sq = 1.f, sk = 1.f, sv = 1.f;
  WinGeom gl = g;
  if (F8) {
    block_amax_load<3>(am, sRed, NT);
    sq = fp8_scale(am[0]);
    sk = fp8_scale(am[1]);
    sv = fp8_scale(am[2]);
    gl.scale = g.scale / (sq * sk);           // exact: powers of two
  }
  // S^T = K Q^T for every key tile of this wave's queries
  f32x16_t acc[NT];
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) zero16(acc[kt]);
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
      const bf16x8_t ka = *reinterpret_cast<const bf16x8_t*>(sK + (32 * kt + r) * PK + 16 * st + 8 * hh);
      if (F8)
        acc[kt] = mfma_fp8(fp8_frag(ka, sk), fp8_frag(qb[st], sq), acc[kt]);
      else
        acc[kt] = mfma16(ka, qb[st], acc[kt]);
    }
  float m = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    logits_tile(acc[kt], gl, sTok, sBias, kt, qt, r, hh);
#pragma unroll
    for (int i = 0; i < 16; ++i) m = fmaxf(m, acc[kt][i]);
  }
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int kt = 0; kt < NT; ++kt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      acc[kt][i] = __expf(acc[kt][i] - m);
      sum += acc[kt][i];
    }
  sum += __shfl_xor(sum, 32, 64);
  const float lq = m + __logf(sum);
  const float inv = F8 ? 1.f / (sum * kP8Scale * sv) : 1.f / sum;
  // O^T = V^T P^T
  f32x16_t o;
  zero16(o);
#pragma unroll
  for (int t = 0; t < 2 * NT; ++t) {
    const int kt = t >> 1, th = t & 1;
    const bf16x8_t a = ld_perm(sVt + r * PT, 32 * kt + 16 * th + 4 * hh);
    if (F8)
      o = mfma_fp8(fp8_frag(a, sv), fp8_acc8(acc[kt], 8 * th, kP8Scale), o);
    else
      o = mfma16(a, pack8(acc[kt], 8 * th), o);
  }
  const int q = 32 * qt + r;
  if (q < N) {
    bf16* dst = out + ((size_t)bw * N + q) * C + h * kD;
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) {
      bf16x4_t v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = bf16_bits(o[4 * grp + e] * inv);
      *reinterpret_cast<bf16x4_t*>(dst + 8 * grp + 4 * hh) = v;
    }
    if (hh == 0) lse[((size_t)bw * g.heads + h) * N + q] = lq;
  }
}

template <int NT, bool F8>
__global__ void __launch_bounds__(64 * NT) win_attn_bwd_mfma_big(
    const bf16* __restrict__ qkv, const float* __restrict__ table, const bf16* __restrict__ out,
    const float* __restrict__ lse, const bf16* __restrict__ gout, bf16* __restrict__ gqkv,
    float* __restrict__ gtable_part, WinGeom g) {
  constexpr int NP = 32 * NT, PT = NP + 8, PK = 40;
  constexpr int kNat = NP * PK, kTB = NP * PT;
  constexpr int kU = 2 * kNat > kTB ? 2 * kNat : kTB;
  __shared__ __attribute__((aligned(16))) short sU[kU];        // K, V [token][d]; then P^T / dS^T [key][q]
  __shared__ __attribute__((aligned(16))) short sQT[32 * PT];  // Q^T [d][q]
  __shared__ __attribute__((aligned(16))) short sKT[32 * PT];  // K^T [d][key]
  __shared__ __attribute__((aligned(16))) short sDoT[32 * PT]; // dO^T [d][q]
  __shared__ float sBias[kMaxT2Big];
  __shared__ int sTok[NP];
  __shared__ float sRed[F8 ? NT * 2 : 1];
  short* sK = sU;
  short* sV = sU + kNat;
  short* sT = sU;
  const int bw = blockIdx.x, h = blockIdx.y;
  const int qt = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int N = g.N, C = g.heads * kD, C3 = 3 * C;
  const bf16* win = qkv + (size_t)bw * N * C3;
  const bf16* gwin_o = gout + (size_t)bw * N * C + h * kD;
  window_tokens_blk<NT>(g, bw, sTok);
  for (int t = threadIdx.x; t < g.T2; t += blockDim.x) sBias[t] = table[t * g.heads + h];
  float am[2] = {0.f, 0.f};                   // |q|, |k| maxima (F8)
  for (int p = threadIdx.x; p < NP * 4; p += blockDim.x) {
    const int t = p >> 2, c = p & 3;
    bf16x8_t q = zero8(), k = zero8(), v = zero8(), d = zero8();
    if (t < N) {
      q = ld8(win + (size_t)t * C3 + h * kD + 8 * c);
      k = ld8(win + (size_t)t * C3 + C + h * kD + 8 * c);
      v = ld8(win + (size_t)t * C3 + 2 * C + h * kD + 8 * c);
      d = ld8(gwin_o + (size_t)t * C + 8 * c);
      if (F8) {
        am[0] = amax8(q, am[0]);
        am[1] = amax8(k, am[1]);
      }
    }
    *reinterpret_cast<bf16x8_t*>(sK + t * PK + 8 * c) = k;
    *reinterpret_cast<bf16x8_t*>(sV + t * PK + 8 * c) = v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sQT[(8 * c + j) * PT + t] = q[j];
      sKT[(8 * c + j) * PT + t] = k[j];
      sDoT[(8 * c + j) * PT + t] = d[j];
    }
  }
  const int q = 32 * qt + r;
  bf16x8_t qb[2], db[2];
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    const int off = 16 * st + 8 * hh;
    qb[st] = q < N ? ld8(win + (size_t)q * C3 + h * kD + off) : zero8();
    db[st] = q < N ? ld8(gwin_o + (size_t)q * C + off) : zero8();
  }
  // D_q = dO_q . O_q and the saved log-sum-exp of this lane's query
  float Dq = 0.f, Lq = 0.f;
  if (q < N) {
    const bf16* orow = out + ((size_t)bw * N + q) * C + h * kD + 16 * hh;
    const bf16* grow = gwin_o + (size_t)q * C + 16 * hh;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const bf16x8_t ov = ld8(orow + 8 * c), gv = ld8(grow + 8 * c);
#pragma unroll
      for (int j = 0; j < 8; ++j) Dq += bf16_bits_to_f32((unsigned short)ov[j]) * bf16_bits_to_f32((unsigned short)gv[j]);
    }
    Lq = lse[((size_t)bw * g.heads + h) * N + q];
  }
  Dq += __shfl_xor(Dq, 32, 64);
  if (F8) wave_amax_store<2>(am, sRed);
  __syncthreads();
  float sq = 1.f, sk = 1.f;
  WinGeom gl = g;
  if (F8) {                                   // the forward's scales: identical logits
    block_amax_load<2>(am, sRed, NT);
    sq = fp8_scale(am[0]);
    sk = fp8_scale(am[1]);
    gl.scale = g.scale / (sq * sk);
  }
  // S^T = K Q^T and dP^T = V dO^T for every key tile of this wave's queries
  f32x16_t sacc[NT], dacc[NT];
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    zero16(sacc[kt]);
    zero16(dacc[kt]);
  }
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
      const int o = (32 * kt + r) * PK + 16 * st + 8 * hh;
      if (F8)
        sacc[kt] = mfma_fp8(fp8_frag(*reinterpret_cast<const bf16x8_t*>(sK + o), sk), fp8_frag(qb[st], sq), sacc[kt]);
      else
        sacc[kt] = mfma16(*reinterpret_cast<const bf16x8_t*>(sK + o), qb[st], sacc[kt]);
      dacc[kt] = mfma16(*reinterpret_cast<const bf16x8_t*>(sV + o), db[st], dacc[kt]);
    }
  __syncthreads();                            // K / V staging is overwritten by P^T below
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    logits_tile(sacc[kt], gl, sTok, sBias, kt, qt, r, hh);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = 32 * kt + crow(i, hh);
      const float p = q < N ? __expf(sacc[kt][i] - Lq) : 0.f;
      sT[key * PT + q] = bf16_bits(p);
      dacc[kt][i] = p * (dacc[kt][i] - Dq);
    }
  }
  __syncthreads();
  // dV = P^T dO for key tile kw = wave (k over all queries)
  const int kw = qt;
  bf16* gw = gqkv + (size_t)bw * N * C3 + h * kD;
  {
    f32x16_t dv;
    zero16(dv);
#pragma unroll
    for (int t = 0; t < 2 * NT; ++t) {
      const bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(sDoT + r * PT + 16 * t + 8 * hh);
      const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(sT + (32 * kw + r) * PT + 16 * t + 8 * hh);
      dv = mfma16(a, b, dv);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = 32 * kw + crow(i, hh);
      if (key < N) gw[(size_t)key * C3 + 2 * C + r] = __float2bfloat16(dv[i]);
    }
  }
  __syncthreads();                            // every wave has read P^T
#pragma unroll
  for (int kt = 0; kt < NT; ++kt)
#pragma unroll
    for (int i = 0; i < 16; ++i) sT[(32 * kt + crow(i, hh)) * PT + q] = bf16_bits(dacc[kt][i]);
  __syncthreads();
  // dK = scale * dS^T Q for key tile kw
  {
    f32x16_t dk;
    zero16(dk);
#pragma unroll
    for (int t = 0; t < 2 * NT; ++t) {
      const bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(sQT + r * PT + 16 * t + 8 * hh);
      const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(sT + (32 * kw + r) * PT + 16 * t + 8 * hh);
      dk = mfma16(a, b, dk);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = 32 * kw + crow(i, hh);
      if (key < N) gw[(size_t)key * C3 + C + r] = __float2bfloat16(dk[i] * g.scale);
    }
  }
  // dQ^T = scale * K^T dS^T for this wave's queries (dS^T from registers)
  {
    f32x16_t dq;
    zero16(dq);
#pragma unroll
    for (int t = 0; t < 2 * NT; ++t) {
      const int kt = t >> 1, th = t & 1;
      const bf16x8_t a = ld_perm(sKT + r * PT, 32 * kt + 16 * th + 4 * hh);
      dq = mfma16(a, pack8(dacc[kt], 8 * th), dq);
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
  }
  __syncthreads();                            // (sT still holds dS^T)
  bias_grad_bins(sT, PT, g, threadIdx.x, blockDim.x, gtable_part + ((size_t)bw * g.heads + h) * g.T2);
}

int check_geom(WinGeom& g, int Bw, int heads, int ws, int shift, int nWh, int nWw, float scale) {
  g.heads = heads; g.ws = ws; g.shift = shift; g.nWh = nWh; g.nWw = nWw; g.scale = scale;
  g.N = ws * ws;
  g.T2 = (2 * ws - 1) * (2 * ws - 1);
  return Bw > 0 && heads > 0 && ws > 0 && ws <= 16 && shift >= 0 && shift < ws && nWh > 0 && nWw > 0 &&
         Bw % (nWh * nWw) == 0;
}

}  // namespace
}  // namespace vs

using namespace vs;

// VS_WIN_ATTN_SCALAR=1 selects the scalar-FMA kernels for bf16 too (A/B and debugging)
static bool use_mfma() {
  const char* e = getenv("VS_WIN_ATTN_SCALAR");
  return !(e && atoi(e) != 0);
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
    const int nt = (g.N + 31) / 32;
    if (nt == 3)
      hipLaunchKernelGGL((win_attn_fwd_mfma_big<3, false>), grid, dim3(192), 0, st, (const bf16*)qkv, table, (bf16*)out, lse, g);
    else if (nt == 4)
      hipLaunchKernelGGL((win_attn_fwd_mfma_big<4, false>), grid, dim3(256), 0, st, (const bf16*)qkv, table, (bf16*)out, lse, g);
    else
      hipLaunchKernelGGL((win_attn_fwd_mfma_big<5, false>), grid, dim3(320), 0, st, (const bf16*)qkv, table, (bf16*)out, lse, g);
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
  if (dtype == VS_BF16 && g.N <= 64 && use_mfma()) {
    const int items = Bw * heads;
    hipLaunchKernelGGL(win_attn_bwd_mfma, dim3((items + kBwdWaves - 1) / kBwdWaves), dim3(64 * kBwdWaves), 0, st,
                       (const bf16*)qkv, table, (const bf16*)out, lse, (const bf16*)grad_out, (bf16*)grad_qkv,
                       grad_table_partial, g, items);
  } else if (dtype == VS_BF16 && g.N <= 160 && use_mfma()) {
    const int nt = (g.N + 31) / 32;
#define VS_WIN_BWD_BIG(NT_)                                                                                       \
  hipLaunchKernelGGL((win_attn_bwd_mfma_big<NT_, false>), grid, dim3(64 * NT_), 0, st, (const bf16*)qkv, table,            \
                     (const bf16*)out, lse, (const bf16*)grad_out, (bf16*)grad_qkv, grad_table_partial, g)
    if (nt == 3)
      VS_WIN_BWD_BIG(3);
    else if (nt == 4)
      VS_WIN_BWD_BIG(4);
    else
      VS_WIN_BWD_BIG(5);
#undef VS_WIN_BWD_BIG
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
  dim3 grid(Bw, heads);
  hipStream_t st = (hipStream_t)stream;
  const int nt = (g.N + 31) / 32;
#define VS_WIN_FWD_F8(NT_)                                                                                        \
  hipLaunchKernelGGL((win_attn_fwd_mfma_big<NT_, true>), grid, dim3(64 * NT_), 0, st, (const bf16*)qkv, table,    \
                     (bf16*)out, lse, g)
  switch (nt) {
    case 1: case 2: VS_WIN_FWD_F8(2); break;
    case 3: VS_WIN_FWD_F8(3); break;
    case 4: VS_WIN_FWD_F8(4); break;
    default: VS_WIN_FWD_F8(5); break;
  }
#undef VS_WIN_FWD_F8
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
  dim3 grid(Bw, heads);
  hipStream_t st = (hipStream_t)stream;
  const int nt = (g.N + 31) / 32;
#define VS_WIN_BWD_F8(NT_)                                                                                        \
  hipLaunchKernelGGL((win_attn_bwd_mfma_big<NT_, true>), grid, dim3(64 * NT_), 0, st, (const bf16*)qkv, table,    \
                     (const bf16*)out, lse, (const bf16*)grad_out, (bf16*)grad_qkv, grad_table_partial, g)
  switch (nt) {
    case 1: case 2: VS_WIN_BWD_F8(2); break;
    case 3: VS_WIN_BWD_F8(3); break;
    case 4: VS_WIN_BWD_F8(4); break;
    default: VS_WIN_BWD_F8(5); break;
  }
#undef VS_WIN_BWD_F8
  VS_LAUNCH_CHECK();
  return VS_OK;
}
