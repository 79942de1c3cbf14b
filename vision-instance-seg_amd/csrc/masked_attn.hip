// Masked cross-attention core of the Mask2Former decoder (HF:m2f:1644-1650: an
// nn.MultiheadAttention with a boolean attn_mask, True = blocked; rows blocked at
// every key are un-blocked before use, HF:m2f:1912-1914 — the bitmask producer
// (vs_attn_bitmask) already wrote such rows as all-zero).
//
//   O_i = softmax_{j unblocked}( (q_i . k_j) * scale ) V      per (batch, head)
//
// Layout: q [B, Q, heads*32], k/v [B, S, heads*32] (batch-first in_proj outputs),
// words u32 [B, Q, ceil(S/32)] (bit j%32 of word j/32 = key j blocked, shared by all
// heads), out [B, Q, heads*32], lse f32 [B, heads, Q].
//
// Forward = split-K ("flash-decoding"): the keys are cut into chunks so the grid has
// ~B*heads*32 workgroups even though Q is only 100; each workgroup stages its K/V
// chunk in LDS (128 keys per stage, f32) and gives one lane per query (two-pass max
// then exp-sum/PV per chunk, blocked keys skipped); a combine kernel merges the chunk
// partials (m, l, o) into O and the log-sum-exp.  Backward: dQ per chunk (lane per
// query, P recomputed from the saved lse, partials summed over chunks by a combine
// kernel — deterministic) and dK/dV with one lane per key over all queries staged in
// LDS.  Those are the f32 (parity) kernels; bf16 runs the MFMA kernels further below.
#include "lds_dma.h"
#include "mfma_util.h"

#include <algorithm>

namespace vs {
namespace {

constexpr int kD = 32;
constexpr int kStage = 128;   // keys per LDS stage
constexpr int kQTile = 128;   // queries per workgroup (lanes)

__device__ __forceinline__ float dot32_lds(const float* a, const float* b_lds) {
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
__device__ __forceinline__ void load_head_row(const T* src, float* dst) {
  constexpr int V = Vec16<T>::N;
#pragma unroll
  for (int c = 0; c < kD; c += V) Vec16<T>::load(src + c, dst + c);
}

template <typename T>
__device__ __forceinline__ void stage_kv(const T* base, int C, int h, int j0, int n, float* dst) {
  constexpr int V = Vec16<T>::N;
  constexpr int CH = kD / V;
  for (int idx = threadIdx.x; idx < kStage * CH; idx += blockDim.x) {
    const int t = idx / CH, c = (idx % CH) * V;
    float tmp[V];
    if (t < n) {
      Vec16<T>::load(base + (size_t)(j0 + t) * C + h * kD + c, tmp);
    } else {
#pragma unroll
      for (int e = 0; e < V; ++e) tmp[e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < V; ++e) dst[t * kD + c + e] = tmp[e];
  }
}

struct XGeom {
  int B, Q, S, heads, nw, chunk, nchunk;
  float scale;
};

// partial layout: po [B, heads, nchunk, Q, 32], pml [B, heads, nchunk, Q, 2]
template <typename T>
__global__ void __launch_bounds__(kQTile) xattn_fwd_partial(const T* __restrict__ q, const T* __restrict__ k,
                                                            const T* __restrict__ v, const uint32_t* __restrict__ words,
                                                            float* __restrict__ po, float* __restrict__ pml, XGeom g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sk = smem;
  float* sv = sk + kStage * kD;
  const int chunk = blockIdx.x, h = blockIdx.y;
  const int qg = blockIdx.z % ((g.Q + kQTile - 1) / kQTile);
  const int b = blockIdx.z / ((g.Q + kQTile - 1) / kQTile);
  const int C = g.heads * kD;
  const int i = qg * kQTile + threadIdx.x;
  const bool active = i < g.Q;
  float qi[kD];
  if (active) {
    load_head_row(q + ((size_t)b * g.Q + i) * C + h * kD, qi);
#pragma unroll
    for (int c = 0; c < kD; ++c) qi[c] *= g.scale;
  }
  const uint32_t* wrow = words + ((size_t)b * g.Q + (active ? i : 0)) * g.nw;
  const int jbeg = chunk * g.chunk;
  const int jend = min(g.S, jbeg + g.chunk);
  const T* kb = k + (size_t)b * g.S * C;
  const T* vb = v + (size_t)b * g.S * C;
  float m = -INFINITY, l = 0.f;
  float o[kD];
#pragma unroll
  for (int c = 0; c < kD; ++c) o[c] = 0.f;
  for (int j0 = jbeg; j0 < jend; j0 += kStage) {
    const int n = min(kStage, jend - j0);
    __syncthreads();
    stage_kv(kb, C, h, j0, n, sk);
    stage_kv(vb, C, h, j0, n, sv);
    __syncthreads();
    if (!active) continue;
    // pass 1: stage max (the running max only grows; rescale once per stage)
    float ms = -INFINITY;
    for (int t = 0; t < n; ++t) {
      const int j = j0 + t;
      if ((wrow[j >> 5] >> (j & 31)) & 1u) continue;
      ms = fmaxf(ms, dot32_lds(qi, sk + t * kD));
    }
    if (ms == -INFINITY) continue;
    const float mn = fmaxf(m, ms);
    const float alpha = __expf(m - mn);  // m = -inf -> 0
    l *= alpha;
#pragma unroll
    for (int c = 0; c < kD; ++c) o[c] *= alpha;
    m = mn;
    for (int t = 0; t < n; ++t) {
      const int j = j0 + t;
      if ((wrow[j >> 5] >> (j & 31)) & 1u) continue;
      const float p = __expf(dot32_lds(qi, sk + t * kD) - m);
      l += p;
      const float4* v4 = reinterpret_cast<const float4*>(sv + t * kD);
#pragma unroll
      for (int c = 0; c < kD / 4; ++c) {
        const float4 vv = v4[c];
        o[4 * c + 0] = fmaf(p, vv.x, o[4 * c + 0]);
        o[4 * c + 1] = fmaf(p, vv.y, o[4 * c + 1]);
        o[4 * c + 2] = fmaf(p, vv.z, o[4 * c + 2]);
        o[4 * c + 3] = fmaf(p, vv.w, o[4 * c + 3]);
      }
    }
  }
  if (!active) return;
  const size_t prow = (((size_t)b * g.heads + h) * g.nchunk + chunk) * g.Q + i;
  float4* dst = reinterpret_cast<float4*>(po + prow * kD);
#pragma unroll
  for (int c = 0; c < kD / 4; ++c) dst[c] = make_float4(o[4 * c], o[4 * c + 1], o[4 * c + 2], o[4 * c + 3]);
  pml[prow * 2 + 0] = m;
  pml[prow * 2 + 1] = l;
}

// merge chunk partials: 32 lanes per (b, h, q) = 8 channel quads x 4 chunk phases (lane
// phase s takes chunks s, s + 4, ...), reduced across the phases by shuffles -- 4x the
// lanes of one-lane-per-quad, whose serial walk over 64 chunks (C2's 128^2 level) left
// the launch latency-bound on 100 workgroups
template <typename T>
__global__ void __launch_bounds__(256) xattn_fwd_combine(const float* __restrict__ po, const float* __restrict__ pml,
                                                         T* __restrict__ out, float* __restrict__ lse, XGeom g) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long rows = (long long)g.B * g.heads * g.Q;
  const int quad = (int)(gid & 7), ph = (int)((gid >> 3) & 3);
  const long long row = gid >> 5;  // (b, h, q); the grid is whole waves, rows beyond are idle
  const bool live = row < rows;
  const long long rr = live ? row : 0;
  const int i = (int)(rr % g.Q);
  const long long bh = rr / g.Q;
  const int h = (int)(bh % g.heads);
  const long long b = bh / g.heads;
  float M = -INFINITY;
#pragma unroll 4
  for (int c = ph; c < g.nchunk; c += 4) M = fmaxf(M, pml[((bh * g.nchunk + c) * g.Q + i) * 2]);
  M = fmaxf(M, __shfl_xor(M, 8, 64));
  M = fmaxf(M, __shfl_xor(M, 16, 64));
  float lsum = 0.f, acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int c = ph; c < g.nchunk; c += 4) {
    const size_t pr = (bh * g.nchunk + c) * g.Q + i;
    const float2 ml = *reinterpret_cast<const float2*>(pml + pr * 2);
    const float4 v = reinterpret_cast<const float4*>(po + pr * kD)[quad];
    if (ml.x == -INFINITY) continue;         // a chunk whose keys are all blocked
    const float w = __expf(ml.x - M);
    lsum += w * ml.y;
    acc[0] += w * v.x; acc[1] += w * v.y; acc[2] += w * v.z; acc[3] += w * v.w;
  }
#pragma unroll
  for (int sh = 8; sh <= 16; sh <<= 1) {
    lsum += __shfl_xor(lsum, sh, 64);
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2) acc[e2] += __shfl_xor(acc[e2], sh, 64);
  }
  if (!live || ph != 0) return;
  const float inv = 1.f / lsum;
  T* dst = out + ((size_t)b * g.Q + i) * (g.heads * kD) + h * kD + quad * 4;
#pragma unroll
  for (int e2 = 0; e2 < 4; ++e2) dst[e2] = from_f32<T>(acc[e2] * inv);
  if (quad == 0) lse[row] = M + __logf(lsum);
}

// dQ partials per key chunk (lane = query) + D_i = dO_i . O_i (written by chunk 0)
template <typename T>
__global__ void __launch_bounds__(kQTile) xattn_bwd_dq_partial(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, const uint32_t* __restrict__ words,
    const T* __restrict__ out, const float* __restrict__ lse, const T* __restrict__ gout, float* __restrict__ pdq,
    float* __restrict__ Dbuf, XGeom g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sk = smem;
  float* sv = sk + kStage * kD;
  const int chunk = blockIdx.x, h = blockIdx.y;
  const int nqg = (g.Q + kQTile - 1) / kQTile;
  const int qg = blockIdx.z % nqg, b = blockIdx.z / nqg;
  const int C = g.heads * kD;
  const int i = qg * kQTile + threadIdx.x;
  const bool active = i < g.Q;
  float qi[kD], di[kD], dq[kD];
  float Li = 0.f, Di = 0.f;
  if (active) {
    float oi[kD];
    load_head_row(q + ((size_t)b * g.Q + i) * C + h * kD, qi);
    load_head_row(gout + ((size_t)b * g.Q + i) * C + h * kD, di);
    load_head_row(out + ((size_t)b * g.Q + i) * C + h * kD, oi);
#pragma unroll
    for (int c = 0; c < kD; ++c) { Di = fmaf(di[c], oi[c], Di); qi[c] *= g.scale; dq[c] = 0.f; }
    Li = lse[((size_t)b * g.heads + h) * g.Q + i];
    if (chunk == 0) Dbuf[((size_t)b * g.heads + h) * g.Q + i] = Di;
  }
  const uint32_t* wrow = words + ((size_t)b * g.Q + (active ? i : 0)) * g.nw;
  const int jbeg = chunk * g.chunk, jend = min(g.S, jbeg + g.chunk);
  const T* kb = k + (size_t)b * g.S * C;
  const T* vb = v + (size_t)b * g.S * C;
  for (int j0 = jbeg; j0 < jend; j0 += kStage) {
    const int n = min(kStage, jend - j0);
    __syncthreads();
    stage_kv(kb, C, h, j0, n, sk);
    stage_kv(vb, C, h, j0, n, sv);
    __syncthreads();
    if (!active) continue;
    for (int t = 0; t < n; ++t) {
      const int j = j0 + t;
      if ((wrow[j >> 5] >> (j & 31)) & 1u) continue;
      const float p = __expf(dot32_lds(qi, sk + t * kD) - Li);
      const float ds = p * (dot32_lds(di, sv + t * kD) - Di);
      const float4* k4 = reinterpret_cast<const float4*>(sk + t * kD);
#pragma unroll
      for (int c = 0; c < kD / 4; ++c) {
        const float4 kk = k4[c];
        dq[4 * c + 0] = fmaf(ds, kk.x, dq[4 * c + 0]);
        dq[4 * c + 1] = fmaf(ds, kk.y, dq[4 * c + 1]);
        dq[4 * c + 2] = fmaf(ds, kk.z, dq[4 * c + 2]);
        dq[4 * c + 3] = fmaf(ds, kk.w, dq[4 * c + 3]);
      }
    }
  }
  if (!active) return;
  const size_t prow = (((size_t)b * g.heads + h) * g.nchunk + chunk) * g.Q + i;
  float4* dst = reinterpret_cast<float4*>(pdq + prow * kD);
#pragma unroll
  for (int c = 0; c < kD / 4; ++c)
    dst[c] = make_float4(dq[4 * c] * g.scale, dq[4 * c + 1] * g.scale, dq[4 * c + 2] * g.scale, dq[4 * c + 3] * g.scale);
}

template <typename T>
__global__ void __launch_bounds__(256) xattn_bwd_dq_combine(const float* __restrict__ pdq, T* __restrict__ gq, XGeom g) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)g.B * g.heads * g.Q * kD;
  if (gid >= total) return;
  const int c = (int)(gid % kD);
  const long long row = gid / kD;  // (b, h, q)
  const int i = (int)(row % g.Q);
  const long long bh = row / g.Q;
  const int h = (int)(bh % g.heads);
  const long long b = bh / g.heads;
  float s = 0.f;
  for (int ch = 0; ch < g.nchunk; ++ch) s += pdq[((bh * g.nchunk + ch) * g.Q + i) * kD + c];
  gq[((size_t)b * g.Q + i) * (g.heads * kD) + h * kD + c] = from_f32<T>(s);
}

// dK, dV: lane = key; all queries of (b, h) staged in LDS
template <typename T>
__global__ void __launch_bounds__(256) xattn_bwd_dkdv(const T* __restrict__ q, const T* __restrict__ k,
                                                      const T* __restrict__ v, const uint32_t* __restrict__ words,
                                                      const float* __restrict__ lse, const float* __restrict__ Dbuf,
                                                      const T* __restrict__ gout, T* __restrict__ gk,
                                                      T* __restrict__ gv, XGeom g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Q = g.Q;
  float* sq = smem;               // [Q][32] (pre-scaled)
  float* sdo = sq + Q * kD;       // [Q][32]
  float* sl = sdo + Q * kD;       // [Q]
  float* sD = sl + Q;             // [Q]
  const int h = blockIdx.y, b = blockIdx.z;
  const int C = g.heads * kD;
  {
    constexpr int V = Vec16<T>::N;
    constexpr int CH = kD / V;
    for (int idx = threadIdx.x; idx < Q * CH; idx += blockDim.x) {
      const int t = idx / CH, c = (idx % CH) * V;
      float a[V], d[V];
      Vec16<T>::load(q + ((size_t)b * Q + t) * C + h * kD + c, a);
      Vec16<T>::load(gout + ((size_t)b * Q + t) * C + h * kD + c, d);
#pragma unroll
      for (int e = 0; e < V; ++e) { sq[t * kD + c + e] = a[e] * g.scale; sdo[t * kD + c + e] = d[e]; }
    }
    for (int t = threadIdx.x; t < Q; t += blockDim.x) {
      sl[t] = lse[((size_t)b * g.heads + h) * Q + t];
      sD[t] = Dbuf[((size_t)b * g.heads + h) * Q + t];
    }
  }
  __syncthreads();
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= g.S) return;
  float kj[kD], vj[kD], dk[kD], dv[kD];
  load_head_row(k + ((size_t)b * g.S + j) * C + h * kD, kj);
  load_head_row(v + ((size_t)b * g.S + j) * C + h * kD, vj);
#pragma unroll
  for (int c = 0; c < kD; ++c) { dk[c] = 0.f; dv[c] = 0.f; }
  const uint32_t* wcol = words + (size_t)b * Q * g.nw + (j >> 5);
  const uint32_t bit = 1u << (j & 31);
  for (int i = 0; i < Q; ++i) {
    if (wcol[(size_t)i * g.nw] & bit) continue;
    const float p = __expf(dot32_lds(kj, sq + i * kD) - sl[i]);
    const float ds = p * (dot32_lds(vj, sdo + i * kD) - sD[i]);
    const float4* q4 = reinterpret_cast<const float4*>(sq + i * kD);
    const float4* d4 = reinterpret_cast<const float4*>(sdo + i * kD);
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
  }
  // sq was pre-scaled, so dk already carries the 'scale' factor of dS/dK
  constexpr int V = Vec16<T>::N;
#pragma unroll
  for (int c = 0; c < kD; c += V) {
    Vec16<T>::store(gk + ((size_t)b * g.S + j) * C + h * kD + c, dk + c);
    Vec16<T>::store(gv + ((size_t)b * g.S + j) * C + h * kD + c, dv + c);
  }
}

// ---------------------------------------------------------------------------------------
// bf16 MFMA path (32x32x16 bf16 tiles, helpers in mfma_util.h, lds_dma.h).
//
// Forward (xattn_fwd_mfma2): workgroup = (256-key chunk, head, image x 128-query group), 4 waves
// = 4 query tiles of 32.  Per 32-key tile a wave computes S^T = K Q^T (keys on rows: a lane
// holds 16 keys of ONE query, the other 16 in lane^32), applies the blocked-key bits (one
// 32-bit word per lane per tile), runs the online softmax in registers and accumulates
// O^T += V^T P^T with P^T taken straight from the accumulators (permuted k).  Chunk partials
// (o, m, l) go to xattn_fwd_combine.
//
// Backward (xattn_bwd_mfma2): workgroup = (chunk of 1-8 128-key blocks, head, image), all
// queries (<= 128, padded) in the workgroup, wave w owns keys 32w..32w+31 of each block; the
// query tiles are walked one at a time (one tile's S / dP accumulators live: 2 waves/SIMD) and
// the dQ partial accumulates over the chunk's blocks in registers.  S = Q K^T and dP = dO V^T
// with QUERIES on rows, so dV^T = dO^T P and dK^T = scale Q^T dS take P / dS straight from
// registers; dS^T goes to LDS once so that wave w can form the chunk's dQ partial for query
// tile w, summed over chunks by xattn_bwd_dq_combine.  (The round-4 kernels of the same split,
// which re-read operand fragments from global memory inside their tile loops, are gone:
// backward 0.135 -> 0.085 ms, forward 0.068 -> 0.055 ms at the 128^2 level,
// profiles/r5_xattn_ab.txt.)
constexpr int kFChunk = 256;
constexpr int kBChunk = 128;
constexpr int kBQ = 128;

// Forward (xattn_fwd_mfma2): K and V staged
// once in their natural layout (64-B rows, lds_dma.h swz64: 16-B chunk stores, no
// transposing two-byte stores) -- the round-4 kernel read every 32-key tile's K fragment and
// blocked-bits word from global memory inside the tile loop, one L2 round trip per tile with
// nothing else in flight.  V^T in the permuted key order comes from the transposed LDS read;
// a lane's blocked bits for the chunk (8 words) are requested with the staging loads.
__global__ void __launch_bounds__(256) xattn_fwd_mfma2(const bf16* __restrict__ q, const bf16* __restrict__ k,
                                                       const bf16* __restrict__ v, const uint32_t* __restrict__ words,
                                                       float* __restrict__ po, float* __restrict__ pml, XGeom g) {
  __shared__ __attribute__((aligned(16))) short sK[kFChunk * 32];
  __shared__ __attribute__((aligned(16))) short sV[kFChunk * 32];
  const int chunk = blockIdx.x, h = blockIdx.y;
  const int nqg = (g.Q + 127) / 128;
  const int qg = blockIdx.z % nqg, b = blockIdx.z / nqg;
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int C = g.heads * kD;
  const int jbeg = chunk * kFChunk;
  const int n = min(kFChunk, g.S - jbeg);
  const bf16* kb = k + ((size_t)b * g.S + jbeg) * C + h * kD;
  const bf16* vb = v + ((size_t)b * g.S + jbeg) * C + h * kD;
  constexpr int kIt = kFChunk * 4 / 256;        // 16-B chunks per thread and tensor
  bf16x8_t kc[kIt], vc[kIt];
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int p = threadIdx.x + 256 * it, t = p >> 2, c = p & 3;
    kc[it] = t < n ? ld8(kb + (size_t)t * C + 8 * c) : zero8();
    vc[it] = t < n ? ld8(vb + (size_t)t * C + 8 * c) : zero8();
  }
  const int qi = qg * 128 + wave * 32 + r;
  const bool qok = qi < g.Q;
  bf16x8_t qf[2];
#pragma unroll
  for (int st = 0; st < 2; ++st) qf[st] = qok ? ld8(q + ((size_t)b * g.Q + qi) * C + h * kD + 16 * st + 8 * hh) : zero8();
  const int ntiles = (n + 31) / 32;
  const uint32_t* wrow = words + ((size_t)b * g.Q + (qok ? qi : 0)) * g.nw + (jbeg >> 5);
  uint32_t wv[kFChunk / 32];
#pragma unroll
  for (int kt = 0; kt < kFChunk / 32; ++kt) wv[kt] = (qok && kt < ntiles) ? wrow[kt] : 0xffffffffu;
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int p = threadIdx.x + 256 * it, t = p >> 2, c = p & 3;
    *reinterpret_cast<bf16x8_t*>(sK + swz64(t, c)) = kc[it];
    *reinterpret_cast<bf16x8_t*>(sV + swz64(t, c)) = vc[it];
  }
  __syncthreads();
  float m = -INFINITY, lsum = 0.f;
  f32x16_t o;
  zero16(o);
#pragma unroll
  for (int kt = 0; kt < kFChunk / 32; ++kt) {
    if (kt >= ntiles) break;
    f32x16_t sc;
    zero16(sc);
#pragma unroll
    for (int st = 0; st < 2; ++st)
      sc = mfma16(*reinterpret_cast<const bf16x8_t*>(sK + swz64(32 * kt + r, 2 * st + hh)), qf[st], sc);
    const uint32_t w = wv[kt];
    float mt = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int kl = crow(i, hh);
      const bool blocked = (kt * 32 + kl >= n) || ((w >> kl) & 1u);
      sc[i] = blocked ? -INFINITY : sc[i] * g.scale;
      mt = fmaxf(mt, sc[i]);
    }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float mn = fmaxf(m, mt);
    const float safe = mn == -INFINITY ? 0.f : mn;
    const float alpha = __expf(m - safe);
    lsum *= alpha;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      o[i] *= alpha;
      sc[i] = __expf(sc[i] - safe);
      lsum += sc[i];
    }
    m = mn;
#pragma unroll
    for (int th = 0; th < 2; ++th) o = mfma16(tr_perm64(sV, kt * 32 + 16 * th, l), pack8(sc, 8 * th), o);
  }
  lsum += __shfl_xor(lsum, 32, 64);
  if (qok) {
    const size_t prow = (((size_t)b * g.heads + h) * g.nchunk + chunk) * g.Q + qi;
    float* dst = po + prow * kD;
#pragma unroll
    for (int grp = 0; grp < 4; ++grp)
      *reinterpret_cast<float4*>(dst + 8 * grp + 4 * hh) =
          make_float4(o[4 * grp], o[4 * grp + 1], o[4 * grp + 2], o[4 * grp + 3]);
    if (hh == 0) {
      pml[prow * 2 + 0] = m;
      pml[prow * 2 + 1] = lsum;
    }
  }
}

// D_i = dO_i . O_i per (b, h, q)
template <typename T>
__global__ void __launch_bounds__(256) xattn_bwd_prep(const T* __restrict__ out, const T* __restrict__ gout,
                                                      float* __restrict__ Dbuf, XGeom g) {
  const long long row = (long long)blockIdx.x * blockDim.x + threadIdx.x;   // (b, h, q)
  if (row >= (long long)g.B * g.heads * g.Q) return;
  const int i = (int)(row % g.Q);
  const long long bh = row / g.Q;
  const int h = (int)(bh % g.heads);
  const long long b = bh / g.heads;
  float o[kD], d[kD];
  load_head_row(out + ((size_t)b * g.Q + i) * (g.heads * kD) + h * kD, o);
  load_head_row(gout + ((size_t)b * g.Q + i) * (g.heads * kD) + h * kD, d);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < kD; ++c) s = fmaf(o[c], d[c], s);
  Dbuf[row] = s;
}

// Backward (xattn_bwd_mfma2): the workgroup / wave split above with
// every operand read from LDS, staged once in its natural layout:
//  * Q and dO of the (image, head) -- the round-4 kernel re-read their fragments from global
//    memory inside the query-tile loop of every key block, a round trip to L2 per tile with
//    nothing else in flight (the finest level ran at ~14 % of HBM rate); Q^T / dO^T for
//    dK / dV now come from the transposed LDS read of the same natural copies;
//  * the blocked-key bits transposed to [key group][query], so a lane's 4 consecutive query
//    rows are one 16-B read (16 scalar reads before);
//  * dS stored transposed, [key][query] (256-B rows, lds_dma.h image b): a lane writes its 4
//    consecutive queries as one 8-B store (16 two-byte stores before), and dQ^T = K^T dS^T
//    takes both operands by transposed reads; a lane's dQ partial is then 16 channels of
//    ONE query (4 x 16-B stores).
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) xattn_bwd_mfma2(const bf16* __restrict__ q, const bf16* __restrict__ k,
                                                       const bf16* __restrict__ v, const uint32_t* __restrict__ words,
                                                       const float* __restrict__ lse, const float* __restrict__ Dbuf,
                                                       const bf16* __restrict__ gout, bf16* __restrict__ gk,
                                                       bf16* __restrict__ gv, float* __restrict__ pdq, XGeom g) {
  __shared__ __attribute__((aligned(16))) short sQ[kBQ * 32];         // Q [q][d], 64-B rows (swz64)
  __shared__ __attribute__((aligned(16))) short sDo[kBQ * 32];        // dO [q][d]
  __shared__ __attribute__((aligned(16))) short sK[kBChunk * 32];     // K [key][d] of the block
  __shared__ __attribute__((aligned(16))) unsigned char sDSt[kBChunk * kBQ * 2];   // dS^T [key][q]
  __shared__ __attribute__((aligned(16))) uint32_t sWt[kBChunk / 32][kBQ];       // blocked bits
  __shared__ __attribute__((aligned(16))) float sL[kBQ], sD[kBQ];
  const int chunk = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int C = g.heads * kD, Q = g.Q;
  const bf16* qb = q + (size_t)b * Q * C + h * kD;
  const bf16* ob = gout + (size_t)b * Q * C + h * kD;
  // Q, dO natural (4 chunks of 16 B a row): 1024 chunks over 256 threads; lse and D rows
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int p = threadIdx.x + 256 * it, part = p >> 9, t = (p >> 2) & 127, c = p & 3;
    const bf16* src = part ? ob : qb;
    const bf16x8_t x = t < Q ? ld8(src + (size_t)t * C + 8 * c) : zero8();
    *reinterpret_cast<bf16x8_t*>((part ? sDo : sQ) + swz64(t, c)) = x;
  }
  if (threadIdx.x < kBQ) {
    const int t = threadIdx.x;
    sL[t] = t < Q ? lse[((size_t)b * g.heads + h) * Q + t] : 0.f;
    sD[t] = t < Q ? Dbuf[((size_t)b * g.heads + h) * Q + t] : 0.f;
  }
  f32x16_t dq;                                 // dQ^T of query tile `wave`: rows d, column q
  zero16(dq);
  const int nblk = g.chunk / kBChunk;
  const int kl = wave * 32 + r;                 // key within a block (this lane's column)
  // a block's global operands: this lane's K / V row slices, the K staging chunks and the
  // blocked bits -- requested one block ahead, so their latency hides behind a block's work
  bf16x8_t kf[2], vf[2], kst[2];
  uint32_t wst[2];
  auto load_block = [&](int kb) {
    const int jbeg = chunk * g.chunk + kb * kBChunk;
    const int n = min(kBChunk, g.S - jbeg);     // <= 0 past the end: everything zero
    const bf16* kb_ = k + ((size_t)b * g.S + jbeg) * C + h * kD;
    const bf16* vb = v + ((size_t)b * g.S + jbeg) * C + h * kD;
    const bool kok = kl < n;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      kf[st] = kok ? ld8(kb_ + (size_t)kl * C + 16 * st + 8 * hh) : zero8();
      vf[st] = kok ? ld8(vb + (size_t)kl * C + 16 * st + 8 * hh) : zero8();
    }
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int p = threadIdx.x + 256 * it, t = p >> 2, c = p & 3;
      kst[it] = t < n ? ld8(kb_ + (size_t)t * C + 8 * c) : zero8();
      const int qq = p & 127, wg = p >> 7, wi = (jbeg >> 5) + wg;
      wst[it] = (n > 0 && qq < Q && wi < g.nw) ? words[((size_t)b * Q + qq) * g.nw + wi] : 0xffffffffu;
    }
  };
  load_block(0);
  for (int kb = 0; kb < nblk; ++kb) {
    const int jbeg = chunk * g.chunk + kb * kBChunk;
    if (jbeg >= g.S) break;                     // uniform over the workgroup
    const int n = min(kBChunk, g.S - jbeg);
    const bool kok = kl < n;
    const bf16x8_t kfc[2] = {kf[0], kf[1]}, vfc[2] = {vf[0], vf[1]};
    __syncthreads();                            // the previous block's K / dS^T / bits are read
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int p = threadIdx.x + 256 * it, t = p >> 2, c = p & 3;
      *reinterpret_cast<bf16x8_t*>(sK + swz64(t, c)) = kst[it];
      sWt[p >> 7][p & 127] = wst[it];
    }
    if (kb + 1 < nblk) load_block(kb + 1);
    __syncthreads();
    f32x16_t dv, dk;
    zero16(dv);
    zero16(dk);
#pragma unroll 1
    for (int qt = 0; qt < 4; ++qt) {
      f32x16_t sacc, dacc;
      zero16(sacc);
      zero16(dacc);
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const int t = 32 * qt + r, c = 2 * st + hh;
        sacc = mfma16(*reinterpret_cast<const bf16x8_t*>(sQ + swz64(t, c)), kfc[st], sacc);
        dacc = mfma16(*reinterpret_cast<const bf16x8_t*>(sDo + swz64(t, c)), vfc[st], dacc);
      }
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int q0 = 32 * qt + 8 * g4 + 4 * hh;
        const uint4 w4 = *reinterpret_cast<const uint4*>(&sWt[wave][q0]);
        const float4 L4 = *reinterpret_cast<const float4*>(sL + q0);
        const float4 D4 = *reinterpret_cast<const float4*>(sD + q0);
        const uint32_t wv[4] = {w4.x, w4.y, w4.z, w4.w};
        const float Lv[4] = {L4.x, L4.y, L4.z, L4.w}, Dv[4] = {D4.x, D4.y, D4.z, D4.w};
        bf16x4_t ds4;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * g4 + e;
          const bool ok = kok && q0 + e < Q && !((wv[e] >> r) & 1u);
          const float p = ok ? __expf(sacc[i] * g.scale - Lv[e]) : 0.f;
          sacc[i] = p;
          dacc[i] = p * (dacc[i] - Dv[e]);
          ds4[e] = bf16_bits(dacc[i]);
        }
        *reinterpret_cast<bf16x4_t*>(sDSt + woff(kl, q0 >> 3) + 8 * hh) = ds4;
      }
#pragma unroll
      for (int th = 0; th < 2; ++th) {           // k over the tile's queries, permuted order
        const int base = 32 * qt + 16 * th;
        dv = mfma16(tr_perm64(sDo, base, l), pack8(sacc, 8 * th), dv);
        dk = mfma16(tr_perm64(sQ, base, l), pack8(dacc, 8 * th), dk);
      }
    }
    if (kok) {
      bf16* gvr = gv + ((size_t)b * g.S + jbeg + kl) * C + h * kD;
      bf16* gkr = gk + ((size_t)b * g.S + jbeg + kl) * C + h * kD;
#pragma unroll
      for (int grp = 0; grp < 4; ++grp) {
        bf16x4_t av, ck;
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          av[e2] = bf16_bits(dv[4 * grp + e2]);
          ck[e2] = bf16_bits(dk[4 * grp + e2] * g.scale);
        }
        *reinterpret_cast<bf16x4_t*>(gvr + 8 * grp + 4 * hh) = av;
        *reinterpret_cast<bf16x4_t*>(gkr + 8 * grp + 4 * hh) = ck;
      }
    }
    __syncthreads();                            // every wave's dS^T is in LDS
    // dQ^T of query tile `wave` += K^T dS^T over the block's keys
#pragma unroll
    for (int tt = 0; tt < kBChunk / 16; ++tt)
      dq = mfma16(tr_nat64(sK, 16 * tt, l), tr_frag(sDSt, 16 * tt, 32 * wave, l), dq);
  }
  const int qr = 32 * wave + r;
  if (qr < Q) {
    float* dst = pdq + ((((size_t)b * g.heads + h) * g.nchunk + chunk) * Q + qr) * kD;
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) {
      float4 o;
      o.x = dq[4 * grp + 0] * g.scale;
      o.y = dq[4 * grp + 1] * g.scale;
      o.z = dq[4 * grp + 2] * g.scale;
      o.w = dq[4 * grp + 3] * g.scale;
      *reinterpret_cast<float4*>(dst + 8 * grp + 4 * hh) = o;
    }
  }
}

XGeom make_geom(int B, int Q, int S, int heads, float scale) {
  XGeom g;
  g.B = B; g.Q = Q; g.S = S; g.heads = heads; g.scale = scale;
  g.nw = (S + 31) / 32;
  // ~32 key chunks per (b, head) on long maps, at least one 128-key stage per chunk
  int chunk = (S + 31) / 32;
  chunk = ((chunk + kStage - 1) / kStage) * kStage;
  if (chunk < kStage) chunk = kStage;
  g.chunk = chunk;
  g.nchunk = (S + chunk - 1) / chunk;
  return g;
}

}  // namespace
}  // namespace vs

using namespace vs;

// chunking of the bf16 MFMA kernels (forward 256 keys, backward 128 keys per workgroup)
static XGeom mfma_geom(int B, int Q, int S, int heads, float scale, int chunk) {
  XGeom g = make_geom(B, Q, S, heads, scale);
  g.chunk = chunk;
  g.nchunk = (S + chunk - 1) / chunk;
  return g;
}

// VS_XATTN_SCALAR=1 selects the scalar-FMA kernels for bf16 too
static bool xattn_use_mfma() {
  const char* e = getenv("VS_XATTN_SCALAR");
  return !(e && atoi(e) != 0);
}

extern "C" long long vs_masked_attn_workspace_bytes(int B, int Q, int S, int heads) {
  XGeom g = make_geom(B, Q, S, heads, 1.f);
  const int nchunk = std::max(g.nchunk, (S + kBChunk - 1) / kBChunk);
  const long long rows = (long long)B * heads * nchunk * Q;
  return rows * (kD + 2) * 4 + (long long)B * heads * Q * 4 + 256;
}

extern "C" int vs_masked_attn_forward(int dtype, const void* q, const void* k, const void* v,
                                      const uint32_t* words, void* out, float* lse, void* workspace,
                                      int B, int Q, int S, int heads, float scale, void* stream) {
  VS_CHECK(q && k && v && words && out && lse && workspace, "null pointer");
  VS_CHECK(B > 0 && Q > 0 && S > 0 && heads > 0, "bad sizes");
  if (dtype == VS_BF16 && xattn_use_mfma()) {
    XGeom g = mfma_geom(B, Q, S, heads, scale, kFChunk);
    float* po = (float*)workspace;
    float* pml = po + (size_t)B * heads * g.nchunk * Q * kD;
    hipStream_t st = (hipStream_t)stream;
    dim3 grid(g.nchunk, heads, B * ((Q + 127) / 128));
    hipLaunchKernelGGL(xattn_fwd_mfma2, grid, dim3(256), 0, st, (const bf16*)q, (const bf16*)k, (const bf16*)v,
                       words, po, pml, g);
    const long long crows = (long long)B * heads * Q * 32;
    hipLaunchKernelGGL(xattn_fwd_combine<bf16>, dim3((int)((crows + 255) / 256)), dim3(256), 0, st, po, pml,
                       (bf16*)out, lse, g);
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
  XGeom g = make_geom(B, Q, S, heads, scale);
  float* po = (float*)workspace;
  float* pml = po + (size_t)B * heads * g.nchunk * Q * kD;
  hipStream_t st = (hipStream_t)stream;
  const int nqg = (Q + kQTile - 1) / kQTile;
  dim3 grid(g.nchunk, heads, B * nqg);
  const size_t lds = 2 * kStage * kD * sizeof(float);
  const long long crows = (long long)B * heads * Q * 32;
  const int cgrid = (int)((crows + 255) / 256);
  if (dtype == VS_BF16) {
    hipLaunchKernelGGL(xattn_fwd_partial<bf16>, grid, dim3(kQTile), lds, st, (const bf16*)q, (const bf16*)k,
                       (const bf16*)v, words, po, pml, g);
    hipLaunchKernelGGL(xattn_fwd_combine<bf16>, dim3(cgrid), dim3(256), 0, st, po, pml, (bf16*)out, lse, g);
  } else if (dtype == VS_F32) {
    hipLaunchKernelGGL(xattn_fwd_partial<float>, grid, dim3(kQTile), lds, st, (const float*)q, (const float*)k,
                       (const float*)v, words, po, pml, g);
    hipLaunchKernelGGL(xattn_fwd_combine<float>, dim3(cgrid), dim3(256), 0, st, po, pml, (float*)out, lse, g);
  } else {
    VS_CHECK(false, "dtype must be VS_F32 or VS_BF16");
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_masked_attn_backward(int dtype, const void* q, const void* k, const void* v,
                                       const uint32_t* words, const void* out, const float* lse,
                                       const void* grad_out, void* grad_q, void* grad_k, void* grad_v,
                                       void* workspace, int B, int Q, int S, int heads, float scale,
                                       void* stream) {
  VS_CHECK(q && k && v && words && out && lse && grad_out && grad_q && grad_k && grad_v && workspace,
           "null pointer");
  VS_CHECK(B > 0 && Q > 0 && S > 0 && heads > 0, "bad sizes");
  if (dtype == VS_BF16 && Q <= kBQ && xattn_use_mfma()) {
    // 128-key blocks, several per workgroup once there are >= 2048 blocks in the grid
    // (the Q^T / dO^T staging and the dQ partial are per workgroup; VS_XATTN_BLOCKS=n
    // forces n blocks per workgroup, for tests)
    const long long nb128 = (long long)B * heads * ((S + kBChunk - 1) / kBChunk);
    // C2's 128^2 level: 8 (one round of 2 workgroups per CU; kbench op 0.088 -> 0.085 ms with the
    // round-5 kernel, profiles/r5_xattn_ab.txt; 4 with the round-4 one: 0.174 -> 0.135 ms)
    int per = nb128 >= 4096 ? 8 : nb128 >= 2048 ? 2 : 1;
    if (const char* e = getenv("VS_XATTN_BLOCKS")) per = std::max(1, std::min(16, atoi(e)));
    XGeom g = mfma_geom(B, Q, S, heads, scale, kBChunk * per);
    float* pdq = (float*)workspace;
    float* Dbuf = pdq + (size_t)B * heads * g.nchunk * Q * kD + (size_t)B * heads * g.nchunk * Q * 2;
    hipStream_t st = (hipStream_t)stream;
    const long long rows = (long long)B * heads * Q;
    hipLaunchKernelGGL(xattn_bwd_prep<bf16>, dim3((int)((rows + 255) / 256)), dim3(256), 0, st, (const bf16*)out,
                       (const bf16*)grad_out, Dbuf, g);
    hipLaunchKernelGGL(xattn_bwd_mfma2, dim3(g.nchunk, heads, B), dim3(256), 0, st, (const bf16*)q, (const bf16*)k,
                       (const bf16*)v, words, lse, Dbuf, (const bf16*)grad_out, (bf16*)grad_k, (bf16*)grad_v, pdq, g);
    const long long total = rows * kD;
    hipLaunchKernelGGL(xattn_bwd_dq_combine<bf16>, dim3((int)((total + 255) / 256)), dim3(256), 0, st, pdq,
                       (bf16*)grad_q, g);
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
  XGeom g = make_geom(B, Q, S, heads, scale);
  const size_t lds_dkdv = (2 * (size_t)Q * kD + 2 * Q) * sizeof(float);
  VS_CHECK(lds_dkdv <= 160 * 1024, "too many queries for the dK/dV kernel");
  float* pdq = (float*)workspace;
  float* Dbuf = pdq + (size_t)B * heads * g.nchunk * Q * kD + (size_t)B * heads * g.nchunk * Q * 2;
  hipStream_t st = (hipStream_t)stream;
  const int nqg = (Q + kQTile - 1) / kQTile;
  dim3 grid(g.nchunk, heads, B * nqg);
  const size_t lds = 2 * kStage * kD * sizeof(float);
  const long long total = (long long)B * heads * Q * kD;
  const int cgrid = (int)((total + 255) / 256);
  dim3 kgrid((S + 255) / 256, heads, B);
  if (dtype == VS_BF16) {
    hipLaunchKernelGGL(xattn_bwd_dq_partial<bf16>, grid, dim3(kQTile), lds, st, (const bf16*)q, (const bf16*)k,
                       (const bf16*)v, words, (const bf16*)out, lse, (const bf16*)grad_out, pdq, Dbuf, g);
    hipLaunchKernelGGL(xattn_bwd_dq_combine<bf16>, dim3(cgrid), dim3(256), 0, st, pdq, (bf16*)grad_q, g);
    hipLaunchKernelGGL(xattn_bwd_dkdv<bf16>, kgrid, dim3(256), lds_dkdv, st, (const bf16*)q, (const bf16*)k,
                       (const bf16*)v, words, lse, Dbuf, (const bf16*)grad_out, (bf16*)grad_k, (bf16*)grad_v, g);
  } else if (dtype == VS_F32) {
    hipLaunchKernelGGL(xattn_bwd_dq_partial<float>, grid, dim3(kQTile), lds, st, (const float*)q, (const float*)k,
                       (const float*)v, words, (const float*)out, lse, (const float*)grad_out, pdq, Dbuf, g);
    hipLaunchKernelGGL(xattn_bwd_dq_combine<float>, dim3(cgrid), dim3(256), 0, st, pdq, (float*)grad_q, g);
    hipLaunchKernelGGL(xattn_bwd_dkdv<float>, kgrid, dim3(256), lds_dkdv, st, (const float*)q, (const float*)k,
                       (const float*)v, words, lse, Dbuf, (const float*)grad_out, (float*)grad_k, (float*)grad_v, g);
  } else {
    VS_CHECK(false, "dtype must be VS_F32 or VS_BF16");
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}
