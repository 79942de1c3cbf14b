// Decoder self-attention core (HF:m2f:1659-1664: Mask2FormerAttention over the queries,
// q = k = tgt + query_pos, v = tgt, no mask; MaskDINO's decoder runs the same core with the
// denoising-group mask, upstream dn_components attn_mask, True = blocked):
//
//   O_i = softmax_{j unblocked}( (q_i . k_j) * scale ) V      per (image, head), d = 32
//
// Layout: q [B, Q, heads*32], k / v [B, S, heads*32] bf16 (the fused in-projection outputs),
// optional words u32 [Q, ceil(S/32)] (shared by the batch, word_bstride = 0) or
// [B, Q, ceil(S/32)] (bit j%32 of word j/32 = key j blocked, shared by the heads),
// out [B, Q, heads*32] bf16, lse f32 [B, heads, Q] (natural log units; +inf for a row
// blocked at every key, whose output is 0).
//
// Precision: the two products whose operand is a softmax-derived f32 value (O = P V in the
// forward; dV = P^T dO, dK = dS^T Q, dQ = dS K in the backward) take that operand as an
// exact-to-2^-17 pair of bf16 values (hi = bf16(x), lo = bf16(x - hi)), two MFMAs per
// k-step; q / k / v / dO are bf16 already, so every product is f32-accumulated from
// f32-accurate operands.  The softmax, lse, D = rowsum(dO * O) and dS stay f32.  (PyTorch's
// SDPA on ROCm ran AOTriton kernels that round P and dS to bf16 -- the self-attention q / k
// weight gradients sat at 3.8x the bf16 yardstick of the training-step parity test.)
//
// Forward: workgroup = (128-query block, head, image), 4 waves of 32 queries; the keys are
// staged 128 at a time in their natural layout (lds_dma.h swz64, 64-B rows); per 32-key tile
// a wave forms S^T = K Q^T (a lane holds 16 keys of ONE query), applies the blocked bits
// (one word per lane and tile), runs the online softmax in registers (exp2, logits in log2
// units) and accumulates O^T += V^T P^T, V^T by the transposed LDS read in the permuted key
// order.  No split-K: Q and S are a few hundred at most, one workgroup sees every key.
//
// Backward: ONE launch, two workgroup roles (FlashAttention-2 split, no atomics, no
// partials):
//  * key role (blockIdx.x < key blocks): wave w owns 32 keys; the queries are staged 128 at a
//    time (Q, dO natural, lse, D, the blocked bits transposed to [key tile][query]); per
//    32-query tile S = Q K^T and dP = dO V^T (queries on rows), P and dS in registers, then
//    dV^T += dO^T P and dK^T += Q^T dS with dO^T / Q^T by the transposed read;
//  * query role: wave w owns 32 queries; the keys are staged 128 at a time; per 32-key tile
//    S^T and dP^T (keys on rows), dS^T in registers, dQ^T += K^T dS^T.
// D_i = dO_i . O_i is formed by each role from dO and the f32 copy of O the forward wrote
// (out_f32): with the bf16 output instead, D's rounding (2^-9 of |O| per channel) reached
// 0.5 % of max |dQ| at the C2 shape.
#include "lds_dma.h"

namespace vs {
namespace {

constexpr int kSaD = 32;      // head dim
constexpr int kSaBlk = 128;   // keys (forward / query role) or queries (key role) per stage
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

struct SaGeom {
  int B, Q, S, heads, nw;
  long long wbs;              // batch stride of the bitmask words (0: shared)
  float c1;                   // scale * log2(e)
  float scale;
};

// 8 consecutive C-tile registers -> (hi, lo) bf16 operands, x = hi + lo to 2^-17
__device__ __forceinline__ void pack8_hilo(const f32x16_t& a, int base, bf16x8_t& hi, bf16x8_t& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const short h = bf16_bits(a[base + j]);
    hi[j] = h;
    lo[j] = bf16_bits(a[base + j] - bf16_bits_to_f32((uint16_t)h));
  }
}

__device__ __forceinline__ bf16x8_t ld8_or0(const bf16* p, bool ok) { return ok ? ld8(p) : zero8(); }

// sum_j a[j] * o[j] over 8 bf16 values and 8 f32 values (two 16-B loads); 0 when !ok
__device__ __forceinline__ float dot8f(bf16x8_t a, const float* o, bool ok) {
  if (!ok) return 0.f;
  const float4 x = *reinterpret_cast<const float4*>(o), y = *reinterpret_cast<const float4*>(o + 4);
  const float ov[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s = fmaf(bf16_bits_to_f32((uint16_t)a[j]), ov[j], s);
  return s;
}

// stage 128 rows (token0 + t, t < 128) of one head of a [B, *, C] tensor into a natural
// 64-B-row image; rows past n are zero
__device__ __forceinline__ void stage_rows(short* img, const bf16* base, int C, int n) {
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int p = threadIdx.x + 256 * it, t = p >> 2, c = p & 3;
    *reinterpret_cast<bf16x8_t*>(img + swz64(t, c)) = ld8_or0(base + (size_t)t * C + 8 * c, t < n);
  }
}

template <bool MASK>
__global__ void __launch_bounds__(256) sa_fwd_kernel(const bf16* __restrict__ q, const bf16* __restrict__ k,
                                                     const bf16* __restrict__ v, const uint32_t* __restrict__ words,
                                                     bf16* __restrict__ out, float* __restrict__ out32,
                                                     float* __restrict__ lse, SaGeom g) {
  __shared__ __attribute__((aligned(16))) short sK[kSaBlk * kSaD];
  __shared__ __attribute__((aligned(16))) short sV[kSaBlk * kSaD];
  const int h = blockIdx.y, b = blockIdx.z;
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int C = g.heads * kSaD;
  const int qi = blockIdx.x * kSaBlk + wave * 32 + r;
  const bool qok = qi < g.Q;
  bf16x8_t qf[2];
#pragma unroll
  for (int st = 0; st < 2; ++st) qf[st] = ld8_or0(q + ((size_t)b * g.Q + qi) * C + h * kSaD + 16 * st + 8 * hh, qok);
  const uint32_t* wrow = MASK ? words + b * g.wbs + (size_t)(qok ? qi : 0) * g.nw : nullptr;
  float m = -INFINITY, lsum = 0.f;
  f32x16_t o;
  zero16(o);
  const int nkb = (g.S + kSaBlk - 1) / kSaBlk;
  for (int kb = 0; kb < nkb; ++kb) {
    const int j0 = kb * kSaBlk;
    const int n = min(kSaBlk, g.S - j0);
    if (kb > 0) __syncthreads();                 // the previous block's K / V are read
    stage_rows(sK, k + ((size_t)b * g.S + j0) * C + h * kSaD, C, n);
    stage_rows(sV, v + ((size_t)b * g.S + j0) * C + h * kSaD, C, n);
    uint32_t wv[kSaBlk / 32];
#pragma unroll
    for (int kt = 0; kt < kSaBlk / 32; ++kt)
      wv[kt] = MASK ? ((qok && kt * 32 < n) ? wrow[(j0 >> 5) + kt] : 0xffffffffu) : 0u;
    __syncthreads();
    const int ntiles = (n + 31) / 32;
#pragma unroll
    for (int kt = 0; kt < kSaBlk / 32; ++kt) {
      if (kt >= ntiles) break;
      f32x16_t sc;
      zero16(sc);
#pragma unroll
      for (int st = 0; st < 2; ++st)
        sc = mfma16(*reinterpret_cast<const bf16x8_t*>(sK + swz64(32 * kt + r, 2 * st + hh)), qf[st], sc);
      float mt = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kl = crow(i, hh);
        const bool blocked = (kt * 32 + kl >= n) || (MASK && ((wv[kt] >> kl) & 1u));
        sc[i] = blocked ? -INFINITY : sc[i] * g.c1;
        mt = fmaxf(mt, sc[i]);
      }
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float mn = fmaxf(m, mt);
      const float safe = mn == -INFINITY ? 0.f : mn;
      const float alpha = exp2f(m - safe);
      lsum *= alpha;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        o[i] *= alpha;
        sc[i] = exp2f(sc[i] - safe);
        lsum += sc[i];
      }
      m = mn;
#pragma unroll
      for (int th = 0; th < 2; ++th) {
        bf16x8_t ph, pl;
        pack8_hilo(sc, 8 * th, ph, pl);
        const bf16x8_t vt = tr_perm64(sV, kt * 32 + 16 * th, l);
        o = mfma16(vt, ph, o);
        o = mfma16(vt, pl, o);
      }
    }
  }
  lsum += __shfl_xor(lsum, 32, 64);
  if (qok) {
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    bf16* dst = out + ((size_t)b * g.Q + qi) * C + h * kSaD;
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) {
      bf16x4_t ov;
#pragma unroll
      for (int e = 0; e < 4; ++e) ov[e] = bf16_bits(o[4 * grp + e] * inv);
      *reinterpret_cast<bf16x4_t*>(dst + 8 * grp + 4 * hh) = ov;
      if (out32)
        *reinterpret_cast<float4*>(out32 + ((size_t)b * g.Q + qi) * C + h * kSaD + 8 * grp + 4 * hh) =
            make_float4(o[4 * grp] * inv, o[4 * grp + 1] * inv, o[4 * grp + 2] * inv, o[4 * grp + 3] * inv);
    }
    if (hh == 0) lse[((size_t)b * g.heads + h) * g.Q + qi] = lsum > 0.f ? (m + log2f(lsum)) * kLn2 : INFINITY;
  }
}

template <bool MASK>
__global__ void __launch_bounds__(256) sa_bwd_kernel(const bf16* __restrict__ q, const bf16* __restrict__ k,
                                                     const bf16* __restrict__ v, const uint32_t* __restrict__ words,
                                                     const float* __restrict__ out32, const float* __restrict__ lse,
                                                     const bf16* __restrict__ gout, bf16* __restrict__ gq,
                                                     bf16* __restrict__ gk, bf16* __restrict__ gv, SaGeom g) {
  __shared__ __attribute__((aligned(16))) short sA[kSaBlk * kSaD];    // Q (key role) / K (query role)
  __shared__ __attribute__((aligned(16))) short sB[kSaBlk * kSaD];    // dO (key role) / V (query role)
  __shared__ __attribute__((aligned(16))) float sL[kSaBlk], sD[kSaBlk];
  __shared__ __attribute__((aligned(16))) uint32_t sWt[kSaBlk / 32][kSaBlk];
  const int h = blockIdx.y, b = blockIdx.z;
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int C = g.heads * kSaD;
  const int nkb = (g.S + kSaBlk - 1) / kSaBlk, nqb = (g.Q + kSaBlk - 1) / kSaBlk;
  const size_t hq = (size_t)h * kSaD;
  if ((int)blockIdx.x < nkb) {
    // ---------------- key role: dK, dV of keys kb*128 + 32 wave + r
    const int kb = blockIdx.x;
    const int kl = kb * kSaBlk + wave * 32 + r;
    const bool kok = kl < g.S;
    bf16x8_t kf[2], vf[2];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      kf[st] = ld8_or0(k + ((size_t)b * g.S + kl) * C + hq + 16 * st + 8 * hh, kok);
      vf[st] = ld8_or0(v + ((size_t)b * g.S + kl) * C + hq + 16 * st + 8 * hh, kok);
    }
    f32x16_t dv, dk;
    zero16(dv);
    zero16(dk);
    for (int qb = 0; qb < nqb; ++qb) {
      const int i0 = qb * kSaBlk;
      const int nq = min(kSaBlk, g.Q - i0);
      if (qb > 0) __syncthreads();
      stage_rows(sA, q + ((size_t)b * g.Q + i0) * C + hq, C, nq);
      stage_rows(sB, gout + ((size_t)b * g.Q + i0) * C + hq, C, nq);
      {  // lse (log2 units) and D = dO . O: two threads per query, 16 channels each
        const int t = threadIdx.x >> 1, half = threadIdx.x & 1;
        const bool ok = t < nq;
        const size_t row = ((size_t)b * g.Q + i0 + t) * C + hq + 16 * half;
        float dsum = dot8f(ld8_or0(gout + row, ok), out32 + row, ok) + dot8f(ld8_or0(gout + row + 8, ok), out32 + row + 8, ok);
        dsum += __shfl_xor(dsum, 1, 64);
        if (half == 0) {
          sD[t] = dsum;
          sL[t] = ok ? lse[((size_t)b * g.heads + h) * g.Q + i0 + t] * kLog2e : INFINITY;
        }
      }
      if (MASK) {
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          const int p = threadIdx.x + 256 * it, qq = p & 127, wg = p >> 7;
          const int wi = kb * (kSaBlk / 32) + wg;
          sWt[wg][qq] = (qq < nq && wi < g.nw) ? words[b * g.wbs + (size_t)(i0 + qq) * g.nw + wi] : 0xffffffffu;
        }
      }
      __syncthreads();
      const int nqt = (nq + 31) / 32;
#pragma unroll 1
      for (int qt = 0; qt < nqt; ++qt) {
        f32x16_t sacc, dacc;
        zero16(sacc);
        zero16(dacc);
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const int t = 32 * qt + r, c = 2 * st + hh;
          sacc = mfma16(*reinterpret_cast<const bf16x8_t*>(sA + swz64(t, c)), kf[st], sacc);
          dacc = mfma16(*reinterpret_cast<const bf16x8_t*>(sB + swz64(t, c)), vf[st], dacc);
        }
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int q0 = 32 * qt + 8 * g4 + 4 * hh;
          const float4 L4 = *reinterpret_cast<const float4*>(sL + q0);
          const float4 D4 = *reinterpret_cast<const float4*>(sD + q0);
          const float Lv[4] = {L4.x, L4.y, L4.z, L4.w}, Dv[4] = {D4.x, D4.y, D4.z, D4.w};
          uint32_t wv[4] = {0u, 0u, 0u, 0u};
          if (MASK) {
            const uint4 w4 = *reinterpret_cast<const uint4*>(&sWt[wave][q0]);
            wv[0] = w4.x; wv[1] = w4.y; wv[2] = w4.z; wv[3] = w4.w;
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int i = 4 * g4 + e;
            const bool ok = kok && !(MASK && ((wv[e] >> r) & 1u));
            const float p = ok ? exp2f(sacc[i] * g.c1 - Lv[e]) : 0.f;
            sacc[i] = p;
            dacc[i] = p * (dacc[i] - Dv[e]);
          }
        }
#pragma unroll
        for (int th = 0; th < 2; ++th) {           // k over the tile's queries, permuted order
          const int base = 32 * qt + 16 * th;
          bf16x8_t hi, lo;
          pack8_hilo(sacc, 8 * th, hi, lo);
          const bf16x8_t dot_ = tr_perm64(sB, base, l);
          dv = mfma16(dot_, hi, dv);
          dv = mfma16(dot_, lo, dv);
          pack8_hilo(dacc, 8 * th, hi, lo);
          const bf16x8_t qt_ = tr_perm64(sA, base, l);
          dk = mfma16(qt_, hi, dk);
          dk = mfma16(qt_, lo, dk);
        }
      }
    }
    if (kok) {
      bf16* gvr = gv + ((size_t)b * g.S + kl) * C + hq;
      bf16* gkr = gk + ((size_t)b * g.S + kl) * C + hq;
#pragma unroll
      for (int grp = 0; grp < 4; ++grp) {
        bf16x4_t av, ck;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          av[e] = bf16_bits(dv[4 * grp + e]);
          ck[e] = bf16_bits(dk[4 * grp + e] * g.scale);
        }
        *reinterpret_cast<bf16x4_t*>(gvr + 8 * grp + 4 * hh) = av;
        *reinterpret_cast<bf16x4_t*>(gkr + 8 * grp + 4 * hh) = ck;
      }
    }
    return;
  }
  // ---------------- query role: dQ of queries qb*128 + 32 wave + r
  const int qb = blockIdx.x - nkb;
  if (qb >= nqb) return;
  const int qi = qb * kSaBlk + wave * 32 + r;
  const bool qok = qi < g.Q;
  bf16x8_t qf[2], of[2];
  float dpart = 0.f;
  const size_t qrow = ((size_t)b * g.Q + qi) * C + hq;
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    qf[st] = ld8_or0(q + qrow + 16 * st + 8 * hh, qok);
    of[st] = ld8_or0(gout + qrow + 16 * st + 8 * hh, qok);
    dpart += dot8f(of[st], out32 + qrow + 16 * st + 8 * hh, qok);
  }
  const float Dq = dpart + __shfl_xor(dpart, 32, 64);
  const float L2 = qok ? lse[((size_t)b * g.heads + h) * g.Q + qi] * kLog2e : INFINITY;
  const uint32_t* wrow = MASK ? words + b * g.wbs + (size_t)(qok ? qi : 0) * g.nw : nullptr;
  f32x16_t dq;
  zero16(dq);
  for (int kb = 0; kb < nkb; ++kb) {
    const int j0 = kb * kSaBlk;
    const int n = min(kSaBlk, g.S - j0);
    if (kb > 0) __syncthreads();
    stage_rows(sA, k + ((size_t)b * g.S + j0) * C + hq, C, n);
    stage_rows(sB, v + ((size_t)b * g.S + j0) * C + hq, C, n);
    uint32_t wv[kSaBlk / 32];
#pragma unroll
    for (int kt = 0; kt < kSaBlk / 32; ++kt)
      wv[kt] = MASK ? ((qok && kt * 32 < n) ? wrow[(j0 >> 5) + kt] : 0xffffffffu) : 0u;
    __syncthreads();
    const int ntiles = (n + 31) / 32;
#pragma unroll
    for (int kt = 0; kt < kSaBlk / 32; ++kt) {
      if (kt >= ntiles) break;
      f32x16_t sacc, dacc;
      zero16(sacc);
      zero16(dacc);
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const int t = 32 * kt + r, c = 2 * st + hh;
        sacc = mfma16(*reinterpret_cast<const bf16x8_t*>(sA + swz64(t, c)), qf[st], sacc);
        dacc = mfma16(*reinterpret_cast<const bf16x8_t*>(sB + swz64(t, c)), of[st], dacc);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kl = crow(i, hh);
        const bool ok = (kt * 32 + kl < n) && !(MASK && ((wv[kt] >> kl) & 1u));
        const float p = ok ? exp2f(sacc[i] * g.c1 - L2) : 0.f;
        dacc[i] = p * (dacc[i] - Dq);
      }
#pragma unroll
      for (int th = 0; th < 2; ++th) {
        bf16x8_t hi, lo;
        pack8_hilo(dacc, 8 * th, hi, lo);
        const bf16x8_t kt_ = tr_perm64(sA, kt * 32 + 16 * th, l);
        dq = mfma16(kt_, hi, dq);
        dq = mfma16(kt_, lo, dq);
      }
    }
  }
  if (qok) {
    bf16* dst = gq + qrow;
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) {
      bf16x4_t o4;
#pragma unroll
      for (int e = 0; e < 4; ++e) o4[e] = bf16_bits(dq[4 * grp + e] * g.scale);
      *reinterpret_cast<bf16x4_t*>(dst + 8 * grp + 4 * hh) = o4;
    }
  }
}

SaGeom sa_geom(int B, int Q, int S, int heads, float scale, long long word_bstride) {
  SaGeom g;
  g.B = B; g.Q = Q; g.S = S; g.heads = heads;
  g.nw = (S + 31) / 32;
  g.wbs = word_bstride;
  g.scale = scale;
  g.c1 = scale * kLog2e;
  return g;
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" int vs_self_attn_forward(int dtype, const void* q, const void* k, const void* v, const uint32_t* words,
                                    long long word_bstride, void* out, float* out_f32, float* lse, int B, int Q, int S,
                                    int heads, float scale, void* stream) {
  VS_CHECK(dtype == VS_BF16, "the self-attention kernels take bf16 q / k / v (f32: vs_masked_attn_forward)");
  VS_CHECK(q && k && v && out && lse, "null pointer");
  VS_CHECK(B > 0 && Q > 0 && S > 0 && heads > 0, "bad sizes");
  VS_CHECK(word_bstride >= 0, "bad word batch stride");
  VS_CHECK(((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)out | (uintptr_t)out_f32) % 16 == 0,
           "q / k / v / out must be 16-B aligned");
  const SaGeom g = sa_geom(B, Q, S, heads, scale, word_bstride);
  const dim3 grid((Q + kSaBlk - 1) / kSaBlk, heads, B);
  hipStream_t st = (hipStream_t)stream;
  if (words)
    hipLaunchKernelGGL(sa_fwd_kernel<true>, grid, dim3(256), 0, st, (const bf16*)q, (const bf16*)k, (const bf16*)v,
                       words, (bf16*)out, out_f32, lse, g);
  else
    hipLaunchKernelGGL(sa_fwd_kernel<false>, grid, dim3(256), 0, st, (const bf16*)q, (const bf16*)k, (const bf16*)v,
                       words, (bf16*)out, out_f32, lse, g);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_self_attn_backward(int dtype, const void* q, const void* k, const void* v, const uint32_t* words,
                                     long long word_bstride, const float* out_f32, const float* lse, const void* grad_out,
                                     void* grad_q, void* grad_k, void* grad_v, int B, int Q, int S, int heads,
                                     float scale, void* stream) {
  VS_CHECK(dtype == VS_BF16, "the self-attention kernels take bf16 q / k / v (f32: vs_masked_attn_backward)");
  VS_CHECK(q && k && v && out_f32 && lse && grad_out && grad_q && grad_k && grad_v, "null pointer");
  VS_CHECK(B > 0 && Q > 0 && S > 0 && heads > 0, "bad sizes");
  VS_CHECK(word_bstride >= 0, "bad word batch stride");
  VS_CHECK(((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)out_f32 | (uintptr_t)grad_out | (uintptr_t)grad_q |
            (uintptr_t)grad_k | (uintptr_t)grad_v) % 16 == 0,
           "operands must be 16-B aligned");
  const SaGeom g = sa_geom(B, Q, S, heads, scale, word_bstride);
  const int nkb = (S + kSaBlk - 1) / kSaBlk, nqb = (Q + kSaBlk - 1) / kSaBlk;
  const dim3 grid(nkb + nqb, heads, B);
  hipStream_t st = (hipStream_t)stream;
  if (words)
    hipLaunchKernelGGL(sa_bwd_kernel<true>, grid, dim3(256), 0, st, (const bf16*)q, (const bf16*)k, (const bf16*)v,
                       words, out_f32, lse, (const bf16*)grad_out, (bf16*)grad_q, (bf16*)grad_k,
                       (bf16*)grad_v, g);
  else
    hipLaunchKernelGGL(sa_bwd_kernel<false>, grid, dim3(256), 0, st, (const bf16*)q, (const bf16*)k, (const bf16*)v,
                       words, out_f32, lse, (const bf16*)grad_out, (bf16*)grad_q, (bf16*)grad_k,
                       (bf16*)grad_v, g);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
