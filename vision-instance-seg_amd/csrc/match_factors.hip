// Matcher cost and decoder attention masks from the mask head's FACTORS (round 4).
//
// The mask logits of decoder step s are L_s[b, q, n] = E_s[b, q, :] . F[b, n, :] (E = the
// mask embedding, F = the channels-last pixel embedding; csrc/mask_head.hip).  Everything
// the training step reads from the full-resolution L_s other than the matched rows is a
// LINEAR resampling of it:
//   * the matcher's point logits (HF:m2f:453-459, point_sample = grid_sample bilinear,
//     align_corners=False, zero padding): L_s at point p = E_s . F(p), F(p) = the same
//     bilinear combination of F's pixel rows;
//   * the next layer's attention mask (HF:m2f:2049-2055): bilinear resize of L_s to the
//     level's size = E_s . resize(F).
// So F is resampled ONCE per step (C channels instead of S x Q logit maps) and the
// logits at the few positions needed are small GEMMs.  The resampled rows are kept as an
// exact-to-2^-17 pair of bf16 values (hi = bf16(v), lo = bf16(v - hi)), so with E in bf16
// the MFMA products reproduce the f32 logits of the full-resolution path up to the f32
// summation order (no extra rounding of the features).
//
// Kernels:
//   feat_resize_hilo   F [B, H*W, C] bf16 -> [B, th*tw, 2C] bf16 (hi | lo), PyTorch
//                      upsample_bilinear2d (align_corners=False) index rule;
//   feat_sample_hilo   F at grid points [B, P, 2] (grid_sample rule) -> [B, P, 2C];
//   match_cost_fac     per (image, column group of 256 (step, query) columns, point range):
//                      X^T tile = F(p) E^T on v_mfma_f32_32x32x16_bf16 (hi and lo), then in
//                      registers sp = softplus(x), sg = sigmoid(x) and the sums the costs
//                      need (SP_q = sum sp, SG_q = sum sg, N_qk = sum sg t_k, X_qk = sum x t_k,
//                      T_k = sum t_k) -> f32 partials per point range;
//   match_cost_fac_fin partials summed in a fixed order -> cost[s, b, q, k] as
//                      HungarianMatcher (HF:m2f:434-481):
//                      wm (SP - X)/P + wc (-prob[cls_k]) + wd (1 - (2N + 1)/(SG + T + 1))
//                      (softplus(-x) t + softplus(x)(1 - t) = softplus(x) - x t), clamped to
//                      +-1e10, NaN -> 0.
// Deterministic: no atomics, fixed reduction orders.
#include "common.h"
#include "mfma_util.h"

namespace vs {
namespace {

__device__ __forceinline__ void hilo8(const float* v, bf16x8_t& hi, bf16x8_t& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const short h = bf16_bits(v[j]);
    hi[j] = h;
    lo[j] = bf16_bits(v[j] - bf16_bits_to_f32((unsigned short)h));
  }
}

__device__ __forceinline__ void add8(float* acc, const bf16x8_t& x, float w) {
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = fmaf(w, bf16_bits_to_f32((unsigned short)x[j]), acc[j]);
}

// PyTorch upsample_bilinear2d (align_corners=False, scale = in / out) source index, one axis
__device__ __forceinline__ void lin_src(int dst, int in, int out, int& i0, int& i1, float& l0, float& l1) {
  const float scale = (float)in / (float)out;
  float s = scale * ((float)dst + 0.5f) - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = (int)s;
  i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  l1 = s - (float)i0;
  l0 = 1.f - l1;
}

// one thread per (output row, 8-channel chunk)
__global__ void __launch_bounds__(256) feat_resize_hilo_kernel(const bf16* __restrict__ F, bf16* __restrict__ out,
                                                               int B, int H, int W, int C, int th, int tw) {
  const int chunks = C / 8;
  const long long total = (long long)B * th * tw * chunks;
  for (long long id = (long long)blockIdx.x * 256 + threadIdx.x; id < total; id += (long long)gridDim.x * 256) {
    const int c = (int)(id % chunks) * 8;
    const long long row = id / chunks;
    const int x = (int)(row % tw), y = (int)((row / tw) % th), b = (int)(row / ((long long)tw * th));
    int y0, y1, x0, x1;
    float ly0, ly1, lx0, lx1;
    lin_src(y, H, th, y0, y1, ly0, ly1);
    lin_src(x, W, tw, x0, x1, lx0, lx1);
    const bf16* Fb = F + (size_t)b * H * W * C + c;
    const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(Fb + ((size_t)y0 * W + x0) * C);
    const bf16x8_t bb = *reinterpret_cast<const bf16x8_t*>(Fb + ((size_t)y0 * W + x1) * C);
    const bf16x8_t cc = *reinterpret_cast<const bf16x8_t*>(Fb + ((size_t)y1 * W + x0) * C);
    const bf16x8_t d = *reinterpret_cast<const bf16x8_t*>(Fb + ((size_t)y1 * W + x1) * C);
    float top[8] = {}, bot[8] = {}, v[8];
    add8(top, a, lx0);
    add8(top, bb, lx1);
    add8(bot, cc, lx0);
    add8(bot, d, lx1);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ly0 * top[j] + ly1 * bot[j];
    bf16x8_t hi, lo;
    hilo8(v, hi, lo);
    bf16* o = out + row * 2 * C + c;
    *reinterpret_cast<bf16x8_t*>(o) = hi;
    *reinterpret_cast<bf16x8_t*>(o + C) = lo;
  }
}

// grid_sample (bilinear, zeros padding, align_corners=False) of F at grid [B, P, 2]
__global__ void __launch_bounds__(256) feat_sample_hilo_kernel(const bf16* __restrict__ F, const float* __restrict__ grid,
                                                               bf16* __restrict__ out, int B, int H, int W, int C,
                                                               int P) {
  const int chunks = C / 8;
  const long long total = (long long)B * P * chunks;
  for (long long id = (long long)blockIdx.x * 256 + threadIdx.x; id < total; id += (long long)gridDim.x * 256) {
    const int c = (int)(id % chunks) * 8;
    const long long row = id / chunks;                 // (b, p)
    const int b = (int)(row / P);
    const float2 g = *reinterpret_cast<const float2*>(grid + row * 2);
    const float ix = ((g.x + 1.f) * W - 1.f) / 2.f;
    const float iy = ((g.y + 1.f) * H - 1.f) / 2.f;
    const float fx = floorf(ix), fy = floorf(iy);
    const int x0 = (int)fx, y0 = (int)fy;
    const float wx1 = ix - fx, wx0 = (fx + 1.f) - ix, wy1 = iy - fy, wy0 = (fy + 1.f) - iy;
    const bf16* Fb = F + (size_t)b * H * W * C + c;
    float v[8] = {};
#pragma unroll
    for (int cn = 0; cn < 4; ++cn) {
      const int yy = y0 + (cn >> 1), xx = x0 + (cn & 1);
      if (xx >= 0 && xx < W && yy >= 0 && yy < H) {
        const float w = ((cn >> 1) ? wy1 : wy0) * ((cn & 1) ? wx1 : wx0);
        add8(v, *reinterpret_cast<const bf16x8_t*>(Fb + ((size_t)yy * W + xx) * C), w);
      }
    }
    bf16x8_t hi, lo;
    hilo8(v, hi, lo);
    bf16* o = out + row * 2 * C + c;
    *reinterpret_cast<bf16x8_t*>(o) = hi;
    *reinterpret_cast<bf16x8_t*>(o + C) = lo;
  }
}

constexpr int kCostWaves = 8;                 // 8 column tiles of 32 = 256 columns per workgroup
constexpr int kCols = 32 * kCostWaves;

// Partials layout: part[b][ps][f][col], f = 0: SP, 1: SG, 2..2+KT: N_k, 2+KT..2+2KT: X_k
// (col padded to NCG * 256); tpart[b][ps][k] = sum of t_k over the range's points.
template <int KC, int KT>
__global__ void __launch_bounds__(64 * kCostWaves, 1) match_cost_fac_kernel(
    const bf16* __restrict__ E, const bf16* __restrict__ Fp, const float* __restrict__ tp, float* __restrict__ part,
    float* __restrict__ tpart, int S, int B, int Q, int P, int Kc, int NCG, int PS, int tiles_per) {
  constexpr int LD = 2 * KC + 8;              // LDS row pitch (shorts): hi | lo + 16 B
  constexpr int NF = 2 + 2 * KT;
  __shared__ __attribute__((aligned(16))) short sF[32 * LD];
  __shared__ __attribute__((aligned(16))) float sT[KT * 32];
  // logical id: consecutive ids = the column groups of one (image, point range); the
  // XCD-aware remap keeps them on one XCD, so the range's feature rows go through one L2
  const int id = xcd_swizzle(blockIdx.x, gridDim.x);
  const int cg = id % NCG, ps = (id / NCG) % PS, b = id / (NCG * PS);
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int SQ = S * Q, SQp = NCG * kCols;
  const int col = cg * kCols + wave * 32 + r;
  // this lane's column (step, query) of E^T: KC/16 fragments kept in registers
  bf16x8_t ef[KC / 16];
  {
    const bool ok = col < SQ;
    const int s = ok ? col / Q : 0, q = ok ? col % Q : 0;
    const bf16* er = E + (((size_t)s * B + b) * Q + q) * KC + 8 * hh;
#pragma unroll
    for (int k = 0; k < KC / 16; ++k)
      ef[k] = ok ? *reinterpret_cast<const bf16x8_t*>(er + 16 * k) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  }
  const int ntiles = (P + 31) / 32;
  const int t0 = ps * tiles_per, t1 = min(ntiles, t0 + tiles_per);
  // staging map: 32 rows x (2 KC / 8) 16-B chunks over 512 threads
  constexpr int CH = 2 * KC / 8;
  constexpr int PER = 32 * CH / (64 * kCostWaves);
  static_assert(PER * 64 * kCostWaves == 32 * CH, "staging map");
  const bf16* Fb = Fp + (size_t)b * P * 2 * KC;
  const float* tb = tp + (size_t)b * Kc * P;
  uint4 nf[PER];
  float nt = 0.f, tacc = 0.f;
  const int tk = threadIdx.x >> 5, tj = threadIdx.x & 31;      // this thread's t slot (k, point)
  auto fetch = [&](int tile) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int idx = threadIdx.x + u * 64 * kCostWaves, row = idx / CH, c = idx % CH;
      const int p = tile * 32 + row;
      nf[u] = p < P ? *reinterpret_cast<const uint4*>(Fb + (size_t)p * 2 * KC + 8 * c) : make_uint4(0, 0, 0, 0);
    }
    const int p = tile * 32 + tj;
    nt = (tk < Kc && p < P) ? tb[(size_t)tk * P + p] : 0.f;
  };
  float SP = 0.f, SG = 0.f, N[KT], X[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) N[k] = X[k] = 0.f;
  if (t0 < t1) fetch(t0);
  for (int tile = t0; tile < t1; ++tile) {
    __syncthreads();                          // previous tile's LDS reads done
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int idx = threadIdx.x + u * 64 * kCostWaves, row = idx / CH, c = idx % CH;
      *reinterpret_cast<uint4*>(sF + row * LD + 8 * c) = nf[u];
    }
    if (tk < KT) {
      sT[tk * 32 + tj] = nt;
      tacc += nt;
    }
    __syncthreads();
    if (tile + 1 < t1) fetch(tile + 1);
    f32x16_t ah, al;
    zero16(ah);
    zero16(al);
#pragma unroll
    for (int k = 0; k < KC / 16; ++k) {
      const bf16x8_t fh = *reinterpret_cast<const bf16x8_t*>(sF + r * LD + 16 * k + 8 * hh);
      const bf16x8_t fl = *reinterpret_cast<const bf16x8_t*>(sF + r * LD + KC + 16 * k + 8 * hh);
      ah = mfma16(fh, ef[k], ah);
      al = mfma16(fl, ef[k], al);
    }
    // rows = points crow(i, hh) of the tile, column = this lane's (step, query)
    float sg[16], xv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int p = tile * 32 + crow(i, hh);
      const float x = ah[i] + al[i];
      const float vm = p < P ? 1.f : 0.f;
      // one exponential for both: e = exp(-|x|), sigmoid = (x >= 0 ? 1 : e) / (1 + e),
      // softplus = max(x, 0) + log(1 + e)
      const float e = __expf(-fabsf(x));
      const float inv = __frcp_rn(1.f + e);
      xv[i] = x;
      sg[i] = (x >= 0.f ? 1.f : e) * inv;
      SP = fmaf(vm, fmaxf(x, 0.f) + __logf(1.f + e), SP);
      SG = fmaf(vm, sg[i], SG);
    }
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      if (k < Kc) {                           // uniform branch
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const float4 t4 = *reinterpret_cast<const float4*>(sT + k * 32 + 8 * g4 + 4 * hh);
          const float tv[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            N[k] = fmaf(sg[4 * g4 + e], tv[e], N[k]);
            X[k] = fmaf(xv[4 * g4 + e], tv[e], X[k]);
          }
        }
      }
    }
  }
  // lane halves hold the same column's two point halves
  SP += __shfl_xor(SP, 32, 64);
  SG += __shfl_xor(SG, 32, 64);
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    N[k] += __shfl_xor(N[k], 32, 64);
    X[k] += __shfl_xor(X[k], 32, 64);
  }
  if (hh == 0) {
    float* pb = part + ((size_t)b * PS + ps) * NF * SQp + col;
    pb[0] = SP;
    pb[(size_t)SQp] = SG;
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      pb[(size_t)(2 + k) * SQp] = N[k];
      pb[(size_t)(2 + KT + k) * SQp] = X[k];
    }
  }
  if (cg == 0 && tk < KT) {                   // column group 0 also reports sum_p t_k
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) tacc += __shfl_xor(tacc, o, 64);
    if (tj == 0) tpart[((size_t)b * PS + ps) * KT + tk] = tacc;
  }
}

// 4 lanes per column, each summing every 4th point range; the four partial sums are then
// combined in lane order (fixed: deterministic) -- a quarter of the serial load rounds
template <int KT>
__global__ void __launch_bounds__(256) match_cost_fac_fin_kernel(const float* __restrict__ part,
                                                                 const float* __restrict__ tpart,
                                                                 const float* __restrict__ probs, int C1,
                                                                 const long long* __restrict__ tcls,
                                                                 float* __restrict__ cost, int S, int B, int Q, int P,
                                                                 int Kc, int NCG, int PS, float wm, float wc,
                                                                 float wd) {
  constexpr int NF = 2 + 2 * KT;
  const int b = blockIdx.y;
  const int j = threadIdx.x & 3;
  const int col = blockIdx.x * 64 + (threadIdx.x >> 2);
  const int SQ = S * Q, SQp = NCG * kCols;
  const bool ok = col < SQ;                  // no early return: the shuffles need all lanes
  const int cc = ok ? col : 0;
  float SP = 0.f, SG = 0.f, N[KT], X[KT], T[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) N[k] = X[k] = T[k] = 0.f;
#pragma unroll 2
  for (int ps = j; ps < PS; ps += 4) {
    const float* pb = part + ((size_t)b * PS + ps) * NF * SQp + cc;
    SP += pb[0];
    SG += pb[(size_t)SQp];
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      if (k < Kc) {
        N[k] += pb[(size_t)(2 + k) * SQp];
        X[k] += pb[(size_t)(2 + KT + k) * SQp];
        T[k] += tpart[((size_t)b * PS + ps) * KT + k];
      }
    }
  }
  // lane order 0 + 1 + 2 + 3 (the 4 lanes of a column are consecutive)
  auto comb = [&](float v) {
    const float v1 = __shfl_down(v, 1, 64), v2 = __shfl_down(v, 2, 64), v3 = __shfl_down(v, 3, 64);
    return ((v + v1) + v2) + v3;
  };
  SP = comb(SP);
  SG = comb(SG);
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    N[k] = comb(N[k]);
    X[k] = comb(X[k]);
    T[k] = comb(T[k]);
  }
  if (!ok || j != 0) return;
  const int s = col / Q, q = col % Q;
  const float* pr = probs + (((size_t)s * B + b) * Q + q) * C1;
  float* out = cost + (((size_t)s * B + b) * Q + q) * Kc;
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    if (k < Kc) {
      const float prob = pr[(int)tcls[(size_t)b * Kc + k]];
      const float cm = (SP - X[k]) / (float)P;
      const float cd = 1.f - (2.f * N[k] + 1.f) / (SG + T[k] + 1.f);
      float c = wm * cm + wc * (-prob) + wd * cd;
      c = fminf(fmaxf(c, -1e10f), 1e10f);
      if (c != c) c = 0.f;
      out[k] = c;
    }
  }
}

// Attention bitmask of the next decoder layer straight from the factors at the level's size:
// x = E . (hi + lo) per (query, key) on the MFMA (2 products per k-step sharing E), key
// blocked iff 1 / (1 + exp(-x)) < 0.5 -- the same expression as vs_attn_bitmask -- packed
// per lane into the query's 32-key word.  One wave per (32-query tile, 32-key
// tile); a workgroup's 4 waves take 4 query tiles of one key tile (they read the same
// feature rows: L1).  The logits never reach HBM.  Rows blocked at every key are un-blocked
// afterwards by bitmask_row_fix_kernel (HF:m2f:1912-1914).
template <int KC>
__global__ void __launch_bounds__(256) level_bitmask_kernel(const bf16* __restrict__ E, const bf16* __restrict__ Fhl,
                                                            uint32_t* __restrict__ words, int B, int Q, int N,
                                                            int nwords, int qgroups, int ktiles) {
  const int id = xcd_swizzle(blockIdx.x, gridDim.x);
  const int qg = id % qgroups, kt = (id / qgroups) % ktiles, b = id / (qgroups * ktiles);
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int q0 = (qg * 4 + wave) * 32;
  if (q0 >= Q) return;                                   // whole wave: no barrier below
  const int q = q0 + r, n = kt * 32 + r;
  // rows past Q / N are clamped onto row 0: their results are never stored (q >= Q) or
  // masked out of the bits (keys >= N), so no selects; every load of a batch is issued
  // before its products (the k-step loop is latency-bound otherwise)
  const bf16* er = E + ((size_t)b * Q + (q < Q ? q : 0)) * KC + 8 * hh;
  const bf16* fr = Fhl + ((size_t)b * N + (n < N ? n : 0)) * 2 * KC + 8 * hh;
  f32x16_t acc;
  zero16(acc);
  constexpr int KB = KC / 16 < 8 ? KC / 16 : 8;
#pragma unroll
  for (int k0 = 0; k0 < KC / 16; k0 += KB) {
    bf16x8_t a[KB], fh[KB], fl[KB];
#pragma unroll
    for (int j = 0; j < KB; ++j) {
      a[j] = *reinterpret_cast<const bf16x8_t*>(er + 16 * (k0 + j));
      fh[j] = *reinterpret_cast<const bf16x8_t*>(fr + 16 * (k0 + j));
      fl[j] = *reinterpret_cast<const bf16x8_t*>(fr + KC + 16 * (k0 + j));
    }
#pragma unroll
    for (int j = 0; j < KB; ++j) {
      acc = mfma16(fh[j], a[j], acc);        // rows = keys, column = query (S^T layout)
      acc = mfma16(fl[j], a[j], acc);
    }
  }
  // acc[i] = the logit of query q (this lane's column) at key kt*32 + crow(i, hh): each
  // lane packs its 16 keys' bits, the other lane half holds the other 16 keys
  unsigned bits = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float sg = 1.f / (1.f + expf(-acc[i]));
    if (sg < 0.5f && kt * 32 + crow(i, hh) < N) bits |= 1u << crow(i, hh);
  }
  // the two lane halves hold disjoint key sets of the same query: OR them
  bits |= __shfl_xor((int)bits, 32, 64);
  if (hh == 0 && q < Q) words[((size_t)b * Q + q) * nwords + kt] = bits;
}

// a row blocked at every key is written un-blocked (all-zero), as vs_attn_bitmask
__global__ void __launch_bounds__(256) bitmask_row_fix_kernel(uint32_t* __restrict__ words, int rows, int nkeys,
                                                              int nwords) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  uint32_t* w = words + (size_t)row * nwords;
  const uint32_t lastmask = (nkeys & 31) ? ((1u << (nkeys & 31)) - 1u) : 0xffffffffu;
  bool full = true;
  for (int i = lane; i < nwords; i += 64) full = full && (w[i] == (i == nwords - 1 ? lastmask : 0xffffffffu));
  if (__all(full))
    for (int i = lane; i < nwords; i += 64) w[i] = 0u;
}

struct CostPlan {
  int NCG, PS, tiles_per, KT;
};

CostPlan cost_plan(int S, int B, int Q, int P, int Kc) {
  CostPlan pl;
  pl.NCG = (S * Q + kCols - 1) / kCols;
  const int ntiles = (P + 31) / 32;
  int ps = 512 / (B * pl.NCG);
  if (ps < 1) ps = 1;
  if (ps > ntiles) ps = ntiles;
  pl.tiles_per = (ntiles + ps - 1) / ps;
  pl.PS = (ntiles + pl.tiles_per - 1) / pl.tiles_per;
  pl.KT = Kc <= 4 ? 4 : Kc <= 8 ? 8 : 16;
  return pl;
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" int vs_feature_resize_hilo(const void* features, void* out, int batch, int height, int width,
                                      int channels, int target_h, int target_w, void* stream) {
  VS_CHECK(features && out, "null pointer");
  VS_CHECK(batch > 0 && height > 0 && width > 0 && target_h > 0 && target_w > 0, "bad sizes");
  VS_CHECK(channels > 0 && channels % 8 == 0, "channels must be a positive multiple of 8");
  VS_CHECK(((uintptr_t)features & 15) == 0 && ((uintptr_t)out & 15) == 0, "16-B aligned buffers required");
  const long long work = (long long)batch * target_h * target_w * (channels / 8);
  hipLaunchKernelGGL(feat_resize_hilo_kernel, dim3(grid_for(work, 256, 8192)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)features, (bf16*)out, batch, height, width, channels, target_h, target_w);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_feature_sample_hilo(const void* features, const float* grid, void* out, int batch, int height,
                                      int width, int channels, int num_points, void* stream) {
  VS_CHECK(features && grid && out, "null pointer");
  VS_CHECK(batch > 0 && height > 0 && width > 0 && num_points > 0, "bad sizes");
  VS_CHECK(channels > 0 && channels % 8 == 0, "channels must be a positive multiple of 8");
  VS_CHECK(((uintptr_t)features & 15) == 0 && ((uintptr_t)out & 15) == 0 && ((uintptr_t)grid & 7) == 0,
           "aligned buffers required (features / out 16 B, grid 8 B)");
  const long long work = (long long)batch * num_points * (channels / 8);
  hipLaunchKernelGGL(feat_sample_hilo_kernel, dim3(grid_for(work, 256, 8192)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)features, grid, (bf16*)out, batch, height, width, channels, num_points);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" long long vs_match_cost_factors_workspace_bytes(int num_steps, int batch, int num_queries,
                                                           int num_points, int max_targets) {
  if (num_steps <= 0 || batch <= 0 || num_queries <= 0 || num_points <= 0 || max_targets <= 0) return 0;
  const CostPlan pl = cost_plan(num_steps, batch, num_queries, num_points, max_targets);
  const long long part = (long long)batch * pl.PS * (2 + 2 * pl.KT) * pl.NCG * kCols;
  const long long tpart = (long long)batch * pl.PS * pl.KT;
  return (part + tpart) * 4 + 16;
}

extern "C" int vs_match_cost_factors(const void* mask_embed, const void* point_features, int num_steps,
                                     const float* class_probs, int num_classes_plus1, const long long* target_classes,
                                     const float* target_point_labels, float* cost, void* workspace, int batch,
                                     int num_queries, int channels, int num_points, int max_targets,
                                     float mask_weight, float class_weight, float dice_weight, void* stream) {
  VS_CHECK(mask_embed && point_features && class_probs && target_classes && target_point_labels && cost && workspace,
           "null pointer");
  VS_CHECK(num_steps >= 1 && batch > 0 && num_queries > 0 && num_points > 0 && num_classes_plus1 > 0, "bad sizes");
  VS_CHECK(max_targets >= 1 && max_targets <= 16, "1 <= padded targets <= 16");
  VS_CHECK(channels == 64 || channels == 128 || channels == 256, "channels must be 64, 128 or 256");
  VS_CHECK((long long)num_steps * num_queries < (1LL << 24), "too many (step, query) columns");
  VS_CHECK(((uintptr_t)mask_embed & 15) == 0 && ((uintptr_t)point_features & 15) == 0 &&
               ((uintptr_t)target_point_labels & 3) == 0 && ((uintptr_t)workspace & 15) == 0,
           "aligned buffers required");
  const CostPlan pl = cost_plan(num_steps, batch, num_queries, num_points, max_targets);
  float* part = (float*)workspace;
  float* tpart = part + (size_t)batch * pl.PS * (2 + 2 * pl.KT) * pl.NCG * kCols;
  hipStream_t st = (hipStream_t)stream;
  const int wgs = batch * pl.PS * pl.NCG;
#define VS_MCF(KC_, KT_)                                                                                       \
  hipLaunchKernelGGL((match_cost_fac_kernel<KC_, KT_>), dim3(wgs), dim3(64 * kCostWaves), 0, st,                \
                     (const bf16*)mask_embed, (const bf16*)point_features, target_point_labels, part, tpart,    \
                     num_steps, batch, num_queries, num_points, max_targets, pl.NCG, pl.PS, pl.tiles_per)
#define VS_MCF_KT(KC_)            \
  if (pl.KT == 4)                 \
    VS_MCF(KC_, 4);               \
  else if (pl.KT == 8)            \
    VS_MCF(KC_, 8);               \
  else                            \
    VS_MCF(KC_, 16);
  if (channels == 256) {
    VS_MCF_KT(256)
  } else if (channels == 128) {
    VS_MCF_KT(128)
  } else {
    VS_MCF_KT(64)
  }
#undef VS_MCF_KT
#undef VS_MCF
  VS_LAUNCH_CHECK();
  const dim3 fg((num_steps * num_queries + 63) / 64, batch);
#define VS_FIN(KT_)                                                                                               \
  hipLaunchKernelGGL((match_cost_fac_fin_kernel<KT_>), fg, dim3(256), 0, st, part, tpart, class_probs,            \
                     num_classes_plus1, target_classes, cost, num_steps, batch, num_queries, num_points, max_targets, \
                     pl.NCG, pl.PS, mask_weight, class_weight, dice_weight)
  if (pl.KT == 4)
    VS_FIN(4);
  else if (pl.KT == 8)
    VS_FIN(8);
  else
    VS_FIN(16);
#undef VS_FIN
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_level_bitmask_hilo(const void* mask_embed, const void* level_features, uint32_t* words, int batch,
                                     int num_queries, int channels, int height, int width, void* stream) {
  VS_CHECK(mask_embed && level_features && words, "null pointer");
  VS_CHECK(batch > 0 && num_queries > 0 && height > 0 && width > 0, "bad sizes");
  VS_CHECK(channels == 64 || channels == 128 || channels == 256, "channels must be 64, 128 or 256");
  VS_CHECK(((uintptr_t)mask_embed & 15) == 0 && ((uintptr_t)level_features & 15) == 0, "16-B aligned buffers");
  const int N = height * width, nwords = (N + 31) / 32;
  const int qgroups = (num_queries + 127) / 128;
  const long long wgs = (long long)batch * nwords * qgroups;
  VS_CHECK(wgs < (1LL << 31), "too many tiles");
  hipStream_t st = (hipStream_t)stream;
#define VS_LB(KC_)                                                                                           \
  hipLaunchKernelGGL((level_bitmask_kernel<KC_>), dim3((unsigned)wgs), dim3(256), 0, st, (const bf16*)mask_embed, \
                     (const bf16*)level_features, words, batch, num_queries, N, nwords, qgroups, nwords)
  if (channels == 256)
    VS_LB(256);
  else if (channels == 128)
    VS_LB(128);
  else
    VS_LB(64);
#undef VS_LB
  VS_LAUNCH_CHECK();
  const int rows = batch * num_queries;
  hipLaunchKernelGGL(bitmask_row_fix_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, words, rows, N, nwords);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
