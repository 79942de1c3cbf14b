// Row-wise top-k selection for the mask losses' importance sampling (point_sample uncertainty,
// HF:m2f:689-724 `sample_points_using_uncertainty`: the k most uncertain of the oversampled
// points per (prediction, target) pair; MaskDINO C4: 4000 rows of 37 632 values, k = 9 408
// per decoder step).  torch.topk runs a segmented radix sort / multi-block digit passes for
// these shapes (~6.6 ms per C4 step); here one workgroup per row selects the k largest by
// RADIX SELECT and writes their indices, no sort:
//   * values -> order-preserving u32 keys (larger float <=> larger key; -0 < +0);
//   * 4 passes of 8 bits, most significant first: an LDS histogram (integer LDS atomics)
//     of the digit among the keys that match the prefix found so far, then the bin holding
//     the k-th largest -> the exact k-th largest key T and how many keys equal to T the
//     selection needs (the rest of the k are > T);
//   * one compaction pass in index order: every key > T, and the first `need` keys == T;
//     positions by wave ballots + a block prefix in LDS, so the output is the selected
//     indices in ascending order (deterministic; the same SET as torch.topk when the values
//     at the threshold are distinct, the lowest indices among ties otherwise).
// Values are read from L2 after the first pass (a 37 632-value row is 147 KB).
#include "common.h"

namespace vs {
namespace {

__device__ __forceinline__ unsigned order_key(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

constexpr int kTkThreads = 256;

__global__ void __launch_bounds__(kTkThreads) topk_rows_kernel(const float* __restrict__ x,
                                                               long long* __restrict__ idx, int n, int k) {
  __shared__ unsigned hist[256];
  __shared__ unsigned s_prefix, s_need, s_base;
  __shared__ unsigned wcnt[kTkThreads / 64][2];
  const float* row = x + (size_t)blockIdx.x * n;
  long long* out = idx + (size_t)blockIdx.x * k;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  unsigned prefix = 0, pmask = 0;              // the key bits fixed so far, and their mask
  unsigned need = (unsigned)k;                 // how many of the keys matching the prefix are still wanted
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    hist[tid] = 0u;
    __syncthreads();
    for (int i = tid; i < n; i += kTkThreads) {
      const unsigned key = order_key(row[i]);
      if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 0xffu], 1u);
    }
    __syncthreads();
    if (tid == 0) {                            // the bin of the need-th largest, from the top
      unsigned cum = 0;
      int b = 255;
      for (; b > 0; --b) {
        if (cum + hist[b] >= need) break;
        cum += hist[b];
      }
      s_prefix = prefix | ((unsigned)b << shift);
      s_need = need - cum;                     // wanted among the keys of bin b
    }
    __syncthreads();
    prefix = s_prefix;
    need = s_need;
    pmask |= 0xffu << shift;
    __syncthreads();                           // hist / s_* reused next pass
  }
  // prefix = T, the k-th largest key; `need` keys equal to T complete the selection
  const unsigned T = prefix;
  if (tid == 0) s_base = 0u;
  unsigned eq_seen = 0;                        // keys == T met so far (block-wide, uniform)
  __syncthreads();
  for (int c0 = 0; c0 < n; c0 += kTkThreads) {
    const int i = c0 + tid;
    const unsigned key = i < n ? order_key(row[i]) : 0u;
    const bool gt = i < n && key > T, eq = i < n && key == T;
    const unsigned long long bg = __ballot(gt), be = __ballot(eq);
    if (lane == 0) {
      wcnt[wave][0] = (unsigned)__popcll(bg);
      wcnt[wave][1] = (unsigned)__popcll(be);
    }
    __syncthreads();
    unsigned gt_before = 0, eq_before = 0, eq_tot = 0, gt_tot = 0;
#pragma unroll
    for (int w = 0; w < kTkThreads / 64; ++w) {
      if (w < wave) {
        gt_before += wcnt[w][0];
        eq_before += wcnt[w][1];
      }
      gt_tot += wcnt[w][0];
      eq_tot += wcnt[w][1];
    }
    const unsigned long long lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;
    const unsigned my_gt = gt_before + (unsigned)__popcll(bg & lt_mask);
    const unsigned my_eq = eq_before + (unsigned)__popcll(be & lt_mask);
    // equal keys past the `need`-th are not selected; the output position counts the
    // selected elements before this one in index order
    const unsigned eq_taken_before = min(eq_seen + my_eq, need) - min(eq_seen, need);
    const unsigned base = s_base;
    const bool take = gt || (eq && eq_seen + my_eq < need);
    if (take) out[base + my_gt + eq_taken_before] = i;
    const unsigned eq_taken_chunk = min(eq_seen + eq_tot, need) - min(eq_seen, need);
    eq_seen += eq_tot;
    __syncthreads();                           // every thread read s_base / wcnt
    if (tid == 0) s_base = base + gt_tot + eq_taken_chunk;
    __syncthreads();
  }
}

// LDS-resident variant for rows of up to kTkLdsKeys values (C2-C5: 3 x 112^2 = 37 632): the
// row is read from HBM ONCE, as keys, into LDS (a single workgroup may hold 160 KiB on
// gfx950), and the four digit passes and the compaction run over LDS -- the global variant
// re-reads every row five times, and with 8 rows of 147 KB in flight per CU the passes miss
// L2 and go back to HBM.  16 waves per row; the first pass (where most keys share a digit:
// uncertainties are -|logit|, a few binades) adds wave-aggregated counts, one LDS atomic
// per distinct digit in the wave, instead of 64 conflicting ones.
constexpr int kTkLdsThreads = 1024;
constexpr int kTkLdsKeys = 39424;              // 154 KiB of keys + the histogram and scan words

__global__ void __launch_bounds__(kTkLdsThreads) topk_rows_lds_kernel(const float* __restrict__ x,
                                                                      long long* __restrict__ idx, int n, int k) {
  __shared__ __attribute__((aligned(16))) unsigned keys[kTkLdsKeys];
  __shared__ unsigned hist[256];
  __shared__ unsigned s_prefix, s_need;
  __shared__ unsigned wcnt[kTkLdsThreads / 64];
  const float* row = x + (size_t)blockIdx.x * n;
  long long* out = idx + (size_t)blockIdx.x * k;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if ((n & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {   // rows 16-byte aligned: float4 loads
    // every load of the row issued before the first LDS store (one HBM round trip, not 10)
    constexpr int kIt = (kTkLdsKeys / 4 + kTkLdsThreads - 1) / kTkLdsThreads;
    const float4* r4 = reinterpret_cast<const float4*>(row);
    const int n4 = n >> 2;
    float4 buf[kIt];
#pragma unroll
    for (int u = 0; u < kIt; ++u) {
      const int i = tid + u * kTkLdsThreads;
      buf[u] = i < n4 ? r4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < kIt; ++u) {
      const int i = tid + u * kTkLdsThreads;
      if (i < n4)
        *reinterpret_cast<uint4*>(keys + 4 * i) =
            make_uint4(order_key(buf[u].x), order_key(buf[u].y), order_key(buf[u].z), order_key(buf[u].w));
    }
  } else {
    for (int i = tid; i < n; i += kTkLdsThreads) keys[i] = order_key(row[i]);
  }
  unsigned prefix = 0, pmask = 0, need = (unsigned)k;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    if (tid < 256) hist[tid] = 0u;
    __syncthreads();                           // keys loaded / hist cleared
    if (pass == 0) {
      for (int c0 = 0; c0 < n; c0 += kTkLdsThreads) {
        const int i = c0 + tid;
        bool act = i < n;
        const unsigned bin = act ? keys[i] >> 24 : 0u;
        for (;;) {
          const unsigned long long m = __ballot(act);
          if (!m) break;
          const int leader = __ffsll((long long)m) - 1;
          const unsigned lb = __shfl((int)bin, leader);
          const bool same = act && bin == lb;
          const unsigned long long sm = __ballot(same);
          if (lane == leader) atomicAdd(&hist[lb], (unsigned)__popcll(sm));
          act = act && !same;
        }
      }
    } else {
      for (int i = tid; i < n; i += kTkLdsThreads) {
        const unsigned key = keys[i];
        if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 0xffu], 1u);
      }
    }
    __syncthreads();
    if (wave == 0) {                           // the bin of the need-th largest: a wave scan from the top
      // lane l holds bins 255-4l .. 252-4l (descending)
      unsigned h[4], s = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        h[j] = hist[255 - 4 * lane - j];
        s += h[j];
      }
      unsigned incl = s;                       // inclusive prefix over lanes (bins above come first)
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const unsigned t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
      }
      const unsigned excl = incl - s;
      // the lane whose range crosses `need` (exactly one: the total is >= need)
      if (excl < need && incl >= need) {
        unsigned cum = excl;
        int j = 0;
        for (; j < 3; ++j) {
          if (cum + h[j] >= need) break;
          cum += h[j];
        }
        s_prefix = prefix | ((unsigned)(255 - 4 * lane - j) << shift);
        s_need = need - cum;
      }
    }
    __syncthreads();
    prefix = s_prefix;
    need = s_need;
    pmask |= 0xffu << shift;
  }
  // compaction: thread t owns the keys [t E, (t + 1) E), E = ceil(n / 1024) (37 at
  // n = 37 632: an odd stride between lanes, no bank conflicts); its counts of keys > T and
  // == T, one block scan, then each thread writes its selections in index order -- one
  // barrier, where a 1024-key round per barrier pair took 37 rounds
  const unsigned T = prefix;
  const int E = (n + kTkLdsThreads - 1) / kTkLdsThreads;
  const int b0 = min(tid * E, n), b1 = min(b0 + E, n);
  unsigned cnt = 0;                            // (keys > T) | (keys == T) << 16; each < 2^16
  for (int i = b0; i < b1; ++i) {
    const unsigned key = keys[i];
    cnt += (key > T ? 1u : 0u) + (key == T ? 0x10000u : 0u);
  }
  unsigned incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned t = __shfl_up(incl, d);
    if (lane >= d) incl += t;
  }
  if (lane == 63) wcnt[wave] = incl;
  __syncthreads();
  unsigned before = incl - cnt;
  for (int w = 0; w < wave; ++w) before += wcnt[w];
  unsigned gb = before & 0xffffu, eb = before >> 16;
  for (int i = b0; i < b1; ++i) {
    const unsigned key = keys[i];
    if (key > T) {
      out[gb + min(eb, need)] = i;
      ++gb;
    } else if (key == T) {
      if (eb < need) out[gb + eb] = i;
      ++eb;
    }
  }
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" int vs_topk_rows(const float* values, long long* indices, int rows, int n, int k, void* stream) {
  VS_CHECK(rows >= 0 && n > 0 && k > 0 && k <= n, "need 0 < k <= n");
  if (rows == 0) return VS_OK;
  VS_CHECK(values && indices, "null pointer");
  if (n <= kTkLdsKeys)
    hipLaunchKernelGGL(topk_rows_lds_kernel, dim3(rows), dim3(kTkLdsThreads), 0, (hipStream_t)stream, values,
                       indices, n, k);
  else
    hipLaunchKernelGGL(topk_rows_kernel, dim3(rows), dim3(kTkThreads), 0, (hipStream_t)stream, values, indices, n, k);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
