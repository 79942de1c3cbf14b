// Batched linear-sum assignment (Hungarian matching) on the device.
//
// Reference: the Mask2Former / MaskDINO HungarianMatcher runs
// scipy.optimize.linear_sum_assignment(cost.cpu()) per image and decoder layer
// (HF:m2f:489-491; upstream matcher.py), i.e. one device->host sync per training step and
// CPU work while the GPU idles.  Here every (decoder step, image) problem is solved by
// one wave64: a cost matrix of Q queries x K targets (K <= Q), each target assigned to a
// distinct query minimising the total cost — the same optimum scipy returns (unique for
// generic real costs; on exact ties either optimal assignment may be returned).
//
// Algorithm: shortest augmenting paths with dual potentials (Kuhn-Munkres in the
// O(K^2 Q) form).  Rows = targets (added one by one), columns = queries.  Each Dijkstra
// step relaxes all unvisited columns in parallel (a lane owns columns lane+1, lane+65,
// ...), picks the minimum slack with a wave arg-min (lowest column on ties), and updates
// the potentials; the augmentation walk is done by lane 0.  Potentials and slacks are
// f64; the K x Q cost slice is staged transposed in LDS (target-major, so a relaxation
// step reads consecutive queries).
#include "common.h"

#include <cfloat>

namespace vs {
namespace {

constexpr int kMaxQ = 1024;
constexpr int kMaxCols = 64;          // images per launch (per-image target counts by value)

struct ColCounts {
  int k[kMaxCols];
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// cost [S*B][Q][Kmax] f32 -> assign [S*B][Kmax] int32 (query of target k, -1 padding).
// Per-image target counts by value (cc) or, when dcounts is set, read from device memory
// (clamped to [0, Kmax]): a graph-replayed step then serves any counts up to Kmax.
__global__ void __launch_bounds__(64) lsa_kernel(const float* __restrict__ cost, int* __restrict__ assign, int B,
                                                 int Q, int Kmax, ColCounts cc, const int* __restrict__ dcounts) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int prob = blockIdx.x;
  const int K = dcounts ? min(max(dcounts[prob % B], 0), min(Kmax, Q)) : cc.k[prob % B];
  const int lane = threadIdx.x;
  int* out = assign + (size_t)prob * Kmax;
  for (int k = lane; k < Kmax; k += 64) out[k] = -1;
  if (K == 0) return;
  // LDS: a[K][Q] f32 | u[K+1] f64 | v[Q+1] f64 | minv[Q+1] f64 | p[Q+1] int | way[Q+1] int | used[Q+1] u8
  float* a = reinterpret_cast<float*>(smem);
  double* u = reinterpret_cast<double*>(smem + (((size_t)K * Q * 4 + 7) & ~(size_t)7));
  double* v = u + (K + 1);
  double* minv = v + (Q + 1);
  int* p = reinterpret_cast<int*>(minv + (Q + 1));
  int* way = p + (Q + 1);
  unsigned char* used = reinterpret_cast<unsigned char*>(way + (Q + 1));

  const float* c = cost + (size_t)prob * Q * Kmax;
  for (int idx = lane; idx < Q * K; idx += 64) {       // transpose to target-major
    const int q = idx / K, k = idx % K;
    a[k * Q + q] = c[(size_t)q * Kmax + k];
  }
  for (int j = lane; j <= Q; j += 64) {
    v[j] = 0.0;
    p[j] = 0;
    way[j] = 0;
  }
  for (int i = lane; i <= K; i += 64) u[i] = 0.0;
  wave_sync();

  for (int i = 1; i <= K; ++i) {
    if (lane == 0) p[0] = i;
    for (int j = lane; j <= Q; j += 64) {
      minv[j] = DBL_MAX;
      used[j] = 0;
    }
    wave_sync();
    int j0 = 0;
    while (true) {
      if (lane == 0) used[j0] = 1;
      wave_sync();
      const int i0 = p[j0];
      const double ui0 = u[i0];
      const float* arow = a + (size_t)(i0 - 1) * Q;
      double best = DBL_MAX;
      int bj = 0x7fffffff;
      for (int j = lane + 1; j <= Q; j += 64) {
        if (!used[j]) {
          const double cur = (double)arow[j - 1] - ui0 - v[j];
          if (cur < minv[j]) {
            minv[j] = cur;
            way[j] = j0;
          }
          if (minv[j] < best || (minv[j] == best && j < bj)) {
            best = minv[j];
            bj = j;
          }
        }
      }
      // wave arg-min (value, then lowest column)
      for (int s = 32; s >= 1; s >>= 1) {
        const double ob = __shfl_xor(best, s, 64);
        const int oj = __shfl_xor(bj, s, 64);
        if (ob < best || (ob == best && oj < bj)) {
          best = ob;
          bj = oj;
        }
      }
      const double delta = best;
      const int j1 = bj;
      wave_sync();
      for (int j = lane; j <= Q; j += 64) {
        if (used[j]) {
          u[p[j]] += delta;
          v[j] -= delta;
        } else {
          minv[j] -= delta;
        }
      }
      wave_sync();
      j0 = j1;
      if (p[j0] == 0) break;
    }
    if (lane == 0) {                                   // augment along the path
      while (j0) {
        const int j1 = way[j0];
        p[j0] = p[j1];
        j0 = j1;
      }
    }
    wave_sync();
  }
  for (int j = lane + 1; j <= Q; j += 64)
    if (p[j] != 0) out[p[j] - 1] = j - 1;
}

size_t lsa_lds_bytes(int K, int Q) {
  return (((size_t)K * Q * 4 + 7) & ~(size_t)7) + (size_t)(K + 1) * 8 + (size_t)(Q + 1) * (8 + 8 + 4 + 4 + 1);
}

// ---------------------------------------------------------------------------------
// Matcher cost matrix (HungarianMatcher, HF:m2f:413-481) for all decoder steps at once.
// For every (step s, image b, query q) one wave walks the image's P uniform points:
//   v      = bilinear sample of mask logits[s][b, q] at the point (grid_sample,
//            align_corners=False, zero padding -- the same arithmetic as ATen's kernel)
//   A_k   += softplus(-v) t_k + softplus(v) (1 - t_k)      (pair-wise sigmoid BCE, :350-374)
//   N_k   += sigmoid(v) t_k ;  Ssg += sigmoid(v) ;  T_k += t_k   (dice, :328-347)
// with t_k = the target point labels [B, Kc, P] (sampled once by the caller), then
//   cost[s,b,q,k] = wm A_k / P + wc (-prob[s,b,q,cls_k]) + wd (1 - (2 N_k + 1) / (Ssg + T_k + 1))
// clamped to +-1e10 and NaN -> 0 as the reference.  Replaces S grid_sample launches over
// the [B, Q, H, W] logit maps (one thread per point looping over the Q channels: 100
// strided reads per thread) and the pos/neg/sigmoid matmuls with K = P.
constexpr int kMaxSteps = 16;
constexpr int kMaxKc = 16;

struct MaskPtrs {
  const float* p[kMaxSteps];
};

__device__ __forceinline__ float softplus_f(float x) { return x > 20.f ? x : log1pf(expf(x)); }

// One workgroup per (s, b, q); its 4 waves take contiguous quarters of the points (the
// caller orders the points by pixel row, so a wave's taps share cache lines and every
// logit map streams through L2 about once) and combine their sums through LDS.
template <int KC>
__global__ void __launch_bounds__(256) match_cost_kernel(MaskPtrs masks, const float* __restrict__ probs, int C1,
                                                         const long long* __restrict__ tcls,
                                                         const float* __restrict__ grid, const float* __restrict__ tp,
                                                         float* __restrict__ cost, int S, int B, int Q, int H, int W,
                                                         int P, int Kc, float wm, float wc, float wd) {
  __shared__ float red[4][3 * KC + 1];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long item = blockIdx.x;                              // (s, b, q)
  const int q = (int)(item % Q);
  const int b = (int)((item / Q) % B);
  const int s = (int)(item / ((long long)Q * B));
  const float* map = masks.p[s] + ((size_t)b * Q + q) * H * W;
  const float* g2 = grid + (size_t)b * P * 2;
  const float* tb = tp + (size_t)b * Kc * P;
  float A[KC], N[KC], T[KC], ssg = 0.f;
#pragma unroll
  for (int k = 0; k < KC; ++k) A[k] = N[k] = T[k] = 0.f;
  const int per = (P + 3) / 4;
  const int p0 = wave * per, p1 = min(P, p0 + per);
  for (int p = p0 + lane; p < p1; p += 64) {
    const float2 gxy = *reinterpret_cast<const float2*>(g2 + 2 * p);
    // ATen grid_sampler_compute_source_index (zeros padding, align_corners=False)
    const float ix = ((gxy.x + 1.f) * W - 1.f) / 2.f;
    const float iy = ((gxy.y + 1.f) * H - 1.f) / 2.f;
    const float ix_nw = floorf(ix), iy_nw = floorf(iy);
    const float ix_ne = ix_nw + 1.f, iy_ne = iy_nw;
    const float ix_sw = ix_nw, iy_sw = iy_nw + 1.f;
    const float ix_se = ix_nw + 1.f, iy_se = iy_nw + 1.f;
    const float nw = (ix_se - ix) * (iy_se - iy);
    const float ne = (ix - ix_sw) * (iy_sw - iy);
    const float sw = (ix_ne - ix) * (iy - iy_ne);
    const float se = (ix - ix_nw) * (iy - iy_nw);
    const int x0 = (int)ix_nw, y0 = (int)iy_nw;
    float v = 0.f;
    const bool xin0 = x0 >= 0 && x0 < W, xin1 = x0 + 1 >= 0 && x0 + 1 < W;
    const bool yin0 = y0 >= 0 && y0 < H, yin1 = y0 + 1 >= 0 && y0 + 1 < H;
    if (yin0 && xin0) v += map[(size_t)y0 * W + x0] * nw;
    if (yin0 && xin1) v += map[(size_t)y0 * W + x0 + 1] * ne;
    if (yin1 && xin0) v += map[(size_t)(y0 + 1) * W + x0] * sw;
    if (yin1 && xin1) v += map[(size_t)(y0 + 1) * W + x0 + 1] * se;
    const float pos = softplus_f(-v), neg = softplus_f(v);
    const float sg = 1.f / (1.f + expf(-v));
    ssg += sg;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      if (k < Kc) {
        const float t = tb[(size_t)k * P + p];
        A[k] += pos * t + neg * (1.f - t);
        N[k] += sg * t;
        T[k] += t;
      }
    }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    ssg += __shfl_xor(ssg, o, 64);
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      A[k] += __shfl_xor(A[k], o, 64);
      N[k] += __shfl_xor(N[k], o, 64);
      T[k] += __shfl_xor(T[k], o, 64);
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      red[wave][k] = A[k];
      red[wave][KC + k] = N[k];
      red[wave][2 * KC + k] = T[k];
    }
    red[wave][3 * KC] = ssg;
  }
  __syncthreads();
  if (threadIdx.x < Kc) {
    const int k = threadIdx.x;
    const float a = (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]);
    const float n = (red[0][KC + k] + red[1][KC + k]) + (red[2][KC + k] + red[3][KC + k]);
    const float t = (red[0][2 * KC + k] + red[1][2 * KC + k]) + (red[2][2 * KC + k] + red[3][2 * KC + k]);
    const float sgt = (red[0][3 * KC] + red[1][3 * KC]) + (red[2][3 * KC] + red[3][3 * KC]);
    const long long cls = tcls[(size_t)b * Kc + k];
    const float prob = probs[(((size_t)s * B + b) * Q + q) * C1 + (int)cls];
    const float cm = a / (float)P;
    const float cd = 1.f - (2.f * n + 1.f) / (sgt + t + 1.f);
    float cst = wm * cm + wc * (-prob) + wd * cd;
    cst = fminf(fmaxf(cst, -1e10f), 1e10f);
    if (cst != cst) cst = 0.f;
    cost[(((size_t)s * B + b) * Q + q) * Kc + k] = cst;
  }
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" int vs_lsa_max_targets(int num_queries) {
  if (num_queries <= 0 || num_queries > kMaxQ) return 0;
  int k = num_queries;
  while (k > 0 && lsa_lds_bytes(k, num_queries) > 64 * 1024) --k;
  return k;
}

extern "C" int vs_lsa_batch(const float* cost, const int* targets_per_image, int num_steps, int batch,
                            int num_queries, int max_targets, int* assign, void* stream) {
  VS_CHECK(num_steps >= 0 && batch > 0 && batch <= kMaxCols, "1 <= batch <= 64");
  VS_CHECK(num_queries > 0 && num_queries <= kMaxQ, "1 <= queries <= 1024");
  VS_CHECK(max_targets > 0, "max_targets must be positive");
  VS_CHECK(cost && targets_per_image && assign, "null pointer");
  ColCounts cc;
  int kmax_used = 0;
  for (int b = 0; b < batch; ++b) {
    cc.k[b] = targets_per_image[b];
    VS_CHECK(cc.k[b] >= 0 && cc.k[b] <= max_targets, "targets per image out of range");
    VS_CHECK(cc.k[b] <= num_queries, "more targets than queries");
    kmax_used = max(kmax_used, cc.k[b]);
  }
  const size_t lds = lsa_lds_bytes(kmax_used, num_queries);
  VS_CHECK(lds <= 64 * 1024, "cost matrix too large for the device matcher (see vs_lsa_max_targets)");
  if (num_steps == 0) return VS_OK;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(lsa_kernel, dim3(num_steps * batch), dim3(64), lds, st, cost, assign, batch, num_queries,
                     max_targets, cc, (const int*)nullptr);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_lsa_batch_device_counts(const float* cost, const int* targets_per_image_dev, int num_steps,
                                          int batch, int num_queries, int max_targets, int* assign, void* stream) {
  VS_CHECK(num_steps >= 0 && batch > 0, "batch must be positive");
  VS_CHECK(num_queries > 0 && num_queries <= kMaxQ, "1 <= queries <= 1024");
  VS_CHECK(max_targets > 0 && max_targets <= num_queries, "1 <= max_targets <= queries");
  VS_CHECK(cost && targets_per_image_dev && assign, "null pointer");
  const size_t lds = lsa_lds_bytes(max_targets, num_queries);
  VS_CHECK(lds <= 64 * 1024, "cost matrix too large for the device matcher (see vs_lsa_max_targets)");
  if (num_steps == 0) return VS_OK;
  ColCounts cc = {};
  hipLaunchKernelGGL(lsa_kernel, dim3(num_steps * batch), dim3(64), lds, (hipStream_t)stream, cost, assign, batch,
                     num_queries, max_targets, cc, targets_per_image_dev);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_match_cost(const float* const* mask_logits, int num_steps, const float* class_probs,
                             int num_classes_plus1, const long long* target_classes, const float* points,
                             const float* target_point_labels, float* cost, int batch, int num_queries, int height,
                             int width, int num_points, int max_targets, float mask_weight, float class_weight,
                             float dice_weight, void* stream) {
  VS_CHECK(num_steps >= 1 && num_steps <= kMaxSteps, "1 <= decoder steps <= 16");
  VS_CHECK(max_targets >= 1 && max_targets <= kMaxKc, "1 <= padded targets <= 16");
  VS_CHECK(batch > 0 && num_queries > 0 && height > 0 && width > 0 && num_points > 0 && num_classes_plus1 > 0,
           "bad sizes");
  VS_CHECK(mask_logits && class_probs && target_classes && points && target_point_labels && cost, "null pointer");
  MaskPtrs mp = {};
  for (int s = 0; s < num_steps; ++s) {
    VS_CHECK(mask_logits[s], "null mask-logit pointer");
    mp.p[s] = mask_logits[s];
  }
  const long long items = (long long)num_steps * batch * num_queries;
  VS_CHECK(items < (1LL << 31), "too many (step, image, query) items");
  const int grid = (int)items;
  hipStream_t st = (hipStream_t)stream;
#define VS_MC(KC_)                                                                                            \
  hipLaunchKernelGGL(match_cost_kernel<KC_>, dim3(grid), dim3(256), 0, st, mp, class_probs, num_classes_plus1, \
                     target_classes, points, target_point_labels, cost, num_steps, batch, num_queries, height,   \
                     width, num_points, max_targets, mask_weight, class_weight, dice_weight)
  if (max_targets <= 4)
    VS_MC(4);
  else if (max_targets <= 8)
    VS_MC(8);
  else
    VS_MC(16);
#undef VS_MC
  VS_LAUNCH_CHECK();
  return VS_OK;
}
