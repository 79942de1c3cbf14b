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
