// MSDeformAttn prologue (HF:m2f:994-1002; upstream MSDeformAttn.forward in the
// reference's un-vendored MaskDINO/Mask2Former pixel decoder): from the two token-major
// projections of the query,
//   sampling_locations[b,q,h,l,p,:] = ref[b,q,l,:] + offsets[b,q,h,l,p,:] / (W_l, H_l)
//   attention_weights[b,q,h,:]      = softmax(logits[b,q,h,:])   (over L*P, in f32)
// and the adjoint.  The torch composition is a cast, a divide, an add, a cast and a
// softmax forward (five HBM passes over f32 tensors) and as many backward kernels; here
// one launch each way reads / writes each element once.
//   forward:  f32 outputs, the projections in their dtype (bf16 / f32) upcast exactly
//   backward: grad_offsets = grad_loc / (W_l, H_l), grad_logits = a * (g - <g, a>),
//             rounded to the projections' dtype (as the cast's backward)
#include "common.h"

namespace vs {
namespace {

constexpr int kMaxLP = 32;       // levels x points per head

struct PrepGeom {
  float w[4], h[4];              // level width / height as f32 (the HF `normalizer`)
};

// A block owns kGroups consecutive (b, q, head) groups.  Every global access is
// coalesced: the elementwise location / offset-gradient part walks the block's
// elements in memory order (a group's L*P*2 offsets are contiguous within a projection
// row), and the softmax part stages the block's logits (and, backward, the weights and
// their gradients) through LDS so that one thread reduces one group.
constexpr int kGroups = 128;     // LDS: 16 KB forward, 32 KB backward at L*P = 32

template <typename T>
__global__ void __launch_bounds__(256) msda_prep_fwd_kernel(const T* __restrict__ off, const T* __restrict__ logit,
                                                            const float* __restrict__ ref, float* __restrict__ loc,
                                                            float* __restrict__ aw, PrepGeom gm, int Q, int Hh,
                                                            int L, int P, long long off_rs, long long logit_rs,
                                                            long long ref_bs, long long groups) {
  __shared__ float sm[kGroups * kMaxLP];
  const int LP = L * P;
  const long long g0 = (long long)blockIdx.x * kGroups;
  const int ng = (int)min((long long)kGroups, groups - g0);
  // locations: element e of the block = (group g0 + e / (2 LP), level-point-xy e % (2 LP))
  const int rowe = Hh * LP * 2;                       // offset elements per projection row
  const long long e0 = g0 * LP * 2;
  const long long bq0 = e0 / rowe;                    // 64-bit divisions once per block
  const int c0 = (int)(e0 - bq0 * rowe);
  const long long b0 = bq0 / Q;
  const int q0 = (int)(bq0 - b0 * Q);
  for (int e = 2 * threadIdx.x; e < ng * LP * 2; e += 512) {     // one (x, y) pair per thread
    const int t = c0 + e;
    const int dr = t / rowe, c = t - dr * rowe;
    const int qq = q0 + dr;
    const int db = qq / Q, q = qq - db * Q;
    const int l = (c >> 1) / P % L;
    const float2 r = *reinterpret_cast<const float2*>(ref + (b0 + db) * ref_bs + ((long long)q * L + l) * 2);
    const T* o = off + (bq0 + dr) * off_rs + c;
    *reinterpret_cast<float2*>(loc + e0 + e) = make_float2(r.x + to_f32(o[0]) / gm.w[l], r.y + to_f32(o[1]) / gm.h[l]);
  }
  // softmax weights
  const int rowl = Hh * LP;
  const long long f0 = g0 * LP;
  const long long lq0 = f0 / rowl;
  const int l0 = (int)(f0 - lq0 * rowl);
  for (int e = threadIdx.x; e < ng * LP; e += 256) {
    const int t = l0 + e;
    const int dr = t / rowl;
    sm[e] = to_f32(logit[(lq0 + dr) * logit_rs + (t - dr * rowl)]);
  }
  __syncthreads();
  if (threadIdx.x < ng) {
    float* v = sm + threadIdx.x * LP;
    float m = -INFINITY;
    for (int i = 0; i < LP; ++i) m = fmaxf(m, v[i]);
    float sum = 0.f;
    for (int i = 0; i < LP; ++i) {
      const float x = expf(v[i] - m);
      v[i] = x;
      sum += x;
    }
    for (int i = 0; i < LP; ++i) v[i] = v[i] / sum;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < ng * LP; e += 256) aw[f0 + e] = sm[e];
}

template <typename T>
__global__ void __launch_bounds__(256) msda_prep_bwd_kernel(const float* __restrict__ gloc,
                                                            const float* __restrict__ gaw,
                                                            const float* __restrict__ aw, T* __restrict__ goff,
                                                            T* __restrict__ glogit, PrepGeom gm, int Hh, int L, int P,
                                                            long long goff_rs, long long glogit_rs, long long groups) {
  __shared__ float sa[kGroups * kMaxLP];
  __shared__ float sg[kGroups * kMaxLP];
  const int LP = L * P;
  const long long g0 = (long long)blockIdx.x * kGroups;
  const int ng = (int)min((long long)kGroups, groups - g0);
  const int rowe = Hh * LP * 2;
  const long long e0 = g0 * LP * 2;
  const long long bq0 = e0 / rowe;
  const int c0 = (int)(e0 - bq0 * rowe);
  for (int e = 2 * threadIdx.x; e < ng * LP * 2; e += 512) {     // one (x, y) pair per thread
    const int t = c0 + e;
    const int dr = t / rowe, c = t - dr * rowe;
    const int l = (c >> 1) / P % L;
    const float2 gv = *reinterpret_cast<const float2*>(gloc + e0 + e);
    T* o = goff + (bq0 + dr) * goff_rs + c;
    o[0] = from_f32<T>(gv.x / gm.w[l]);
    o[1] = from_f32<T>(gv.y / gm.h[l]);
  }
  const long long f0 = g0 * LP;
  for (int e = threadIdx.x; e < ng * LP; e += 256) {
    sa[e] = aw[f0 + e];
    sg[e] = gaw[f0 + e];
  }
  __syncthreads();
  if (threadIdx.x < ng) {
    const float* a = sa + threadIdx.x * LP;
    float* gg = sg + threadIdx.x * LP;
    float dot = 0.f;
    for (int i = 0; i < LP; ++i) dot += gg[i] * a[i];
    for (int i = 0; i < LP; ++i) gg[i] = a[i] * (gg[i] - dot);
  }
  __syncthreads();
  const int rowl = Hh * LP;
  const long long lq0 = f0 / rowl;
  const int l0 = (int)(f0 - lq0 * rowl);
  for (int e = threadIdx.x; e < ng * LP; e += 256) {
    const int t = l0 + e;
    const int dr = t / rowl;
    glogit[(lq0 + dr) * glogit_rs + (t - dr * rowl)] = from_f32<T>(sg[e]);
  }
}

int fill_geom(PrepGeom* gm, const int64_t* shapes, int L) {
  for (int l = 0; l < 4; ++l) gm->w[l] = gm->h[l] = 1.f;
  for (int l = 0; l < L; ++l) {
    if (shapes[2 * l] <= 0 || shapes[2 * l + 1] <= 0) return 0;
    gm->h[l] = (float)shapes[2 * l];
    gm->w[l] = (float)shapes[2 * l + 1];
  }
  return 1;
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" int vs_msda_prep_forward(int dtype, const void* offsets, long long offsets_row_stride, const void* logits,
                                    long long logits_row_stride, const float* ref, long long ref_batch_stride,
                                    const int64_t* shapes, float* loc, float* attw, int B, int Q, int Hh, int L,
                                    int P, void* stream) {
  VS_CHECK(B >= 0 && Q >= 0 && Hh > 0 && L >= 1 && L <= 4 && P >= 1 && L * P <= kMaxLP, "bad sizes");
  VS_CHECK(offsets_row_stride >= (long long)Hh * L * P * 2 && logits_row_stride >= (long long)Hh * L * P,
           "row strides smaller than a row");
  VS_CHECK(shapes, "null pointer");
  PrepGeom gm;
  VS_CHECK(fill_geom(&gm, shapes, L), "non-positive spatial shape");
  const long long groups = (long long)B * Q * Hh;
  if (groups == 0) return VS_OK;
  VS_CHECK(offsets && logits && ref && loc && attw, "null pointer");
  VS_CHECK(((uintptr_t)ref & 7) == 0 && ref_batch_stride % 2 == 0 && ((uintptr_t)loc & 7) == 0,
           "ref / loc must be 8-byte aligned with an even batch stride");
  hipStream_t st = (hipStream_t)stream;
  const int grid = (int)((groups + kGroups - 1) / kGroups);
  if (dtype == VS_BF16)
    hipLaunchKernelGGL(msda_prep_fwd_kernel<bf16>, dim3(grid), dim3(256), 0, st, (const bf16*)offsets,
                       (const bf16*)logits, ref, loc, attw, gm, Q, Hh, L, P, offsets_row_stride, logits_row_stride,
                       ref_batch_stride, groups);
  else if (dtype == VS_F32)
    hipLaunchKernelGGL(msda_prep_fwd_kernel<float>, dim3(grid), dim3(256), 0, st, (const float*)offsets,
                       (const float*)logits, ref, loc, attw, gm, Q, Hh, L, P, offsets_row_stride, logits_row_stride,
                       ref_batch_stride, groups);
  else
    VS_CHECK(false, "dtype must be VS_F32 or VS_BF16");
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_msda_prep_backward(int dtype, const float* grad_loc, const float* grad_attw, const float* attw,
                                     const int64_t* shapes, void* grad_offsets, long long grad_offsets_row_stride,
                                     void* grad_logits, long long grad_logits_row_stride, int B, int Q, int Hh, int L,
                                     int P, void* stream) {
  VS_CHECK(B >= 0 && Q >= 0 && Hh > 0 && L >= 1 && L <= 4 && P >= 1 && L * P <= kMaxLP, "bad sizes");
  VS_CHECK(grad_offsets_row_stride >= (long long)Hh * L * P * 2 && grad_logits_row_stride >= (long long)Hh * L * P,
           "row strides smaller than a row");
  VS_CHECK(shapes, "null pointer");
  PrepGeom gm;
  VS_CHECK(fill_geom(&gm, shapes, L), "non-positive spatial shape");
  const long long groups = (long long)B * Q * Hh;
  if (groups == 0) return VS_OK;
  VS_CHECK(grad_loc && grad_attw && attw && grad_offsets && grad_logits, "null pointer");
  VS_CHECK(((uintptr_t)grad_loc & 7) == 0, "grad_loc must be 8-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  const int grid = (int)((groups + kGroups - 1) / kGroups);
  if (dtype == VS_BF16)
    hipLaunchKernelGGL(msda_prep_bwd_kernel<bf16>, dim3(grid), dim3(256), 0, st, grad_loc, grad_attw, attw,
                       (bf16*)grad_offsets, (bf16*)grad_logits, gm, Hh, L, P, grad_offsets_row_stride,
                       grad_logits_row_stride, groups);
  else if (dtype == VS_F32)
    hipLaunchKernelGGL(msda_prep_bwd_kernel<float>, dim3(grid), dim3(256), 0, st, grad_loc, grad_attw, attw,
                       (float*)grad_offsets, (float*)grad_logits, gm, Hh, L, P, grad_offsets_row_stride,
                       grad_logits_row_stride, groups);
  else
    VS_CHECK(false, "dtype must be VS_F32 or VS_BF16");
  VS_LAUNCH_CHECK();
  return VS_OK;
}
