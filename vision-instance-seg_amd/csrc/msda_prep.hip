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
#include "mfma_util.h"

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

// P = 4 (the production configuration), bf16 projections: every access a whole 8-, 16- or
// 32-byte vector.  The general kernels above move 2-byte projection elements one at a time
// and pay integer divisions per element (2.7-3.2 TB/s at the C2 encoder shape).
//   locations: one thread per (group, level): the level's 4 (x, y) offsets are one 16-B row
//              piece, its 4 locations two 16-B stores;
//   weights:   one thread per group: its L*4 logits (3 x 8 B at L = 3), softmax in registers,
//              L*4 f32 weights as 16-B stores (no LDS).
// Same arithmetic, same order as the general kernels (x / W_l, f32 softmax).
__device__ __forceinline__ void bf16x4_to_f32(uint2 v, float* o) {
  o[0] = __uint_as_float(v.x << 16);
  o[1] = __uint_as_float(v.x & 0xffff0000u);
  o[2] = __uint_as_float(v.y << 16);
  o[3] = __uint_as_float(v.y & 0xffff0000u);
}

template <int L>
__global__ void __launch_bounds__(256) msda_prep_fwd4_kernel(const bf16* __restrict__ off, const bf16* __restrict__ logit,
                                                             const float* __restrict__ ref, float* __restrict__ loc,
                                                             float* __restrict__ aw, PrepGeom gm, int Q, int Hh,
                                                             long long off_rs, long long logit_rs, long long ref_bs,
                                                             long long groups) {
  constexpr int LP = L * 4;
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t < groups * L) {                                   // locations: item (group, level)
    const long long g = t / L;
    const int l = (int)(t - g * L);
    const long long bq = g / Hh;
    const int h = (int)(g - bq * Hh);
    const long long b = bq / Q;
    const int q = (int)(bq - b * Q);
    const uint4 o = *reinterpret_cast<const uint4*>(off + bq * off_rs + (h * L + l) * 8);
    const float2 r = *reinterpret_cast<const float2*>(ref + b * ref_bs + ((long long)q * L + l) * 2);
    float v[8];
    bf16x4_to_f32(make_uint2(o.x, o.y), v);
    bf16x4_to_f32(make_uint2(o.z, o.w), v + 4);
    const float w = gm.w[l], hgt = gm.h[l];
    float4* dst = reinterpret_cast<float4*>(loc + g * LP * 2 + l * 8);
    dst[0] = make_float4(r.x + v[0] / w, r.y + v[1] / hgt, r.x + v[2] / w, r.y + v[3] / hgt);
    dst[1] = make_float4(r.x + v[4] / w, r.y + v[5] / hgt, r.x + v[6] / w, r.y + v[7] / hgt);
  }
  if (t < groups) {                                       // weights: one group
    const long long g = t;
    const long long bq = g / Hh;
    const int h = (int)(g - bq * Hh);
    const uint2* src = reinterpret_cast<const uint2*>(logit + bq * logit_rs + h * LP);
    float v[LP];
#pragma unroll
    for (int k = 0; k < L; ++k) bf16x4_to_f32(src[k], v + 4 * k);
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < LP; ++i) m = fmaxf(m, v[i]);
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < LP; ++i) {
      v[i] = expf(v[i] - m);
      sum += v[i];
    }
    float4* dst = reinterpret_cast<float4*>(aw + g * LP);
#pragma unroll
    for (int k = 0; k < L; ++k) dst[k] = make_float4(v[4 * k] / sum, v[4 * k + 1] / sum, v[4 * k + 2] / sum, v[4 * k + 3] / sum);
  }
}

template <int L>
__global__ void __launch_bounds__(256) msda_prep_bwd4_kernel(const float* __restrict__ gloc,
                                                             const float* __restrict__ gaw,
                                                             const float* __restrict__ aw, bf16* __restrict__ goff,
                                                             bf16* __restrict__ glogit, PrepGeom gm, int Hh,
                                                             long long goff_rs, long long glogit_rs, long long groups) {
  constexpr int LP = L * 4;
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t < groups * L) {                                   // offsets' gradient: item (group, level)
    const long long g = t / L;
    const int l = (int)(t - g * L);
    const long long bq = g / Hh;
    const int h = (int)(g - bq * Hh);
    const float4* src = reinterpret_cast<const float4*>(gloc + g * LP * 2 + l * 8);
    const float4 a = src[0], c = src[1];
    const float w = gm.w[l], hgt = gm.h[l];
    uint4 o;
    o.x = (unsigned)(unsigned short)bf16_bits(a.x / w) | ((unsigned)(unsigned short)bf16_bits(a.y / hgt) << 16);
    o.y = (unsigned)(unsigned short)bf16_bits(a.z / w) | ((unsigned)(unsigned short)bf16_bits(a.w / hgt) << 16);
    o.z = (unsigned)(unsigned short)bf16_bits(c.x / w) | ((unsigned)(unsigned short)bf16_bits(c.y / hgt) << 16);
    o.w = (unsigned)(unsigned short)bf16_bits(c.z / w) | ((unsigned)(unsigned short)bf16_bits(c.w / hgt) << 16);
    *reinterpret_cast<uint4*>(goff + bq * goff_rs + (h * L + l) * 8) = o;
  }
  if (t < groups) {                                       // logits' gradient: one group
    const long long g = t;
    const long long bq = g / Hh;
    const int h = (int)(g - bq * Hh);
    float a[LP], gg[LP];
#pragma unroll
    for (int k = 0; k < L; ++k) {
      const float4 x = reinterpret_cast<const float4*>(aw + g * LP)[k];
      const float4 y = reinterpret_cast<const float4*>(gaw + g * LP)[k];
      a[4 * k] = x.x; a[4 * k + 1] = x.y; a[4 * k + 2] = x.z; a[4 * k + 3] = x.w;
      gg[4 * k] = y.x; gg[4 * k + 1] = y.y; gg[4 * k + 2] = y.z; gg[4 * k + 3] = y.w;
    }
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < LP; ++i) dot += gg[i] * a[i];
    uint2* dst = reinterpret_cast<uint2*>(glogit + bq * glogit_rs + h * LP);
#pragma unroll
    for (int k = 0; k < L; ++k) {
      float r[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = a[4 * k + e] * (gg[4 * k + e] - dot);
      dst[k] = make_uint2((unsigned)(unsigned short)bf16_bits(r[0]) | ((unsigned)(unsigned short)bf16_bits(r[1]) << 16),
                          (unsigned)(unsigned short)bf16_bits(r[2]) | ((unsigned)(unsigned short)bf16_bits(r[3]) << 16));
    }
  }
}

// the vector kernels' alignment: 16-B offset rows, 8-B logit pieces, 16-B f32 outputs
bool prep4_ok(int dtype, int P, int L, const void* off, long long off_rs, const void* logit, long long logit_rs,
              const void* f1, const void* f2) {
  return dtype == VS_BF16 && P == 4 && L >= 1 && L <= 4 && ((uintptr_t)off & 15) == 0 && off_rs % 8 == 0 &&
         ((uintptr_t)logit & 7) == 0 && logit_rs % 4 == 0 && ((uintptr_t)f1 & 15) == 0 && ((uintptr_t)f2 & 15) == 0;
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
  if (prep4_ok(dtype, P, L, offsets, offsets_row_stride, logits, logits_row_stride, loc, attw)) {
    const dim3 g4((unsigned)((groups * L + 255) / 256));
#define VS_PF4(LL)                                                                                                  \
  hipLaunchKernelGGL((msda_prep_fwd4_kernel<LL>), g4, dim3(256), 0, st, (const bf16*)offsets, (const bf16*)logits, \
                     ref, loc, attw, gm, Q, Hh, offsets_row_stride, logits_row_stride, ref_batch_stride, groups)
    switch (L) {
      case 1: VS_PF4(1); break;
      case 2: VS_PF4(2); break;
      case 3: VS_PF4(3); break;
      default: VS_PF4(4); break;
    }
#undef VS_PF4
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
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
  if (prep4_ok(dtype, P, L, grad_offsets, grad_offsets_row_stride, grad_logits, grad_logits_row_stride, grad_loc,
               grad_attw) && ((uintptr_t)attw & 15) == 0) {
    const dim3 g4((unsigned)((groups * L + 255) / 256));
#define VS_PB4(LL)                                                                                                \
  hipLaunchKernelGGL((msda_prep_bwd4_kernel<LL>), g4, dim3(256), 0, st, grad_loc, grad_attw, attw,                \
                     (bf16*)grad_offsets, (bf16*)grad_logits, gm, Hh, grad_offsets_row_stride,                    \
                     grad_logits_row_stride, groups)
    switch (L) {
      case 1: VS_PB4(1); break;
      case 2: VS_PB4(2); break;
      case 3: VS_PB4(3); break;
      default: VS_PB4(4); break;
    }
#undef VS_PB4
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
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
