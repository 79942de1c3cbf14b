// Multi-scale deformable attention sampling (MSDeformAttn), forward + backward.
//
// Semantics: upstream MSDeformAttn CUDA extension (ms_deform_attn_im2col_bilinear /
// col2im), oracle HF:m2f:798-837.  Layout: value [B,S,H,32], loc [B,Q,H,L,P,2] f32,
// attn [B,Q,H,L,P] f32, out [B,Q,H*32].
//
// Forward (HBM/L2 gather-bound): a "group" = one (b, q, head).  Each lane owns one
// 16-byte slice of the 32 head channels (8 bf16 or 4 f32), so a group is 4 (bf16) or
// 8 (f32) lanes and one wave serves 16 (bf16) / 8 (f32) groups.  Every corner tap is
// one 16-B load per lane, adjacent lanes read adjacent bytes; the group's loc/attn
// rows (96 B / 48 B, 16-B aligned) are read as float4.  Accumulation in f32.
//
// Backward: one lane per channel (32 lanes = one group, 2 groups per wave) so every
// grad_value atomic wave-instruction is two contiguous 128-B row segments (the shape
// the f32 atomic path runs at full rate, MI355X_MICROARCH §Global float atomics);
// grad_loc / grad_attn are 32-lane shuffle reductions, written by lane 0.
#include "common.h"

namespace vs {
namespace {

constexpr int kD = 32;
constexpr int kMaxLevels = 4;

struct Levels {
  int h[kMaxLevels];
  int w[kMaxLevels];
  int start[kMaxLevels];
};

template <typename T>
__global__ void __launch_bounds__(256) msda_fwd_kernel(const T* __restrict__ value,
                                                        const float* __restrict__ loc,
                                                        const float* __restrict__ attw,
                                                        T* __restrict__ out, Levels lv, int S,
                                                        int Hh, int Q, int L, int P,
                                                        long long groups) {
  constexpr int V = Vec16<T>::N;       // channels per lane
  constexpr int LPG = kD / V;          // lanes per group
  long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long stride = (long long)gridDim.x * blockDim.x;
  const int LP = L * P;
  for (; gid < groups * LPG; gid += stride) {
    const long long grp = gid / LPG;
    const int sub = (int)(gid % LPG);
    const int h = (int)(grp % Hh);
    const long long b = grp / Hh / Q;
    const float* lp = loc + grp * LP * 2;
    const float* wp = attw + grp * LP;
    const size_t rowstride = (size_t)Hh * kD;  // elements between spatial positions
    const T* vb = value + ((size_t)b * S * Hh + h) * kD + sub * V;
    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
    for (int l = 0; l < L; ++l) {
      const int Hl = lv.h[l], Wl = lv.w[l];
      const T* vl = vb + (size_t)lv.start[l] * rowstride;
      const float fH = (float)Hl, fW = (float)Wl;
      for (int p = 0; p < P; ++p) {
        const float x = lp[(l * P + p) * 2 + 0];
        const float y = lp[(l * P + p) * 2 + 1];
        const float a = wp[l * P + p];
        const float him = y * fH - 0.5f;
        const float wim = x * fW - 0.5f;
        if (him > -1.f && wim > -1.f && him < fH && wim < fW) {
          const float fh0 = floorf(him), fw0 = floorf(wim);
          const int h0 = (int)fh0, w0 = (int)fw0;
          const float lh = him - fh0, lw = wim - fw0;
          const float hh = 1.f - lh, hw = 1.f - lw;
          const float cw[4] = {hh * hw, hh * lw, lh * hw, lh * lw};
          const bool ok[4] = {h0 >= 0 && w0 >= 0, h0 >= 0 && w0 + 1 <= Wl - 1,
                              h0 + 1 <= Hl - 1 && w0 >= 0, h0 + 1 <= Hl - 1 && w0 + 1 <= Wl - 1};
          const int off[4] = {h0 * Wl + w0, h0 * Wl + w0 + 1, (h0 + 1) * Wl + w0,
                              (h0 + 1) * Wl + w0 + 1};
          float val[V];
#pragma unroll
          for (int i = 0; i < V; ++i) val[i] = 0.f;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            if (ok[c]) {
              float t[V];
              Vec16<T>::load(vl + (size_t)off[c] * rowstride, t);
#pragma unroll
              for (int i = 0; i < V; ++i) val[i] += cw[c] * t[i];
            }
          }
#pragma unroll
          for (int i = 0; i < V; ++i) acc[i] += a * val[i];
        }
      }
    }
    Vec16<T>::store(out + grp * kD + sub * V, acc);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) msda_bwd_kernel(
    const T* __restrict__ value, const float* __restrict__ loc, const float* __restrict__ attw,
    const T* __restrict__ gout, float* __restrict__ gvalue, float* __restrict__ gloc,
    float* __restrict__ gattw, Levels lv, int S, int Hh, int Q, int L, int P, long long groups) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long grp = gid >> 5;
  const int c = (int)(gid & 31);
  if (grp >= groups) return;  // uniform per 32-lane half-wave
  const int LP = L * P;
  const int h = (int)(grp % Hh);
  const long long b = grp / Hh / Q;
  const float* lp = loc + grp * LP * 2;
  const float* wp = attw + grp * LP;
  const size_t rowstride = (size_t)Hh * kD;
  const size_t vbase = ((size_t)b * S * Hh + h) * kD + c;
  const float g = to_f32(gout[grp * kD + c]);
  for (int l = 0; l < L; ++l) {
    const int Hl = lv.h[l], Wl = lv.w[l];
    const size_t lbase = vbase + (size_t)lv.start[l] * rowstride;
    const float fH = (float)Hl, fW = (float)Wl;
    for (int p = 0; p < P; ++p) {
      const int tap = l * P + p;
      const float x = lp[tap * 2 + 0];
      const float y = lp[tap * 2 + 1];
      const float a = wp[tap];
      const float him = y * fH - 0.5f;
      const float wim = x * fW - 0.5f;
      float r_w = 0.f, r_x = 0.f, r_y = 0.f;
      if (him > -1.f && wim > -1.f && him < fH && wim < fW) {
        const float fh0 = floorf(him), fw0 = floorf(wim);
        const int h0 = (int)fh0, w0 = (int)fw0;
        const float lh = him - fh0, lw = wim - fw0;
        const float hh = 1.f - lh, hw = 1.f - lw;
        const float ga = g * a;
        float v1 = 0.f, v2 = 0.f, v3 = 0.f, v4 = 0.f;
        if (h0 >= 0 && w0 >= 0) {
          const size_t o = lbase + (size_t)(h0 * Wl + w0) * rowstride;
          v1 = to_f32(value[o]);
          atomicAdd(gvalue + o, hh * hw * ga);
        }
        if (h0 >= 0 && w0 + 1 <= Wl - 1) {
          const size_t o = lbase + (size_t)(h0 * Wl + w0 + 1) * rowstride;
          v2 = to_f32(value[o]);
          atomicAdd(gvalue + o, hh * lw * ga);
        }
        if (h0 + 1 <= Hl - 1 && w0 >= 0) {
          const size_t o = lbase + (size_t)((h0 + 1) * Wl + w0) * rowstride;
          v3 = to_f32(value[o]);
          atomicAdd(gvalue + o, lh * hw * ga);
        }
        if (h0 + 1 <= Hl - 1 && w0 + 1 <= Wl - 1) {
          const size_t o = lbase + (size_t)((h0 + 1) * Wl + w0 + 1) * rowstride;
          v4 = to_f32(value[o]);
          atomicAdd(gvalue + o, lh * lw * ga);
        }
        const float val = hh * hw * v1 + hh * lw * v2 + lh * hw * v3 + lh * lw * v4;
        r_w = g * val;
        const float dh = -hw * v1 - lw * v2 + hw * v3 + lw * v4;   // d val / d him
        const float dw = -hh * v1 + hh * v2 - lh * v3 + lh * v4;   // d val / d wim
        r_x = fW * ga * dw;
        r_y = fH * ga * dh;
      }
#pragma unroll
      for (int s = 16; s >= 1; s >>= 1) {
        r_w += __shfl_xor(r_w, s, 32);
        r_x += __shfl_xor(r_x, s, 32);
        r_y += __shfl_xor(r_y, s, 32);
      }
      if (c == 0) {
        gattw[grp * LP + tap] = r_w;
        gloc[(grp * LP + tap) * 2 + 0] = r_x;
        gloc[(grp * LP + tap) * 2 + 1] = r_y;
      }
    }
  }
}

int fill_levels(Levels* lv, const int64_t* shapes, const int64_t* starts, int L, int S) {
  long long tot = 0;
  for (int l = 0; l < L; ++l) {
    lv->h[l] = (int)shapes[2 * l];
    lv->w[l] = (int)shapes[2 * l + 1];
    lv->start[l] = (int)starts[l];
    if (lv->h[l] <= 0 || lv->w[l] <= 0 || starts[l] != tot) return 0;
    tot += shapes[2 * l] * shapes[2 * l + 1];
  }
  return tot == S;
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" int vs_msda_forward(int dtype, const void* value, const int64_t* shapes,
                               const int64_t* starts, const float* loc, const float* attw,
                               void* out, int B, int S, int Hh, int D, int L, int Q, int P,
                               void* stream) {
  VS_CHECK(D == kD, "channels per head must be 32");
  VS_CHECK(L >= 1 && L <= kMaxLevels, "1..4 levels supported");
  VS_CHECK(B > 0 && S > 0 && Hh > 0 && Q >= 0 && P > 0, "bad sizes");
  VS_CHECK(value && loc && attw && out && shapes && starts, "null pointer");
  Levels lv;
  VS_CHECK(fill_levels(&lv, shapes, starts, L, S), "spatial shapes / level starts inconsistent with S");
  if (Q == 0) return VS_OK;
  hipStream_t st = (hipStream_t)stream;
  const long long groups = (long long)B * Q * Hh;
  const int block = 256;
  if (dtype == VS_BF16) {
    int grid = grid_for(groups * 4, block, 256 * 64);
    hipLaunchKernelGGL(msda_fwd_kernel<bf16>, dim3(grid), dim3(block), 0, st, (const bf16*)value,
                       loc, attw, (bf16*)out, lv, S, Hh, Q, L, P, groups);
  } else if (dtype == VS_F32) {
    int grid = grid_for(groups * 8, block, 256 * 64);
    hipLaunchKernelGGL(msda_fwd_kernel<float>, dim3(grid), dim3(block), 0, st, (const float*)value,
                       loc, attw, (float*)out, lv, S, Hh, Q, L, P, groups);
  } else {
    VS_CHECK(false, "dtype must be VS_F32 or VS_BF16");
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_msda_backward(int dtype, const void* value, const int64_t* shapes,
                                const int64_t* starts, const float* loc, const float* attw,
                                const void* gout, float* gvalue, float* gloc, float* gattw,
                                int B, int S, int Hh, int D, int L, int Q, int P, void* stream) {
  VS_CHECK(D == kD, "channels per head must be 32");
  VS_CHECK(L >= 1 && L <= kMaxLevels, "1..4 levels supported");
  VS_CHECK(B > 0 && S > 0 && Hh > 0 && Q >= 0 && P > 0, "bad sizes");
  VS_CHECK(value && loc && attw && gout && gvalue && gloc && gattw && shapes && starts, "null pointer");
  Levels lv;
  VS_CHECK(fill_levels(&lv, shapes, starts, L, S), "spatial shapes / level starts inconsistent with S");
  hipStream_t st = (hipStream_t)stream;
  VS_HIP(hipMemsetAsync(gvalue, 0, sizeof(float) * (size_t)B * S * Hh * kD, st));
  if (Q == 0) return VS_OK;
  const long long groups = (long long)B * Q * Hh;
  const int block = 256;
  const long long threads = groups * 32;
  const int grid = (int)((threads + block - 1) / block);
  if (dtype == VS_BF16) {
    hipLaunchKernelGGL(msda_bwd_kernel<bf16>, dim3(grid), dim3(block), 0, st, (const bf16*)value,
                       loc, attw, (const bf16*)gout, gvalue, gloc, gattw, lv, S, Hh, Q, L, P, groups);
  } else if (dtype == VS_F32) {
    hipLaunchKernelGGL(msda_bwd_kernel<float>, dim3(grid), dim3(block), 0, st, (const float*)value,
                       loc, attw, (const float*)gout, gvalue, gloc, gattw, lv, S, Hh, Q, L, P, groups);
  } else {
    VS_CHECK(false, "dtype must be VS_F32 or VS_BF16");
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}
