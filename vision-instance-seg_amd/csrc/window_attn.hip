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
#include "common.h"

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
  if (dtype == VS_BF16) {
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
  if (dtype == VS_BF16) {
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
