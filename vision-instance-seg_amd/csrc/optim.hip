// Per-parameter gradient-norm clipping over a flat f32 gradient buffer.
//
// detectron2's "norm" clip (reference training/maskdino/train_full.py:266-271, clip
// value 0.01) calls torch.nn.utils.clip_grad_norm_(p, 0.01) for EVERY parameter:
// g *= min(1, max_norm / (||g||_2 + 1e-6)).  With ~500 parameters that is thousands of
// tiny launches per step in eager PyTorch.  Here the f32 master gradients live in one
// flat buffer (each parameter 16-B aligned) and a static chunk table splits every
// parameter into chunks of <= kChunk elements:
//   table[c] = {start, len, first chunk of the parameter, chunks of the parameter}.
// Kernel 1 writes each chunk's sum of squares; kernel 2 recomputes its parameter's norm
// from that parameter's chunk partials (same order in every block: deterministic, no
// atomics) and scales the chunk.
#include "common.h"

namespace vs {
namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float block_sum(float v, float* sh) {
  for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s, 64);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) sh[w] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0) {
    for (int i = 0; i < kThreads / 64; ++i) t += sh[i];
    sh[kThreads / 64] = t;
  }
  __syncthreads();
  return sh[kThreads / 64];
}

__global__ void __launch_bounds__(kThreads) chunk_sumsq_kernel(const float* __restrict__ data,
                                                               const int* __restrict__ table,
                                                               float* __restrict__ partial) {
  __shared__ float sh[kThreads / 64 + 1];
  const int c = blockIdx.x;
  const int start = table[c * 4 + 0], len = table[c * 4 + 1];
  const float* p = data + start;               // start % 4 == 0 (16-B aligned parameters)
  float acc = 0.f;
  const int n4 = len >> 2;
  for (int i = threadIdx.x; i < n4; i += kThreads) {
    const float4 v = reinterpret_cast<const float4*>(p)[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  for (int i = (n4 << 2) + threadIdx.x; i < len; i += kThreads) acc += p[i] * p[i];
  const float t = block_sum(acc, sh);
  if (threadIdx.x == 0) partial[c] = t;
}

__global__ void __launch_bounds__(kThreads) chunk_scale_kernel(float* __restrict__ data,
                                                               const int* __restrict__ table,
                                                               const float* __restrict__ partial, float max_norm,
                                                               float eps) {
  __shared__ float scale;
  const int c = blockIdx.x;
  const int start = table[c * 4 + 0], len = table[c * 4 + 1];
  if (threadIdx.x == 0) {
    const int first = table[c * 4 + 2], count = table[c * 4 + 3];
    float s = 0.f;
    for (int i = 0; i < count; ++i) s += partial[first + i];
    scale = fminf(1.f, max_norm / (sqrtf(s) + eps));
  }
  __syncthreads();
  const float k = scale;
  if (k == 1.f) return;
  float* p = data + start;
  const int n4 = len >> 2;
  for (int i = threadIdx.x; i < n4; i += kThreads) {
    float4 v = reinterpret_cast<float4*>(p)[i];
    v.x *= k; v.y *= k; v.z *= k; v.w *= k;
    reinterpret_cast<float4*>(p)[i] = v;
  }
  for (int i = (n4 << 2) + threadIdx.x; i < len; i += kThreads) p[i] *= k;
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" long long vs_segment_clip_workspace_bytes(int num_chunks) {
  return (long long)num_chunks * sizeof(float);
}

extern "C" int vs_segment_clip(float* data, const int* table, int num_chunks, float max_norm, float eps,
                               void* workspace, void* stream) {
  VS_CHECK(num_chunks >= 0, "bad chunk count");
  if (num_chunks == 0) return VS_OK;
  VS_CHECK(data && table && workspace, "null pointer");
  VS_CHECK(max_norm > 0.f, "max_norm must be positive");
  hipStream_t st = (hipStream_t)stream;
  float* partial = (float*)workspace;
  hipLaunchKernelGGL(chunk_sumsq_kernel, dim3(num_chunks), dim3(kThreads), 0, st, data, table, partial);
  hipLaunchKernelGGL(chunk_scale_kernel, dim3(num_chunks), dim3(kThreads), 0, st, data, table, partial, max_norm,
                     eps);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
