// Fused optimiser step over flat parameter / gradient / state buffers.
//
// The reference trains through detectron2's DefaultTrainer (training/maskdino/
// train_full.py:153-167): SGD with momentum 0.9, weight decay 0.05 except on norm
// parameters, and CLIP_GRADIENTS type "norm", value 0.01 (train_full.py:266-271), i.e.
// torch.nn.utils.clip_grad_norm_(p, 0.01) for EVERY parameter before the update.  In
// eager PyTorch that is thousands of tiny launches per step (a norm, a scale and a
// multi-tensor update per parameter, then a bf16 cast-copy of every weight).
//
// Here every buffer of the optimiser is flat: gradients (the model's .grad tensors are
// views of one buffer), f32 master weights, the f32 momentum / Adam moments, and the
// bf16 working weights the model reads (views of one buffer too).  Each parameter starts
// 8-element aligned; a static chunk table splits every parameter into chunks of
// <= kChunk elements:
//   table[c]  = {start, len, first chunk of the parameter, chunks of the parameter, parameter}
//   hyper[c]  = {lr multiplier, weight decay} of the chunk's parameter group.
// Per parameter, a gradient FLAG (> 0.5: the parameter got a gradient this step on some
// rank; it travels in the gradient buffer and is summed by the all-reduce) and a step
// COUNT: torch.optim skips a parameter whose .grad is None -- no decay, no momentum /
// moment update -- and AdamW's bias correction counts the steps that parameter took.
// Two launches per step (three with the "full_model" clip):
//   flat_sumsq_kernel: each chunk's sum of squares of the (averaged) gradient; the first
//                      chunk of a flagged parameter advances its step count; block 0 the
//                      global step counter;
//   flat_total_kernel: ("full_model" only) the one global sum of squares, in chunk order;
//   flat_step_kernel:  recomputes its parameter's norm from that parameter's partials
//                      (per-parameter clip; or reads the global total), then clip-scale +
//                      weight decay + SGD-momentum / AdamW update of the master weights +
//                      bf16 round of the working weights, one pass; unflagged parameters
//                      are left untouched.
// Deterministic: no atomics, every block sums the partials in the same order.
// HBM-bound: per element it reads the gradient (2 or 4 B) and master + state (8 or 12 B)
// and writes master + state + working weight (10 or 14 B).
#include "common.h"

namespace vs {
namespace {

constexpr int kThreads = 256;
constexpr int kVec = 8;

__device__ __forceinline__ float wave_sum(float v) {
  for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s, 64);
  return v;
}

__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
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

template <typename G> __device__ __forceinline__ void load8(const G* p, float* out);
template <> __device__ __forceinline__ void load8<bf16>(const bf16* p, float* out) { Vec16<bf16>::load(p, out); }
template <> __device__ __forceinline__ void load8<float>(const float* p, float* out) {
  Vec16<float>::load(p, out);
  Vec16<float>::load(p + 4, out + 4);
}
__device__ __forceinline__ void store8(float* p, const float* in) {
  Vec16<float>::store(p, in);
  Vec16<float>::store(p + 4, in + 4);
}

constexpr int kCols = 5;          // chunk table columns

template <typename G>
__device__ __forceinline__ bool has_grad(const G* flags, int prm) {
  return flags == nullptr || to_f32(flags[prm]) > 0.5f;
}

template <typename G>
__global__ void __launch_bounds__(kThreads) flat_sumsq_kernel(const G* __restrict__ grad, const G* __restrict__ flags,
                                                              const int* __restrict__ table, float* __restrict__ partial,
                                                              float* __restrict__ step, float* __restrict__ psteps) {
  __shared__ float sh[kThreads / 64 + 1];
  const int c = blockIdx.x;
  if (c == 0 && threadIdx.x == 0 && step) step[0] += 1.f;
  const int start = table[c * kCols + 0], len = table[c * kCols + 1], prm = table[c * kCols + 4];
  if (!has_grad(flags, prm)) {           // uniform per block
    if (threadIdx.x == 0) partial[c] = 0.f;
    return;
  }
  if (threadIdx.x == 0 && table[c * kCols + 2] == c) psteps[prm] += 1.f;
  const G* p = grad + start;                  // start % 8 == 0
  float acc = 0.f;
  const int n8 = len / kVec;
  for (int i = threadIdx.x; i < n8; i += kThreads) {
    float v[kVec];
    load8<G>(p + i * kVec, v);
#pragma unroll
    for (int j = 0; j < kVec; ++j) acc += v[j] * v[j];
  }
  for (int i = n8 * kVec + threadIdx.x; i < len; i += kThreads) {
    const float v = to_f32(p[i]);
    acc += v * v;
  }
  const float t = block_sum(acc, sh);
  if (threadIdx.x == 0) partial[c] = t;
}

// "full_model" clip: partial[num_chunks] = the sum of every chunk's partial (one block,
// fixed order), read by every block of the step kernel instead of num_chunks partials.
__global__ void __launch_bounds__(kThreads) flat_total_kernel(float* __restrict__ partial, int num_chunks) {
  __shared__ float sh[kThreads / 64 + 1];
  float acc = 0.f;
  for (int i = threadIdx.x; i < num_chunks; i += kThreads) acc += partial[i];
  const float t = block_sum(acc, sh);
  if (threadIdx.x == 0) partial[num_chunks] = t;
}

struct StepArgs {
  float grad_scale;      // 1 / world size (gradients summed by the all-reduce)
  int clip;              // 0 none, 1 per parameter (detectron2 "norm"), 2 full model
  float clip_value;
  float clip_eps;        // clip_grad_norm_: max_norm / (norm + 1e-6)
  int optimizer;         // 0 SGD (momentum, dampening 0, no nesterov), 1 AdamW
  float momentum, beta1, beta2, eps;
};

// Per-element update, torch.optim semantics (SGD: torch/optim/sgd.py; AdamW:
// torch/optim/adamw.py, single-tensor path).
__device__ __forceinline__ void update(float g, float& p, float& s1, float& s2, float lr, float wd, bool first,
                                       const StepArgs& a, float bc1, float bc2_sqrt) {
  if (a.optimizer == 0) {
    const float d = g + wd * p;
    s1 = first ? d : a.momentum * s1 + d;
    p -= lr * s1;
  } else {
    p *= 1.f - lr * wd;
    s1 += (1.f - a.beta1) * (g - s1);
    s2 = a.beta2 * s2 + (1.f - a.beta2) * g * g;
    const float denom = sqrtf(s2) / bc2_sqrt + a.eps;
    p -= (lr / bc1) * s1 / denom;
  }
}

template <typename G, typename W>
__global__ void __launch_bounds__(kThreads) flat_step_kernel(const G* __restrict__ grad, const G* __restrict__ flags,
                                                             float* __restrict__ master,
                                                             float* __restrict__ s1buf, float* __restrict__ s2buf,
                                                             W* __restrict__ wout, const int* __restrict__ table,
                                                             const float* __restrict__ hyper,
                                                             const float* __restrict__ partial, int num_chunks,
                                                             const float* __restrict__ lr_ptr,
                                                             const float* __restrict__ psteps, StepArgs a) {
  __shared__ float s_scale;
  const int c = blockIdx.x;
  const int start = table[c * kCols + 0], len = table[c * kCols + 1], prm = table[c * kCols + 4];
  if (!has_grad(flags, prm)) return;     // torch.optim: a parameter without a gradient is skipped
  if (threadIdx.x < 64) {
    float k = 1.f;
    if (a.clip == 1) {
      const int first = table[c * kCols + 2], count = table[c * kCols + 3];
      float s = 0.f;
      for (int i = threadIdx.x; i < count; i += 64) s += partial[first + i];
      s = wave_sum(s);
      k = fminf(1.f, a.clip_value / (sqrtf(s) * a.grad_scale + a.clip_eps));
    } else if (a.clip == 2) {
      k = fminf(1.f, a.clip_value / (sqrtf(partial[num_chunks]) * a.grad_scale + a.clip_eps));
    }
    if (threadIdx.x == 0) s_scale = k * a.grad_scale;
  }
  __syncthreads();
  const float gk = s_scale;
  const float lr = lr_ptr[0] * hyper[c * 2 + 0];
  const float wd = hyper[c * 2 + 1];
  const float t = psteps[prm];           // this parameter's steps, this one included
  const bool first = t <= 1.f;
  float bc1 = 1.f, bc2s = 1.f;
  if (a.optimizer == 1) {
    bc1 = 1.f - powf(a.beta1, t);
    bc2s = sqrtf(1.f - powf(a.beta2, t));
  }
  const int n8 = len / kVec;
  for (int i = threadIdx.x; i < n8; i += kThreads) {
    const int o = start + i * kVec;
    float g[kVec], p[kVec], m[kVec], v[kVec];
    load8<G>(grad + o, g);
    load8<float>(master + o, p);
    load8<float>(s1buf + o, m);
    if (a.optimizer == 1) load8<float>(s2buf + o, v);
#pragma unroll
    for (int j = 0; j < kVec; ++j) update(g[j] * gk, p[j], m[j], v[j], lr, wd, first, a, bc1, bc2s);
    store8(master + o, p);
    store8(s1buf + o, m);
    if (a.optimizer == 1) store8(s2buf + o, v);
    if (wout) Vec16<W>::store(wout + o, p);
  }
  for (int i = n8 * kVec + threadIdx.x; i < len; i += kThreads) {
    const int o = start + i;
    float p = master[o], m = s1buf[o], v = a.optimizer == 1 ? s2buf[o] : 0.f;
    update(to_f32(grad[o]) * gk, p, m, v, lr, wd, first, a, bc1, bc2s);
    master[o] = p;
    s1buf[o] = m;
    if (a.optimizer == 1) s2buf[o] = v;
    if (wout) wout[o] = from_f32<W>(p);
  }
}

template <typename G>
int launch_step(const G* grad, const G* flags, float* master, float* s1, float* s2, bf16* wout, const int* table,
                const float* hyper, int num_chunks, const StepArgs& a, const float* lr, float* step, float* psteps,
                float* partial, hipStream_t st) {
  // always launched: block 0 also advances the step counter
  hipLaunchKernelGGL(flat_sumsq_kernel<G>, dim3(num_chunks), dim3(kThreads), 0, st, grad, flags, table, partial, step,
                     psteps);
  if (a.clip == 2) hipLaunchKernelGGL(flat_total_kernel, dim3(1), dim3(kThreads), 0, st, partial, num_chunks);
  hipLaunchKernelGGL((flat_step_kernel<G, bf16>), dim3(num_chunks), dim3(kThreads), 0, st, grad, flags, master, s1,
                     s2, wout, table, hyper, partial, num_chunks, lr, psteps, a);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" long long vs_flat_step_workspace_bytes(int num_chunks) {
  return ((long long)num_chunks + 1) * sizeof(float);
}

extern "C" int vs_flat_step(int grad_dtype, const void* grad, const void* grad_flags, float grad_scale, float* master,
                            float* state1, float* state2, void* weights_bf16, const int* table, const float* hyper,
                            int num_chunks, int optimizer, int clip, float clip_value, float clip_eps, float momentum,
                            float beta1, float beta2, float eps, const float* lr, float* step, float* param_steps,
                            void* workspace, void* stream) {
  VS_CHECK(num_chunks >= 0, "bad chunk count");
  if (num_chunks == 0) return VS_OK;
  VS_CHECK(grad && master && state1 && table && hyper && lr && step && param_steps && workspace, "null pointer");
  VS_CHECK(grad_dtype == VS_F32 || grad_dtype == VS_BF16, "gradient dtype must be f32 or bf16");
  VS_CHECK(optimizer == 0 || optimizer == 1, "optimizer must be 0 (SGD) or 1 (AdamW)");
  VS_CHECK(optimizer == 0 || state2, "AdamW needs the second-moment buffer");
  VS_CHECK(clip >= 0 && clip <= 2, "clip must be 0 (none), 1 (per parameter) or 2 (full model)");
  VS_CHECK(clip == 0 || clip_value > 0.f, "clip value must be positive");
  VS_CHECK(grad_scale > 0.f, "grad_scale must be positive");
  StepArgs a{grad_scale, clip, clip_value, clip_eps, optimizer, momentum, beta1, beta2, eps};
  hipStream_t st = (hipStream_t)stream;
  float* partial = (float*)workspace;
  bf16* w = (bf16*)weights_bf16;
  if (grad_dtype == VS_BF16)
    return launch_step<bf16>((const bf16*)grad, (const bf16*)grad_flags, master, state1, state2, w, table, hyper,
                             num_chunks, a, lr, step, param_steps, partial, st);
  return launch_step<float>((const float*)grad, (const float*)grad_flags, master, state1, state2, w, table, hyper,
                            num_chunks, a, lr, step, param_steps, partial, st);
}
