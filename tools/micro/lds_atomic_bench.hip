// LDS / global float-atomic throughput microbenchmark on gfx950 (one launch per mode).
//   mode 0: ds_add_f32, lane-consecutive addresses (conflict-free)
//   mode 1: ds_add_f32, all lanes of a half-wave on one address
//   mode 2: plain LDS read-modify-write (ds_read + v_add + ds_write), lane-consecutive
//   mode 3: global atomicAdd f32 to lane-consecutive addresses in a 32 MB buffer
//   mode 4: ds_add_u32 (integer), lane-consecutive, no return
//   mode 5: ds_add_rtn_u32 (integer), lane-consecutive, result used (a rank)
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(256) k_lds(float* out, int iters, int mode) {
  __shared__ float acc[8192];
  for (int i = threadIdx.x; i < 8192; i += 256) acc[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float v = 1.0f + threadIdx.x * 1e-3f;
  for (int it = 0; it < iters; ++it) {
    const int base = ((it * 7 + wave * 13) & 63) * 128;
    int addr = mode == 1 ? base + (lane >> 5) * 64 : base + lane;
    if (mode == 2) {
      acc[addr] += v;
    } else {
      atomicAdd(&acc[addr], v);
    }
  }
  __syncthreads();
  float s = 0.f;
  for (int i = threadIdx.x; i < 8192; i += 256) s += acc[i];
  if (s == 12345.f) out[blockIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_ldsi(int* out, int iters, int mode) {
  __shared__ int acc[8192];
  for (int i = threadIdx.x; i < 8192; i += 256) acc[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int r = 0;
  for (int it = 0; it < iters; ++it) {
    const int base = ((it * 7 + wave * 13) & 63) * 128;
    if (mode == 4) atomicAdd(&acc[base + lane], 1);
    else r += atomicAdd(&acc[base + lane], 1);
  }
  __syncthreads();
  int s = r;
  for (int i = threadIdx.x; i < 8192; i += 256) s += acc[i];
  if (s == 12345) out[blockIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_glb(float* buf, int iters) {
  const int lane = threadIdx.x & 63;
  const size_t n = 8u << 20;
  size_t base = ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
  for (int it = 0; it < iters; ++it) {
    atomicAdd(&buf[(base + (size_t)it * 1048576 * 3 + lane) % n], 1.0f);
  }
}

int main() {
  float *out, *buf;
  hipMalloc(&out, 1 << 20);
  hipMalloc(&buf, 32 << 20);
  hipMemset(buf, 0, 32 << 20);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int blocks = 256 * 8, iters = 4096;
  for (int mode = 0; mode < 3; ++mode) {
    hipLaunchKernelGGL(k_lds, dim3(blocks), dim3(256), 0, 0, out, 64, mode);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_lds, dim3(blocks), dim3(256), 0, 0, out, iters, mode);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double ops = (double)blocks * 256 * iters;
    printf("mode %d: %.3f ms  %.1f G lane-ops/s  (%.2f lane-ops/clk/CU at 2.4 GHz)\n", mode, ms, ops / ms / 1e6,
           ops / (ms * 1e-3) / 2.4e9 / 256);
  }
  for (int mode = 4; mode < 6; ++mode) {
    hipLaunchKernelGGL(k_ldsi, dim3(blocks), dim3(256), 0, 0, (int*)out, 64, mode);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_ldsi, dim3(blocks), dim3(256), 0, 0, (int*)out, iters, mode);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double ops = (double)blocks * 256 * iters;
    printf("mode %d: %.3f ms  %.1f G lane-ops/s  (%.2f lane-ops/clk/CU at 2.4 GHz)\n", mode, ms, ops / ms / 1e6,
           ops / (ms * 1e-3) / 2.4e9 / 256);
  }
  hipLaunchKernelGGL(k_glb, dim3(blocks), dim3(256), 0, 0, buf, 64);
  hipEventRecord(a);
  hipLaunchKernelGGL(k_glb, dim3(blocks), dim3(256), 0, 0, buf, 512);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double ops = (double)blocks * 256 * 512;
  printf("global f32 atomics: %.3f ms  %.1f G lane-ops/s = %.0f GB/s added\n", ms, ops / ms / 1e6, ops * 4 / ms / 1e6);
  return 0;
}
