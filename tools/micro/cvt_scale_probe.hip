// Semantics probe for gfx950's scaled fp8 conversions vs the unscaled ones:
//   v_cvt_scalef32_pk_fp8_bf16 (bf16 pair -> e4m3 pair, with an f32 scale)
//   v_cvt_scalef32_pk_bf16_fp8 (e4m3 pair -> bf16 pair, with an f32 scale)
// against v_cvt_pk_fp8_f32 of x * 2^k / x * 2^-k, for scales 2^k, k in {-3, 0, 5}, over
// every bf16 value of |x| in [2^-20, 448 * 2^5] (both signs): prints the rule each
// direction follows (multiply or divide by the scale) and any mismatch.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

typedef short v2s __attribute__((ext_vector_type(2)));
typedef __bf16 v2bf __attribute__((ext_vector_type(2)));

__global__ void conv(const unsigned short* x, int n, float scale, int* out_scaled, int* out_mul, int* out_div,
                     unsigned short* back_scaled) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  unsigned short a = x[2 * i], b = x[2 * i + 1];
  v2bf src;
  const unsigned int ab = (unsigned int)a | ((unsigned int)b << 16);
  __builtin_memcpy(&src, &ab, 4);
  v2s old = {0, 0};
  v2s r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(old, src, scale, false);
  int rs;
  __builtin_memcpy(&rs, &r, 4);
  out_scaled[i] = rs & 0xffff;
  float fa, fb;
  unsigned int ua = (unsigned int)a << 16, ub = (unsigned int)b << 16;
  __builtin_memcpy(&fa, &ua, 4);
  __builtin_memcpy(&fb, &ub, 4);
  out_mul[i] = __builtin_amdgcn_cvt_pk_fp8_f32(fa * scale, fb * scale, 0, false) & 0xffff;
  out_div[i] = __builtin_amdgcn_cvt_pk_fp8_f32(fa / scale, fb / scale, 0, false) & 0xffff;
  v2bf back = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((unsigned)(rs & 0xffff), scale, false);
  __builtin_memcpy(&back_scaled[2 * i], &back, 4);
}

static float bf(unsigned short h) {
  unsigned int u = (unsigned int)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

#define CK(x) (void)(x)
int main() {
  std::vector<unsigned short> xs;
  for (unsigned int h = 0; h < 0x8000; ++h) {
    const float f = bf((unsigned short)h);
    if (f >= 0x1p-20f && f <= 448.f * 32.f) {
      xs.push_back((unsigned short)h);
      xs.push_back((unsigned short)(h | 0x8000));
    }
  }
  const int n = (int)xs.size(), np = n / 2;
  unsigned short *dx, *dback;
  int *ds, *dm, *dd;
  CK(hipMalloc(&dx, n * 2));
  CK(hipMalloc(&dback, n * 2));
  CK(hipMalloc(&ds, np * 4));
  CK(hipMalloc(&dm, np * 4));
  CK(hipMalloc(&dd, np * 4));
  CK(hipMemcpy(dx, xs.data(), n * 2, hipMemcpyHostToDevice));
  std::vector<int> hs(np), hm(np), hd(np);
  std::vector<unsigned short> hb(n);
  for (int k : {-3, 0, 5}) {
    const float sc = k < 0 ? 1.f / (float)(1 << -k) : (float)(1 << k);
    hipLaunchKernelGGL(conv, dim3((np + 255) / 256), dim3(256), 0, 0, dx, n, sc, ds, dm, dd, dback);
    CK(hipMemcpy(hs.data(), ds, np * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hm.data(), dm, np * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hd.data(), dd, np * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), dback, n * 2, hipMemcpyDeviceToHost));
    int eq_mul = 0, eq_div = 0, inrange = 0, eq_mul_in = 0, eq_div_in = 0, back_mul = 0, back_div = 0;
    for (int i = 0; i < np; ++i) {
      eq_mul += hs[i] == hm[i];
      eq_div += hs[i] == hd[i];
      const float fa = bf(xs[2 * i]);
      const bool in_mul = fabsf(fa * sc) <= 448.f && fabsf(bf(xs[2 * i + 1]) * sc) <= 448.f;
      const bool in_div = fabsf(fa / sc) <= 448.f && fabsf(bf(xs[2 * i + 1]) / sc) <= 448.f;
      inrange += in_mul;
      eq_mul_in += in_mul && hs[i] == hm[i];
      eq_div_in += in_div && hs[i] == hd[i];
    }
    // decode: the bf16 back values vs e4m3 byte value times / divided by scale
    for (int i = 0; i < np; ++i)
      for (int e = 0; e < 2; ++e) {
        const unsigned byte = (hs[i] >> (8 * e)) & 0xff;
        const int s = byte >> 7, ex = (byte >> 3) & 15, m = byte & 7;
        float v = ex ? ldexpf(1.f + m / 8.f, ex - 7) : ldexpf(m / 8.f, -6);
        if (s) v = -v;
        if ((byte & 0x7f) == 0x7f) continue;      // NaN code
        back_mul += bf(hb[2 * i + e]) == v * sc;
        back_div += bf(hb[2 * i + e]) == v / sc;
      }
    printf("k=%+d: pk_fp8_bf16(x, 2^k) == cvt(x*2^k) %d/%d (in-range %d/%d), == cvt(x/2^k) %d/%d (in-range matches %d); "
           "pk_bf16_fp8: == e4m3*2^k %d, == e4m3/2^k %d of %d\n",
           k, eq_mul, np, eq_mul_in, inrange, eq_div, np, eq_div_in, back_mul, back_div, n);
  }
  return 0;
}
