// Operand-layout probe for v_mfma_scale_f32_32x32x64_f8f6f4 with e4m3 A/B (CBSZ = BLGP = 0)
// and per-lane e8m0 scales: exact small-integer data, checked against a host product
// under the hypothesised layout (prints the max error per hypothesis).
//   H: lane l holds A[row l&31][k = 32 (l>>5) + j] in byte j of its 8 dwords and
//      B[k = 32 (l>>5) + j][col l&31]; scale_a (byte 0) of lane l scales A's row l&31,
//      k-block l>>5; scale_b likewise for B's column; C/D as v_mfma_f32_32x32x16_bf16.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ void k(const unsigned char* a, const unsigned char* b, const int* sa, const int* sb, float* d) {
  const int l = threadIdx.x;
  v8i A, B;
  memcpy(&A, a + l * 32, 32);
  memcpy(&B, b + l * 32, 32);
  v16f C = {};
  C = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, C, 0, 0, 0, sa[l], 0, sb[l]);
  for (int i = 0; i < 16; ++i) d[l * 16 + i] = C[i];
}

static const float kVals[13] = {-4, -3, -2, -1.5f, -1, -0.5f, 0, 0.5f, 1, 1.5f, 2, 3, 4};
static const unsigned char kCodes[13] = {0xC8, 0xC4, 0xC0, 0xBC, 0xB8, 0xB0, 0x00, 0x30, 0x38, 0x3C, 0x40, 0x44, 0x48};

int main() {
  float Af[32][64], Bf[64][32];
  unsigned char ha[64 * 32], hb[64 * 32];
  int hsa[64], hsb[64];
  srand(7);
  for (int l = 0; l < 64; ++l) {
    hsa[l] = 125 + rand() % 5;
    hsb[l] = 125 + rand() % 5;
    for (int j = 0; j < 32; ++j) {
      int ia = rand() % 13, ib = rand() % 13;
      ha[l * 32 + j] = kCodes[ia];
      hb[l * 32 + j] = kCodes[ib];
      Af[l & 31][32 * (l >> 5) + j] = kVals[ia] * ldexpf(1.f, hsa[l] - 127);
      Bf[32 * (l >> 5) + j][l & 31] = kVals[ib] * ldexpf(1.f, hsb[l] - 127);
    }
  }
  unsigned char *da, *db;
  int *dsa, *dsb;
  float* dd;
  hipMalloc(&da, 2048); hipMalloc(&db, 2048); hipMalloc(&dsa, 256); hipMalloc(&dsb, 256); hipMalloc(&dd, 4096);
  hipMemcpy(da, ha, 2048, hipMemcpyHostToDevice);
  hipMemcpy(db, hb, 2048, hipMemcpyHostToDevice);
  hipMemcpy(dsa, hsa, 256, hipMemcpyHostToDevice);
  hipMemcpy(dsb, hsb, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
  float hd[64 * 16];
  hipMemcpy(hd, dd, 4096, hipMemcpyDeviceToHost);
  double err = 0, mag = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 16; ++i) {
      const int col = l & 31, row = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5);
      double ref = 0;
      for (int kk = 0; kk < 64; ++kk) ref += (double)Af[row][kk] * Bf[kk][col];
      err = fmax(err, fabs(ref - hd[l * 16 + i]));
      mag = fmax(mag, fabs(ref));
    }
  printf("mfma_scale 32x32x64 e4m3 layout hypothesis: max|err| %.3g (max|ref| %.3g) -> %s\n", err, mag,
         err <= 1e-5 * mag ? "CONFIRMED" : "WRONG");
  return err <= 1e-5 * mag ? 0 : 1;
}
