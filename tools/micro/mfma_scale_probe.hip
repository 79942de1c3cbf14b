// Operand-layout probe for v_mfma_scale_f32_32x32x64_f8f6f4 with e4m3 A/B (CBSZ = BLGP = 0)
// and per-lane e8m0 scales, exact small-integer data vs a host product.
//   k map (A and B alike): lane l holds A[row l&31][k(l, j)] in byte j of 8 dwords,
//   B[k(l, j)][col l&31]; candidate k maps below.  Scale: lane l's byte 0 scales row / col
//   l&31 for the k block that candidate assigns it.  C/D as v_mfma_f32_32x32x16_bf16.
// Experiments: unit scales (layout only), then per-lane random scales.
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

static int kmap(int hyp, int l, int j) {
  const int hh = l >> 5;
  switch (hyp) {
    case 0: return 32 * hh + j;                              // halves of 32
    case 1: return 16 * (j >> 4) * 2 + 16 * hh + (j & 15);   // 16-chunks interleaved: k = 32 (j>>4) + 16 hh + (j&15)
    case 2: return 16 * (j >> 3) + 8 * hh + (j & 7);         // 8-chunks interleaved
    default: return 8 * (j >> 2) + 4 * hh + (j & 3);         // 4-chunks interleaved
  }
}

int main() {
  unsigned char ha[64 * 32], hb[64 * 32];
  int ia[64 * 32], ib[64 * 32], hsa[64], hsb[64];
  unsigned char *da, *db;
  int *dsa, *dsb;
  float* dd;
  (void)hipMalloc(&da, 2048); (void)hipMalloc(&db, 2048); (void)hipMalloc(&dsa, 256); (void)hipMalloc(&dsb, 256);
  (void)hipMalloc(&dd, 4096);
  srand(7);
  for (int i = 0; i < 2048; ++i) {
    ia[i] = rand() % 13;
    ib[i] = rand() % 13;
    ha[i] = kCodes[ia[i]];
    hb[i] = kCodes[ib[i]];
  }
  (void)hipMemcpy(da, ha, 2048, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, hb, 2048, hipMemcpyHostToDevice);
  int rc = 1;
  for (int exp = 0; exp < 2; ++exp) {
    for (int l = 0; l < 64; ++l) {
      hsa[l] = exp ? 125 + rand() % 5 : 127;
      hsb[l] = exp ? 125 + rand() % 5 : 127;
    }
    (void)hipMemcpy(dsa, hsa, 256, hipMemcpyHostToDevice);
    (void)hipMemcpy(dsb, hsb, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
    float hd[64 * 16];
    (void)hipMemcpy(hd, dd, 4096, hipMemcpyDeviceToHost);
    for (int hyp = 0; hyp < 4; ++hyp)
      for (int sm = 0; sm < 2; ++sm) {         // scale block of lane l: sm 0 = l >> 5; sm 1 = block of k
        static double Af[32][64], Bf[64][32];
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 32; ++j) {
            const int kk = kmap(hyp, l, j);
            const int blkA = sm ? kk >> 5 : l >> 5;
            // the lane whose scale covers (row, block): row l&31, block blkA
            const int sla = (l & 31) + 32 * blkA;
            Af[l & 31][kk] = kVals[ia[l * 32 + j]] * ldexp(1.0, hsa[sla] - 127);
            Bf[kk][l & 31] = kVals[ib[l * 32 + j]] * ldexp(1.0, hsb[sla] - 127);
          }
        double err = 0, mag = 0;
        for (int l = 0; l < 64; ++l)
          for (int i = 0; i < 16; ++i) {
            const int col = l & 31, row = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5);
            double ref = 0;
            for (int kk = 0; kk < 64; ++kk) ref += Af[row][kk] * Bf[kk][col];
            err = fmax(err, fabs(ref - hd[l * 16 + i]));
            mag = fmax(mag, fabs(ref));
          }
        const bool ok = err <= 1e-5 * mag;
        printf("%s scales, k map %d, scale block %s: max|err| %.3g (max|ref| %.3g)%s\n", exp ? "random" : "unit",
               hyp, sm ? "by k" : "by lane half", err, mag, ok ? "  <-- MATCH" : "");
        if (exp == 1 && ok && hyp == 0 && sm == 0) rc = 0;
      }
  }
  return rc;
}
