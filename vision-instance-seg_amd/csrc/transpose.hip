// Batched transpose of small bf16 matrices: dst[c][r] = src[r][c] for a LIST of matrices in
// one launch.  The token Linears' input gradient dX = dY W runs on the token GEMM, whose
// operands are both K-contiguous rows, so it reads W^T [K, N]; the transposed copy of every
// such weight was one ATen strided-copy launch per Linear and step (53 per C2 step, ~6 us
// each).  The Python side (visionseg.linear._WeightTransposes) requests the copies in the
// forward and writes them all with this one launch at the first use in the backward.
//
// A workgroup transposes one 64 x 64 tile through LDS: 16-B row loads (8 bf16 of one source
// row), 16-B row stores (8 consecutive source rows of one column); rows % 8 == 0 and
// cols % 8 == 0 (the token Linears' N % 8 == 0, K % 8 == 0).
#include "common.h"

namespace vs {
namespace {

constexpr int kTT = 64;                          // tile edge
constexpr int kMaxItems = 64;                    // matrices per launch (kernel-argument space)

struct TrItem {
  const bf16* src;
  bf16* dst;
  int rows, cols;
  int tile0, tiles_c;                            // first tile of this matrix, tiles along cols
};

struct TrBatch {
  TrItem it[kMaxItems];
  int n;
};

__global__ void __launch_bounds__(256) transpose_batched_kernel(const TrBatch b) {
  __shared__ unsigned short tile[kTT][kTT + 2];  // +2: the column reads step 33 words a row
  const int t = blockIdx.x;
  int k = 0;
  for (int j = 1; j < b.n; ++j)
    if (t >= b.it[j].tile0) k = j;
  const TrItem& I = b.it[k];
  const int local = t - I.tile0;
  const int tr = local / I.tiles_c, tc = local - tr * I.tiles_c;
  const int r0 = tr * kTT, c0 = tc * kTT;
  // load: 64 rows x 8 chunks of 16 B, two per thread
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int idx = threadIdx.x + p * 256;
    const int row = idx >> 3, ch = idx & 7;
    const int r = r0 + row, c = c0 + ch * 8;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (r < I.rows && c < I.cols) v = *reinterpret_cast<const uint4*>(I.src + (size_t)r * I.cols + c);
    const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      tile[row][ch * 8 + 2 * e] = (unsigned short)(w[e] & 0xffffu);
      tile[row][ch * 8 + 2 * e + 1] = (unsigned short)(w[e] >> 16);
    }
  }
  __syncthreads();
  // store: dst row = source column (64 of them), 8 chunks of 8 source rows, two per thread
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int idx = threadIdx.x + p * 256;
    const int col = idx >> 3, ch = idx & 7;
    const int c = c0 + col, r = r0 + ch * 8;
    if (c < I.cols && r < I.rows) {
      unsigned w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        w[e] = (unsigned)tile[ch * 8 + 2 * e][col] | ((unsigned)tile[ch * 8 + 2 * e + 1][col] << 16);
      *reinterpret_cast<uint4*>(I.dst + (size_t)c * I.rows + r) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" int vs_transpose_batched(int dtype, const vs_transpose_item* items, int n, void* stream) {
  VS_CHECK(dtype == VS_BF16, "dtype must be VS_BF16");
  VS_CHECK(n >= 0 && (n == 0 || items), "null item list");
  hipStream_t st = (hipStream_t)stream;
  for (int base = 0; base < n; base += kMaxItems) {
    TrBatch b;
    b.n = std::min(kMaxItems, n - base);
    long long tiles = 0;
    for (int j = 0; j < b.n; ++j) {
      const vs_transpose_item& q = items[base + j];
      VS_CHECK(q.src && q.dst, "null pointer");
      VS_CHECK(q.rows > 0 && q.cols > 0 && q.rows % 8 == 0 && q.cols % 8 == 0, "rows % 8 == 0, cols % 8 == 0");
      VS_CHECK(((uintptr_t)q.src & 15) == 0 && ((uintptr_t)q.dst & 15) == 0, "src / dst must be 16-B aligned");
      VS_CHECK((long long)q.rows * q.cols < (1ll << 31), "matrix too large");
      TrItem& I = b.it[j];
      I.src = (const bf16*)q.src;
      I.dst = (bf16*)q.dst;
      I.rows = q.rows;
      I.cols = q.cols;
      I.tiles_c = (q.cols + kTT - 1) / kTT;
      I.tile0 = (int)tiles;
      tiles += (long long)((q.rows + kTT - 1) / kTT) * I.tiles_c;
    }
    VS_CHECK(tiles < (1ll << 31), "too many tiles");
    if (tiles == 0) continue;
    hipLaunchKernelGGL(transpose_batched_kernel, dim3((unsigned)tiles), dim3(256), 0, st, b);
    VS_LAUNCH_CHECK();
  }
  return VS_OK;
}
