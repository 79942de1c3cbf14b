// Weight (and bias) gradient of a token-major Linear: dW[o, i] = sum_t gY[t, o] X[t, i],
// db[o] = sum_t gY[t, o], for the token-heavy Linears of the Swin blocks and the pixel
// decoder (qkv, proj, fc1, fc2; the encoder's value / output / offset
// projections and FFN).
//
// The reduction runs over tokens -- the strided dimension of both operands.  The vendor path
// was a batched GEMM over token chunks with f32 outputs (hipBLASLt, ~0.3 PF/s at these
// shapes: 105 launches, 4.4 ms of the C2 step) + a sum of the chunks + a separate column-sum
// pass for the bias.  Here one kernel streams 64-token chunks: the gY and X chunk tiles are
// staged by LDS-DMA in their natural [token][feature] layout (lds_dma.h images: 256-B rows,
// XOR-swizzled chunks) and read as MFMA operands with the transposed read ds_read_b64_tr_b16
// (k = token runs down the rows).  A workgroup owns BO output rows x 128 input columns of dW
// for one split of the tokens; the bias gradient rides along as one more MFMA per o-tile with
// an all-ones A operand (its every row = the column sums of gY) in the workgroups of the first
// input block.  Per-split f32 partials are summed in a fixed order by a second kernel that
// writes dW / db in the parameter dtype (deterministic, no atomics).
#include <stdlib.h>

#include "lds_dma.h"

namespace vs {
namespace {

constexpr int kTok = 64;     // tokens per chunk
constexpr int kBI = 128;     // input columns per workgroup

// BO output rows (128 or 256) per workgroup, 8 waves: wave w takes rows (w & 3) BO / 4 and
// input columns (w >> 2) 64 (2 x (BO / 128) MFMA tiles); part [S][N][K], pbias [S][N]
template <int BO>
__global__ void __launch_bounds__(512) token_wgrad_kernel(const bf16* __restrict__ gy, const bf16* __restrict__ x,
                                                          float* __restrict__ part, float* __restrict__ pbias, int T,
                                                          int N, int K, long long ldg, long long ldx, int S) {
  constexpr int NH = BO / 128;                          // gY half-images of 128 columns
  constexpr int GYB = NH * kTok * 256, XB = kTok * 256, STG = GYB + XB;
  constexpr int NBLK = STG / 1024;                      // 1-KB DMA blocks per stage
  constexpr int TO = BO / 128;                          // o-tiles (32 rows) per wave
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * STG];
  const int tiles_o = (N + BO - 1) / BO, tiles_i = (K + kBI - 1) / kBI, tiles = tiles_o * tiles_i;
  const int wg = xcd_swizzle(blockIdx.x, S * tiles);
  const int s = wg / tiles, tile = wg - s * tiles;      // a split's tiles are neighbours (one XCD)
  const int ob = tile / tiles_i, ib = tile - ob * tiles_i;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int wo = (w & 3) * (BO / 4), wi = (w >> 2) * 64;
  const long long nchunk = ((long long)T + kTok - 1) / kTok;
  const long long cb = nchunk * s / S, ce = nchunk * (s + 1) / S;
  const bool do_bias = pbias != nullptr && ib == 0 && wi == 0;

  auto issue = [&](long long c, int st) {
    unsigned char* base = smem + st * STG;
    for (int blk = w; blk < NBLK; blk += 8) {
      const unsigned char* src;
      if (blk < NH * 16) {
        const int half = blk >> 4, row = (blk & 15) * 4 + (l >> 4), ch = (l & 15) ^ img_swz(row);
        const long long t = c * kTok + row;
        const int col = ob * BO + half * 128 + ch * 8;
        src = (t < T && col < N) ? reinterpret_cast<const unsigned char*>(gy + t * ldg + col)
                                 : g_dma_zero_row + ch * 16;
      } else {
        const int row = (blk - NH * 16) * 4 + (l >> 4), ch = (l & 15) ^ img_swz(row);
        const long long t = c * kTok + row;
        const int col = ib * kBI + ch * 8;
        src = (t < T && col < K) ? reinterpret_cast<const unsigned char*>(x + t * ldx + col)
                                 : g_dma_zero_row + ch * 16;
      }
      glds16(src, base + blk * 1024);
    }
  };

  f32x16_t acc[TO][2], accb[TO];
#pragma unroll
  for (int a = 0; a < TO; ++a) {
    zero16(acc[a][0]);
    zero16(acc[a][1]);
    zero16(accb[a]);
  }
  const short one = (short)0x3f80;                      // bf16 1.0
  const bf16x8_t ones = {one, one, one, one, one, one, one, one};
  if (cb < ce) issue(cb, 0);
  for (long long c = cb; c < ce; ++c) {
    const int st = (int)((c - cb) & 1);
    wait_vm<0>();
    raw_barrier();
    if (c + 1 < ce) issue(c + 1, st ^ 1);
    const unsigned char* sg = smem + st * STG;
    const unsigned char* sx = sg + GYB;
#pragma unroll
    for (int k = 0; k < kTok / 16; ++k) {
      bf16x8_t a[2], b[TO];
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) a[ti] = tr_frag(sx, 16 * k, wi + 32 * ti, l);      // X^T: rows i
#pragma unroll
      for (int to = 0; to < TO; ++to) {
        const int oc = wo + 32 * to;                                                     // gY: cols o
        b[to] = tr_frag(sg + (oc >> 7) * (kTok * 256), 16 * k, oc & 127, l);
      }
#pragma unroll
      for (int to = 0; to < TO; ++to) {
#pragma unroll
        for (int ti = 0; ti < 2; ++ti) acc[to][ti] = mfma16(a[ti], b[to], acc[to][ti]);
        if (do_bias) accb[to] = mfma16(ones, b[to], accb[to]);
      }
    }
  }
  // C[i][o]: lane column = o, registers = 4 groups of 4 consecutive i
#pragma unroll
  for (int to = 0; to < TO; ++to) {
    const int o = ob * BO + wo + 32 * to + r;
    if (o >= N) continue;
    float* prow = part + ((size_t)s * N + o) * K;
#pragma unroll
    for (int ti = 0; ti < 2; ++ti) {
      const int i0 = ib * kBI + wi + 32 * ti + 4 * hh;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i = i0 + 8 * g;
        if (i < K)
          *reinterpret_cast<float4*>(prow + i) =
              make_float4(acc[to][ti][4 * g], acc[to][ti][4 * g + 1], acc[to][ti][4 * g + 2], acc[to][ti][4 * g + 3]);
      }
    }
    if (do_bias && hh == 0) pbias[(size_t)s * N + o] = accb[to][0];
  }
}

// dW[n] = sum_s part[s][n] (n < N K, 4 per thread), then db[o] = sum_s pbias[s][o]: fixed order
template <typename T>
__global__ void __launch_bounds__(256) token_wgrad_reduce_kernel(const float* __restrict__ part,
                                                                 const float* __restrict__ pbias, T* __restrict__ dw,
                                                                 T* __restrict__ db, long long nw, int N, int S) {
  const long long q = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long nq = nw / 4;
  if (q < nq) {
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = 0; s < S; ++s) {
      const float4 v = *reinterpret_cast<const float4*>(part + s * nw + 4 * q);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    T* d = dw + 4 * q;
    d[0] = from_f32<T>(a.x);
    d[1] = from_f32<T>(a.y);
    d[2] = from_f32<T>(a.z);
    d[3] = from_f32<T>(a.w);
  } else if (db && q - nq < N) {
    const int o = (int)(q - nq);
    float a = 0.f;
    for (int s = 0; s < S; ++s) a += pbias[(size_t)s * N + o];
    db[o] = from_f32<T>(a);
  }
}

int wgrad_bo(int N) { return N > 128 ? 256 : 128; }

int wgrad_splits(long long T, int N, int K) {
  const int BO = wgrad_bo(N);
  const long long tiles = (long long)((N + BO - 1) / BO) * ((K + kBI - 1) / kBI);
  const long long nchunk = (T + kTok - 1) / kTok;
  static const int target = [] {
    const char* e = getenv("VS_WGRAD_WGS");
    return e ? atoi(e) : 256;
  }();
  long long S = target / tiles;                        // ~one workgroup per CU (96 KB of LDS)
  // at least 4 chunks a split: the per-split f32 partial block costs about as much traffic
  // as 4 chunks of the operands
  if (S > nchunk / 4) S = nchunk / 4;
  if (S < 1) S = 1;
  return (int)S;
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" long long vs_token_wgrad_workspace_bytes(long long tokens, int N, int K) {
  if (tokens <= 0 || N <= 0 || K <= 0) return 0;
  const long long S = wgrad_splits(tokens, N, K);
  return S * ((long long)N * K + N) * 4;
}

extern "C" int vs_token_wgrad(int dtype, const void* grad_y, long long ld_grad_y, const void* x, long long ld_x,
                              void* dw, void* db, void* workspace, long long tokens, int N, int K, void* stream) {
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype (of dw / db) must be VS_F32 or VS_BF16");
  VS_CHECK(grad_y && x && dw && workspace, "null pointer");
  VS_CHECK(tokens > 0 && tokens < (1ll << 31) && N > 0 && K > 0 && N % 8 == 0 && K % 8 == 0,
           "0 < tokens < 2^31, N % 8 == 0, K % 8 == 0");
  VS_CHECK(ld_grad_y >= N && ld_x >= K && ld_grad_y % 8 == 0 && ld_x % 8 == 0, "row strides: >= width, % 8 == 0");
  VS_CHECK(((uintptr_t)grad_y & 15) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)workspace & 15) == 0,
           "grad_y / x / workspace must be 16-B aligned");
  const int S = wgrad_splits(tokens, N, K);
  const int BO = wgrad_bo(N);
  const long long tiles = (long long)((N + BO - 1) / BO) * ((K + kBI - 1) / kBI);
  VS_CHECK(S * tiles < (1ll << 31), "too many workgroups");
  float* part = (float*)workspace;
  float* pb = db ? part + (size_t)S * N * K : nullptr;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g((unsigned)(S * tiles));
  if (BO == 256)
    hipLaunchKernelGGL(token_wgrad_kernel<256>, g, dim3(512), 0, st, (const bf16*)grad_y, (const bf16*)x, part, pb,
                       (int)tokens, N, K, ld_grad_y, ld_x, S);
  else
    hipLaunchKernelGGL(token_wgrad_kernel<128>, g, dim3(512), 0, st, (const bf16*)grad_y, (const bf16*)x, part, pb,
                       (int)tokens, N, K, ld_grad_y, ld_x, S);
  VS_LAUNCH_CHECK();
  const long long nw = (long long)N * K;
  const long long items = nw / 4 + (db ? N : 0);
  const dim3 gr((unsigned)((items + 255) / 256));
  if (dtype == VS_BF16)
    hipLaunchKernelGGL(token_wgrad_reduce_kernel<bf16>, gr, dim3(256), 0, st, part, pb, (bf16*)dw, (bf16*)db, nw, N, S);
  else
    hipLaunchKernelGGL(token_wgrad_reduce_kernel<float>, gr, dim3(256), 0, st, part, pb, (float*)dw, (float*)db, nw,
                       N, S);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
