// Token GEMM: Y[M, N] = X[M, K] W[N, K]^T + b for the token-heavy Linears of the Swin
// blocks (qkv, proj, fc1, fc2), hand-written for gfx950 so that
//   * the MLP's GELU (exact erf, HF `gelu`) runs in the GEMM epilogue: fc1 stores the
//     pre-activation (the backward's input) and the activation in one pass, no separate
//     elementwise kernel reading the pre-activation back (hipBLASLt's GELU epilogue is the
//     tanh approximation, not HF's);
//   * config C5's fp8 path puts the Linears -- 96 % of a Swin-L block's FLOPs -- on the
//     block-scaled MX MFMA v_mfma_scale_f32_32x32x64_f8f6f4 (2x the bf16 MFMA rate) with
//     e4m3 operands and one e8m0 scale per 32 elements along K (vs_mx_quantize).
//
// Both operands are K-contiguous rows ("NT"), the MFMA fragments' own layout.  The kernel
// computes C^T = W X^T tile by tile (rows = output features on the registers, columns =
// tokens on the lanes), so a lane's 16 accumulators are 4 groups of 4 consecutive
// features of ONE token: the epilogue stores 8-byte row segments.
//
// Workgroup: 256 threads (4 waves, 2 x 2), tile 128 tokens x 128 features, one K-step =
// 128 bytes of each row (64 bf16 or 128 e4m3 elements).  X and W tiles are staged by
// LDS-DMA (global_load_lds_dwordx4: no VGPR round trip) into two buffers, the next K-step
// in flight while the current one is multiplied; a counted s_waitcnt vmcnt and raw
// s_barrier keep the DMA in flight across the barrier (cdna_hip_programming.md §5
// "Pipelining across barriers").  LDS rows are 128 B with the 16-B chunks XOR-swizzled by
// (row >> 1) & 7, so the fragment reads (ds_read_b128, 16-lane groups) are conflict-free;
// the DMA writes lane-linear and the swizzle is applied to the global source address.
// fp8: the per-row block scales of the K-step (4 bytes a row) are staged by 4-byte DMA.
#include "mfma_util.h"
#include "mx_util.h"

namespace vs {
namespace {

constexpr int kBM = 128, kBN = 128, kRowB = 128;      // tile tokens, tile features, bytes per K-step row
constexpr int kTileB = 128 * kRowB;                   // one staged operand tile (16 KB)

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (lds_void*)lds_wave_base, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (lds_void*)lds_wave_base, 4, 0, 0);
}

// physical byte offset of (row, 16-B chunk) in a staged tile
__device__ __forceinline__ int tile_off(int row, int chunk) { return row * kRowB + ((chunk ^ ((row >> 1) & 7)) << 4); }

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ float gelu_erf(float z) { return 0.5f * z * (1.f + erff(z * 0.70710678118654752f)); }

// EPI: 0 = bias, 1 = bias + GELU (y2 = pre-activation, y = gelu)
template <bool F8, int EPI>
__global__ void __launch_bounds__(256, 2) token_gemm_kernel(const unsigned char* __restrict__ X,
                                                            const unsigned char* __restrict__ Xs,
                                                            const unsigned char* __restrict__ Wt,
                                                            const unsigned char* __restrict__ Ws,
                                                            const bf16* __restrict__ bias, bf16* __restrict__ Y,
                                                            bf16* __restrict__ Y2, int M, int N, int K) {
  // [stage][X tile | W tile] then (fp8) [stage][X scales | W scales] (128 rows x 4 B each)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * 2 * kTileB + (F8 ? 2 * 2 * 512 : 0)];
  constexpr int ESZ = F8 ? 1 : 2;                      // bytes per element
  const int rowB = K * ESZ;                            // bytes per operand row
  const int nks = (rowB + kRowB - 1) / kRowB;          // K-steps (a partial last step is zero-filled)
  const int tilesM = (M + kBM - 1) / kBM, tilesN = (N + kBN - 1) / kBN;
  const int wg = xcd_swizzle(blockIdx.x, tilesM * tilesN);
  // N-tiles of one token tile are neighbours: the X tile is re-read from L2
  const int tm = wg / tilesN, tn = wg - tm * tilesN;
  const int m0 = tm * kBM, n0 = tn * kBN;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int wm = w & 1, wn = w >> 1;                   // this wave: tokens wm*64.., features wn*64..

  // ---- DMA issue of K-step ks into stage st: every wave moves 4 x 1 KB of X and of W
  // (8 rows per instruction, lane L -> row 8j + L/8, physical chunk L%8)
  auto issue = [&](int ks, int st) {
    unsigned char* sx = smem + st * 2 * kTileB;
    unsigned char* sw = sx + kTileB;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = (w * 4 + j) * 8 + (l >> 3);
      const int chunk = (l & 7) ^ ((row >> 1) & 7);
      const int kb = min(ks * kRowB + chunk * 16, rowB - 16);   // past K: any valid bytes, zeroed later
      const int mr = min(m0 + row, M - 1), nr = min(n0 + row, N - 1);
      glds16(X + (size_t)mr * rowB + kb, sx + (w * 4 + j) * 1024);
      glds16(Wt + (size_t)nr * rowB + kb, sw + (w * 4 + j) * 1024);
    }
    if (F8) {                                         // scales: waves 0-1 X rows, waves 2-3 W rows
      unsigned char* ss = smem + 2 * 2 * kTileB + st * 1024;
      const int sb = K / 32;                          // scale bytes per row
      const int row = (w & 1) * 64 + l;
      if (w < 2) glds4(Xs + (size_t)min(m0 + row, M - 1) * sb + ks * 4, ss + (w & 1) * 256);
      else glds4(Ws + (size_t)min(n0 + row, N - 1) * sb + ks * 4, ss + 512 + (w & 1) * 256);
    }
  };
  constexpr int kIssued = F8 ? 9 : 8;                 // DMA instructions per wave per K-step

  f32x16_t acc[2][2];                                 // [feature tile][token tile]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) zero16(acc[a][b]);

  issue(0, 0);
  for (int ks = 0; ks < nks; ++ks) {
    const int st = ks & 1;
    if (ks + 1 < nks) {
      issue(ks + 1, st ^ 1);
      wait_vm<kIssued>();                             // this wave's DMA of step ks landed
    } else {
      wait_vm<0>();
    }
    raw_barrier();                                    // every wave's DMA of step ks landed
    const unsigned char* sx = smem + st * 2 * kTileB;
    const unsigned char* sw = sx + kTileB;
    if (ks * kRowB + kRowB > rowB) {                  // partial last step: zero the bytes past K
      unsigned char* sxz = const_cast<unsigned char*>(sx);
      for (int idx = threadIdx.x; idx < 2 * 128 * 8; idx += 256) {
        const int op = idx >> 10, row = (idx >> 3) & 127, chunk = idx & 7;
        if (ks * kRowB + chunk * 16 >= rowB)
          *reinterpret_cast<uint4*>(sxz + op * kTileB + tile_off(row, chunk)) = make_uint4(0, 0, 0, 0);
      }
      raw_barrier();
    }
    if (F8) {
      const unsigned* ss = reinterpret_cast<const unsigned*>(smem + 2 * 2 * kTileB + st * 1024);
      unsigned xsc[2], wsc[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        xsc[t] = ss[wm * 64 + t * 32 + r];
        wsc[t] = ss[128 + wn * 64 + t * 32 + r];
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {                // two 64-element MX steps per K-step
        i32x8_t xa[2], wa[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int xr = wm * 64 + t * 32 + r, wr = wn * 64 + t * 32 + r;
          const uint4 x0 = *reinterpret_cast<const uint4*>(sx + tile_off(xr, 4 * kk + hh));
          const uint4 x1 = *reinterpret_cast<const uint4*>(sx + tile_off(xr, 4 * kk + 2 + hh));
          const uint4 w0 = *reinterpret_cast<const uint4*>(sw + tile_off(wr, 4 * kk + hh));
          const uint4 w1 = *reinterpret_cast<const uint4*>(sw + tile_off(wr, 4 * kk + 2 + hh));
          xa[t] = i32x8_t{(int)x0.x, (int)x0.y, (int)x0.z, (int)x0.w, (int)x1.x, (int)x1.y, (int)x1.z, (int)x1.w};
          wa[t] = i32x8_t{(int)w0.x, (int)w0.y, (int)w0.z, (int)w0.w, (int)w1.x, (int)w1.y, (int)w1.z, (int)w1.w};
        }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            acc[a][b] = mfma_mx(wa[a], (int)((wsc[a] >> (8 * (2 * kk + hh))) & 0xffu), xa[b],
                                (int)((xsc[b] >> (8 * (2 * kk + hh))) & 0xffu), acc[a][b]);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {                // four 16-element bf16 steps per K-step
        bf16x8_t xa[2], wa[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          xa[t] = *reinterpret_cast<const bf16x8_t*>(sx + tile_off(wm * 64 + t * 32 + r, 2 * kk + hh));
          wa[t] = *reinterpret_cast<const bf16x8_t*>(sw + tile_off(wn * 64 + t * 32 + r, 2 * kk + hh));
        }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) acc[a][b] = mfma16(wa[a], xa[b], acc[a][b]);
      }
    }
    raw_barrier();                                    // stage st free for the DMA of step ks + 2
  }

  // ---- epilogue: lane = token, registers = 4 groups of 4 consecutive features
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int m = m0 + wm * 64 + b * 32 + r;
    if (m >= M) continue;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + wn * 64 + a * 32 + 8 * g + 4 * hh;
        if (n >= N) continue;                         // N % 4 == 0: a group is all in or all out
        float z[4];
        const bf16x4_t bv = bias ? *reinterpret_cast<const bf16x4_t*>(bias + n) : bf16x4_t{0, 0, 0, 0};
#pragma unroll
        for (int e = 0; e < 4; ++e) z[e] = acc[a][b][4 * g + e] + bf16_bits_to_f32((unsigned short)bv[e]);
        bf16x4_t o;
        if (EPI == 1) {
          bf16x4_t pre;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            pre[e] = bf16_bits(z[e]);
            // GELU of the ROUNDED pre-activation: the value the backward (and an unfused
            // bf16 F.gelu) sees
            o[e] = bf16_bits(gelu_erf(bf16_bits_to_f32((unsigned short)pre[e])));
          }
          *reinterpret_cast<bf16x4_t*>(Y2 + (size_t)m * N + n) = pre;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = bf16_bits(z[e]);
        }
        *reinterpret_cast<bf16x4_t*>(Y + (size_t)m * N + n) = o;
      }
    }
  }
}

// bf16 rows [rows, K] -> e4m3 rows + one e8m0 scale byte per 32 elements (the largest
// power of two 2^k with amax 2^k <= 448; scale byte 127 - k), 4 lanes per block
__global__ void __launch_bounds__(256) mx_quantize_kernel(const bf16* __restrict__ x, unsigned char* __restrict__ q,
                                                          unsigned char* __restrict__ sc, long long nblk) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long blk = t >> 2;
  const bool in = blk < nblk;
  const bf16x8_t c = in ? *reinterpret_cast<const bf16x8_t*>(x + t * 8) : zero8();
  const unsigned am = umax_xor(umax_xor(amax8_bits(c), 1), 2);
  const int k = mx_exp_bits(am);
  const float inv = __builtin_ldexpf(1.f, -k);
  const uint4 u = bits128(c);
  if (in) {
    *reinterpret_cast<uint2*>(q + t * 8) = make_uint2((unsigned)e4m3x4(u.x, u.y, inv), (unsigned)e4m3x4(u.z, u.w, inv));
    if ((t & 3) == 0) sc[blk] = (unsigned char)(127 - k);
  }
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" int vs_mx_quantize(const void* x, void* q, void* scales, int rows, int K, void* stream) {
  VS_CHECK(x && q && scales, "null pointer");
  VS_CHECK(rows >= 0 && K > 0 && K % 32 == 0, "K must be a positive multiple of 32");
  const long long nblk = (long long)rows * (K / 32);
  if (nblk == 0) return VS_OK;
  const long long threads = nblk * 4;
  hipLaunchKernelGGL(mx_quantize_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)x, (unsigned char*)q, (unsigned char*)scales, nblk);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_token_gemm(int mode, const void* x, const void* x_scales, const void* w, const void* w_scales,
                             const void* bias, void* y, void* y_pre, int M, int N, int K, void* stream) {
  const bool f8 = (mode & VS_TGEMM_FP8) != 0, gelu = (mode & VS_TGEMM_GELU) != 0;
  VS_CHECK(x && w && y, "null pointer");
  VS_CHECK(M > 0 && N > 0 && K > 0, "empty GEMM");
  VS_CHECK(N % 4 == 0, "N must be a multiple of 4");
  VS_CHECK(f8 ? (K % 128 == 0 && x_scales && w_scales) : (K % 8 == 0), "fp8: K % 128 == 0 and scales; bf16: K % 8 == 0");
  VS_CHECK(!gelu || y_pre, "gelu needs the pre-activation output");
  const long long tiles = (long long)((M + kBM - 1) / kBM) * ((N + kBN - 1) / kBN);
  VS_CHECK(tiles < (1ll << 31), "too many tiles");
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)tiles), block(256);
#define VS_TG(F8_, E_)                                                                                           \
  hipLaunchKernelGGL((token_gemm_kernel<F8_, E_>), grid, block, 0, st, (const unsigned char*)x,                 \
                     (const unsigned char*)x_scales, (const unsigned char*)w, (const unsigned char*)w_scales,     \
                     (const bf16*)bias, (bf16*)y, (bf16*)y_pre, M, N, K)
  if (f8 && gelu) VS_TG(true, 1);
  else if (f8) VS_TG(true, 0);
  else if (gelu) VS_TG(false, 1);
  else VS_TG(false, 0);
#undef VS_TG
  VS_LAUNCH_CHECK();
  return VS_OK;
}
