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
#include <stdlib.h>

#include <algorithm>

#include "gelu_table.h"
#include "mfma_util.h"
#include "mx_util.h"

namespace vs {
namespace {

constexpr int kRowB = 128;                            // bytes of a row per K-step

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

// bf16 GELU (exact erf) of a bf16 value, branch-free: the generated table (gelu_table.h:
// f64 gelu rounded to bf16) for 2^-10 <= |x| < 16, x (0.5 + x / sqrt(2 pi)) below (the next
// term is 2^-30 relative), x resp. -0 above (Phi(-16) ~ 6e-58 underflows bf16); NaN stays NaN
__device__ __forceinline__ unsigned short gelu_bits(unsigned short pb, const unsigned short* tab) {
  const unsigned e = (pb >> 7) & 0xffu, sgn = pb >> 15;
  const int ti = min(max((int)(pb & 0x7fffu) - kGeluE0 * 128, 0), kGeluNE * 128 - 1) + (int)sgn * (kGeluNE * 128);
  const unsigned short tv = tab[ti];
  const float z = bf16_bits_to_f32(pb);
  const unsigned short small = (unsigned short)bf16_bits(z * (0.5f + 0.3989422804014327f * z));
  const unsigned short big = (sgn && (pb & 0x7fffu) <= 0x7f80u) ? (unsigned short)0x8000 : pb;
  return e < (unsigned)kGeluE0 ? small : (e >= (unsigned)(kGeluE0 + kGeluNE) ? big : tv);
}

// 8 bf16 of dH (the GEMM output, already rounded) times act'(8 bf16 activation inputs /
// outputs), each product rounded once: what the activation backward (norm.hip
// act_bwd_colsum_kernel) computes from the stored dH.  RELU: p is the ReLU's output (> 0
// exactly where its input is), else GELU's pre-activation.
template <bool RELU>
__device__ __forceinline__ float act_grad(float p) {
  return RELU ? (p > 0.f ? 1.f : 0.f) : gelu_grad_erf(p);
}
template <bool RELU>
__device__ __forceinline__ uint4 act_bwd8(uint4 d, uint4 p) {
  const unsigned dw[4] = {d.x, d.y, d.z, d.w}, pw[4] = {p.x, p.y, p.z, p.w};
  unsigned o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float lo = __uint_as_float(dw[i] << 16) * act_grad<RELU>(__uint_as_float(pw[i] << 16));
    const float hi = __uint_as_float(dw[i] & 0xffff0000u) * act_grad<RELU>(__uint_as_float(pw[i] & 0xffff0000u));
    o[i] = (unsigned)(unsigned short)bf16_bits(lo) | ((unsigned)(unsigned short)bf16_bits(hi) << 16);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// Tile shapes: GM x GN waves, each TM x TN MFMA tiles of 32 x 32 (tokens x features):
//   <2, 2, 2, 2>: 128 x 128, 256 threads, 2 workgroups / CU (64 KB of staging);
//   <2, 4, 4, 2>: 256 x 256, 512 threads, 1 workgroup / CU (128 KB): half the L2 -> LDS
//   bytes per flop, for the MFMA-bound shapes.
// EPI: 0 = bias, 1 = bias + GELU (y2 = pre-activation, y = gelu), 2 = as 1 and the GELU
// output also as MX fp8 (yq e4m3 [M, N] + yqs e8m0 [M, N/32]: the next GEMM's operand,
// bit-identical to vs_mx_quantize of y), 3 = GELU BACKWARD (the MLP's fc2 dX: y = bf16(x w^T)
// * gelu'(y2), y2 the saved pre-activation READ in the store loop; no bias): the activation
// backward's pass over dH (written, then read back with the pre-activation) is gone;
// 4 = ReLU backward (the encoder FFN: y2 = the ReLU output, y = bf16(x w^T) * [y2 > 0])
template <bool F8, int EPI, int GM, int GN, int TM, int TN>
__global__ void __launch_bounds__(64 * GM * GN) token_gemm_kernel(const unsigned char* __restrict__ X,
                                                                  const unsigned char* __restrict__ Xs,
                                                                  const unsigned char* __restrict__ Wt,
                                                                  const unsigned char* __restrict__ Ws,
                                                                  const bf16* __restrict__ bias, bf16* __restrict__ Y,
                                                                  bf16* __restrict__ Y2, unsigned char* __restrict__ YQ,
                                                                  unsigned char* __restrict__ YQS, int M, int N, int K) {
  constexpr int BM = GM * TM * 32, BN = GN * TN * 32, NW = GM * GN, NT = 64 * NW;
  constexpr int XB = BM * kRowB, WB = BN * kRowB, STB = XB + WB;      // staged bytes per K-step
  constexpr int SCB = F8 ? (BM + BN) * 4 : 0;                         // staged scale bytes per K-step
  constexpr bool GF = EPI == 1 || EPI == 2, GB = EPI == 3 || EPI == 4;   // GELU forward / act backward
  static_assert(!(GB && F8), "activation backward: bf16");
  // [stage][X tile | W tile] then (fp8) [stage][X scales | W scales] then the GELU table
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * STB + 2 * SCB + (GF ? kGeluEntries * 2 : 0)];
  unsigned short* sgelu = reinterpret_cast<unsigned short*>(smem + 2 * STB + 2 * SCB);
  constexpr int ESZ = F8 ? 1 : 2;                      // bytes per element
  const int rowB = K * ESZ;                            // bytes per operand row
  const int nks = (rowB + kRowB - 1) / kRowB;          // K-steps (a partial last step is zero-filled)
  const int tilesM = (M + BM - 1) / BM, tilesN = (N + BN - 1) / BN;
  const int wg = xcd_swizzle(blockIdx.x, tilesM * tilesN);
  // N-tiles of one token tile are neighbours: the X tile is re-read from L2
  const int tm = wg / tilesN, tn = wg - tm * tilesN;
  const int m0 = tm * BM, n0 = tn * BN;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int wm = w % GM, wn = w / GM;                  // this wave: tokens wm*TM*32.., features wn*TN*32..

  // ---- DMA issue of K-step ks into stage st: 1 KB (8 rows) per wave instruction, lane L ->
  // row 8j + L/8, physical chunk L%8; X rows first, then W rows, spread over the waves
  auto issue = [&](int ks, int st) {
    unsigned char* base = smem + st * STB;
    constexpr int NI = (BM + BN) / 8 / NW;            // instructions per wave
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int blk = w * NI + j;                     // 8-row block of the [X | W] image
      const int row = blk * 8 + (l >> 3);             // < BM: X row, else W row BM..
      const bool isx = row < BM;
      const int rr = isx ? row : row - BM;
      const int chunk = (l & 7) ^ ((rr >> 1) & 7);
      const int kb = min(ks * kRowB + chunk * 16, rowB - 16);   // past K: any valid bytes, zeroed later
      const unsigned char* src = isx ? X + (size_t)min(m0 + rr, M - 1) * rowB + kb
                                     : Wt + (size_t)min(n0 + rr, N - 1) * rowB + kb;
      glds16(src, base + blk * 1024);
    }
    if (F8) {                                         // scales: 4 bytes a row, 64 rows per instruction
      unsigned char* ss = smem + 2 * STB + st * SCB;
      const int sb = K / 32;                          // scale bytes per row
      for (int blk = w; blk < (BM + BN) / 64; blk += NW) {
        const int row = blk * 64 + l;
        const unsigned char* src = row < BM ? Xs + (size_t)min(m0 + row, M - 1) * sb + ks * 4
                                            : Ws + (size_t)min(n0 + row - BM, N - 1) * sb + ks * 4;
        glds4(src, ss + blk * 256);
      }
    }
  };

  f32x16_t acc[TN][TM];                               // [feature tile][token tile]
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) zero16(acc[a][b]);

  auto xrow = [&](int t) { return wm * TM * 32 + t * 32 + r; };
  auto wrow = [&](int t) { return wn * TN * 32 + t * 32 + r; };
  issue(0, 0);
  if (GF) {                                           // GELU table: read at the epilogue, after the loop's barriers
    for (int i = threadIdx.x; i < kGeluEntries / 8; i += NT)
      reinterpret_cast<uint4*>(sgelu)[i] = reinterpret_cast<const uint4*>(kGeluTable)[i];
  }
  // activation backward: this thread's pre-activation chunks of the output tile, requested
  // with the last K-step's operands (the 128 x 128 tile: 8 registers x 4; the 256 x 256
  // tile's 16 would not fit beside its accumulators -- it loads them after the staging)
  constexpr int SPL = (EPI < 2 || GB) ? BM * (BN / 8) / NT : 1;
  constexpr bool PEARLY = GB && SPL <= 8;
  uint4 pv[GB ? SPL : 1];
  auto load_pre = [&]() {
#pragma unroll
    for (int i = 0; i < SPL; ++i) {
      const int idx = threadIdx.x + i * NT, row = idx / (BN / 8), chunk = idx - (idx / (BN / 8)) * (BN / 8);
      const int m = m0 + row, n = n0 + chunk * 8;
      pv[i] = (m < M && n < N) ? *reinterpret_cast<const uint4*>(Y2 + (size_t)m * N + n) : make_uint4(0, 0, 0, 0);
    }
  };
  for (int ks = 0; ks < nks; ++ks) {
    const int st = ks & 1;
    wait_vm<0>();                                     // this wave's DMA of step ks landed
    raw_barrier();                                    // every wave's did; every wave is done with step ks - 1
    const unsigned char* sx = smem + st * STB;
    const unsigned char* sw = sx + XB;
    if (ks * kRowB + kRowB > rowB) {                  // partial last step: zero the bytes past K
      unsigned char* sz = const_cast<unsigned char*>(sx);
      for (int idx = threadIdx.x; idx < (BM + BN) * 8; idx += NT) {
        const int row = idx >> 3, chunk = idx & 7, rr = row < BM ? row : row - BM;
        if (ks * kRowB + chunk * 16 >= rowB)
          *reinterpret_cast<uint4*>(sz + (row < BM ? 0 : XB) + tile_off(rr, chunk)) = make_uint4(0, 0, 0, 0);
      }
      raw_barrier();
    }
    if (ks + 1 < nks) issue(ks + 1, st ^ 1);          // the other buffer: last read in step ks - 1
    else if (PEARLY) load_pre();
    if (F8) {
      const unsigned* ss = reinterpret_cast<const unsigned*>(smem + 2 * STB + st * SCB);
      unsigned xsc[TM], wsc[TN];
#pragma unroll
      for (int t = 0; t < TM; ++t) xsc[t] = ss[xrow(t)];
#pragma unroll
      for (int t = 0; t < TN; ++t) wsc[t] = ss[BM + wrow(t)];
      i32x8_t xa[2][TM], wa[2][TN];                  // [buffer][tile]
      auto ld2 = [&](const unsigned char* img, int row, int kk) {
        const uint4 v0 = *reinterpret_cast<const uint4*>(img + tile_off(row, 4 * kk + hh));
        const uint4 v1 = *reinterpret_cast<const uint4*>(img + tile_off(row, 4 * kk + 2 + hh));
        return i32x8_t{(int)v0.x, (int)v0.y, (int)v0.z, (int)v0.w, (int)v1.x, (int)v1.y, (int)v1.z, (int)v1.w};
      };
      auto load = [&](int kk, int bsel) {
#pragma unroll
        for (int t = 0; t < TM; ++t) xa[bsel][t] = ld2(sx, xrow(t), kk);
#pragma unroll
        for (int t = 0; t < TN; ++t) wa[bsel][t] = ld2(sw, wrow(t), kk);
      };
      load(0, 0);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {                // two 64-element MX steps per K-step
        if (kk + 1 < 2) load(kk + 1, (kk + 1) & 1);
        const int bs = kk & 1;
#pragma unroll
        for (int a = 0; a < TN; ++a)
#pragma unroll
          for (int b = 0; b < TM; ++b)
            acc[a][b] = mfma_mx(wa[bs][a], (int)((wsc[a] >> (8 * (2 * kk + hh))) & 0xffu), xa[bs][b],
                                (int)((xsc[b] >> (8 * (2 * kk + hh))) & 0xffu), acc[a][b]);
      }
    } else {
      bf16x8_t xa[2][TM], wa[2][TN];                 // [buffer][tile]
      auto load = [&](int kk, int bsel) {
#pragma unroll
        for (int t = 0; t < TM; ++t) xa[bsel][t] = *reinterpret_cast<const bf16x8_t*>(sx + tile_off(xrow(t), 2 * kk + hh));
#pragma unroll
        for (int t = 0; t < TN; ++t) wa[bsel][t] = *reinterpret_cast<const bf16x8_t*>(sw + tile_off(wrow(t), 2 * kk + hh));
      };
      load(0, 0);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {                // four 16-element bf16 steps per K-step
        if (kk + 1 < 4) load(kk + 1, (kk + 1) & 1);
        const int bs = kk & 1;
#pragma unroll
        for (int a = 0; a < TN; ++a)
#pragma unroll
          for (int b = 0; b < TM; ++b) acc[a][b] = mfma16(wa[bs][a], xa[bs][b], acc[a][b]);
      }
    }
  }

  if ((EPI < 2 || GB) && N % 8 == 0) {
    // ---- epilogue through LDS: the accumulators are 8-byte pieces of 32 token rows per
    // store instruction (32 lines touched for 512 B); staged in LDS as the [BM][BN] bf16
    // output tile (16-B chunks XOR-swizzled by row & 15: the 8-B writes of 16 rows and the
    // row-contiguous 16-B reads are conflict-free) and stored 16 B a lane, 256 B per row
    // segment (whole 128-B lines).  bias, then GELU: pass 0 writes y, pass 1 (GELU) y_pre.
    constexpr int NCK = BN / 8;                        // 16-B chunks per tile row
    auto so_off = [](int row, int chunk) { return row * (BN * 2) + ((chunk ^ (row & 15)) << 4); };
    raw_barrier();                                     // every wave is done with the staging buffers
#pragma unroll 1
    for (int pass = 0; pass < (GF ? 2 : 1); ++pass) {
#pragma unroll
      for (int b = 0; b < TM; ++b) {
        const int row = xrow(b);
#pragma unroll
        for (int a = 0; a < TN; ++a) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int f = wn * TN * 32 + a * 32 + 8 * g + 4 * hh, n = n0 + f;
            const bf16x4_t bv = (bias && n < N) ? *reinterpret_cast<const bf16x4_t*>(bias + n) : bf16x4_t{0, 0, 0, 0};
            bf16x4_t o;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const short pre = bf16_bits(acc[a][b][4 * g + e] + bf16_bits_to_f32((unsigned short)bv[e]));
              // GELU of the ROUNDED pre-activation: the value the backward (and an unfused
              // bf16 F.gelu) sees
              o[e] = (GF && pass == 0) ? (short)gelu_bits((unsigned short)pre, sgelu) : pre;
            }
            *reinterpret_cast<bf16x4_t*>(smem + so_off(row, f >> 3) + (f & 7) * 2) = o;
          }
        }
      }
      if (GB) {
        static_assert(!GB || SPL * NT == BM * NCK, "store split");
        if (!PEARLY) load_pre();                       // requested before the barrier
        raw_barrier();
#pragma unroll
        for (int i = 0; i < SPL; ++i) {
          const int idx = threadIdx.x + i * NT, row = idx / NCK, chunk = idx - (idx / NCK) * NCK;
          const int m = m0 + row, n = n0 + chunk * 8;
          if (m < M && n < N) {
            const uint4 dv = *reinterpret_cast<const uint4*>(smem + so_off(row, chunk));
            *reinterpret_cast<uint4*>(Y + (size_t)m * N + n) = act_bwd8<EPI == 4>(dv, pv[i]);
          }
        }
        return;
      }
      raw_barrier();
      bf16* out = pass == 0 ? Y : Y2;
      for (int idx = threadIdx.x; idx < BM * NCK; idx += NT) {
        const int row = idx / NCK, chunk = idx - (idx / NCK) * NCK;
        const int m = m0 + row, n = n0 + chunk * 8;
        if (m < M && n < N)
          *reinterpret_cast<uint4*>(out + (size_t)m * N + n) = *reinterpret_cast<const uint4*>(smem + so_off(row, chunk));
      }
      if (GF && pass == 0) raw_barrier();            // the tile is rewritten by pass 1
    }
    return;
  }
  // ---- direct epilogue (N % 8 != 0, or the MX fp8 output): lane = token, registers = 4
  // groups of 4 consecutive features
#pragma unroll
  for (int b = 0; b < TM; ++b) {
    const int m = m0 + xrow(b);
    bf16x4_t ov[TN][4];                                // EPI 2: this token's GELU outputs of the tile
    if (m >= M) continue;
#pragma unroll
    for (int a = 0; a < TN; ++a) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + wn * TN * 32 + a * 32 + 8 * g + 4 * hh;
        if (n >= N) continue;                         // N % 4 == 0: a group is all in or all out
        float z[4];
        const bf16x4_t bv = bias ? *reinterpret_cast<const bf16x4_t*>(bias + n) : bf16x4_t{0, 0, 0, 0};
#pragma unroll
        for (int e = 0; e < 4; ++e) z[e] = acc[a][b][4 * g + e] + bf16_bits_to_f32((unsigned short)bv[e]);
        bf16x4_t o;
        if (EPI >= 1) {
          bf16x4_t pre;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            pre[e] = bf16_bits(z[e]);
            // GELU of the ROUNDED pre-activation: the value the backward (and an unfused
            // bf16 F.gelu) sees
            o[e] = (short)gelu_bits((unsigned short)pre[e], sgelu);
          }
          *reinterpret_cast<bf16x4_t*>(Y2 + (size_t)m * N + n) = pre;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = bf16_bits(z[e]);
        }
        if (EPI == 2) ov[a][g] = o;
        *reinterpret_cast<bf16x4_t*>(Y + (size_t)m * N + n) = o;
      }
      if (EPI == 2) {
        // the 32-feature block of tile a is split between this lane (features 8g + 4hh +
        // 0..3) and its partner lane ^ 32: block amax with one exchange, then e4m3 at the
        // block's power-of-two scale (vs_mx_quantize's rule, the same bytes)
        const int nb = n0 + wn * TN * 32 + a * 32;
        unsigned am = 0;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint2 u = __builtin_bit_cast(uint2, ov[a][g]);
          am = max(am, max(max(u.x & 0x7fffu, (u.x >> 16) & 0x7fffu), max(u.y & 0x7fffu, (u.y >> 16) & 0x7fffu)));
        }
        am = max(am, (unsigned)__shfl_xor((int)am, 32, 64));
        const int k = mx_exp_bits(am);
        const float inv = __builtin_ldexpf(1.f, -k);
        if (nb < N) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const uint2 u = __builtin_bit_cast(uint2, ov[a][g]);
            s16x2_t q = {0, 0};
            q = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(q, __builtin_bit_cast(bf16x2v_t, u.x), inv, false);
            q = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(q, __builtin_bit_cast(bf16x2v_t, u.y), inv, true);
            *reinterpret_cast<int*>(YQ + (size_t)m * N + nb + 8 * g + 4 * hh) = __builtin_bit_cast(int, q);
          }
          if (hh == 0) YQS[(size_t)m * (N / 32) + nb / 32] = (unsigned char)(127 - k);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Streaming token GEMM for short rows (K <= 192: Swin-T stages 1-2, the C2 step's largest
// Linears by bytes).  There a 128 x 128 tile is 2-3 K-steps of work behind one DMA round trip
// and the store tail, so the tile kernel above ran these at 2-3 TB/s (the Linears are
// HBM-bound: 2 N + 2 K bytes per token for 2 N K flops).  Here a workgroup owns a 128-feature
// slice of W -- resident in LDS for the whole launch -- and STREAMS token tiles of BM rows
// through a ring of NBUF X buffers: the X rows of the next NBUF - 1 tiles are in flight
// (LDS-DMA) while the current tile is multiplied and its outputs are staged and stored, so
// HBM sees one continuous stream (one tile of prefetch was ~0.5 us of cover for ~1-2 us of
// latency).
//   * 4 waves, wave w = features 32w..32w+31 of the slice, all BM tokens (BM / 32 MFMA tiles);
//   * images as the tile kernel's (128-B K-steps, chunks XOR-swizzled by (row >> 1) & 7);
//     padding chunks past K are zeroed once and never loaded, sub-steps past K are skipped;
//   * epilogue as the tile kernel's: bias (+ GELU), staged as the [BM][128] bf16 tile, 16-B
//     row stores; a ring buffer is re-filled only after every wave has passed the barrier
//     that follows the last read of it.
// Counted waits: VMEM operations complete in issue order.  Tile j >= NBUF - 1 was requested in
// iteration j - NBUF + 1, so at the top of tile j the wait leaves exactly what was issued after
// it outstanding (NBUF - 1 tiles' stores and NBUF - 2 tiles' DMA); near the end of the
// sequence, where fewer were issued, it waits for everything; the first NBUF - 1 tiles were
// waited for after the prologue.
template <int EPI, int NKS, int TM, int NBUF>
__global__ void __launch_bounds__(256, 2) token_gemm_stream_kernel(const bf16* __restrict__ X, const bf16* __restrict__ Wt,
                                                                   const bf16* __restrict__ bias, bf16* __restrict__ Y,
                                                                   bf16* __restrict__ Y2, int M, int N, int K) {
  constexpr int BM = 32 * TM, BN = 128, NT = 256;
  constexpr int WIMG = BN * kRowB, XIMG = BM * kRowB;                 // bytes per K-step image
  constexpr int WB = NKS * WIMG, XB = NKS * XIMG, OB = BM * BN * 2;
  constexpr int NCK = BN / 8;                                          // 16-B chunks per output row
  constexpr int SPT = BM * NCK / NT;                                   // output stores per thread and pass
  constexpr int XI = BM / 8 * NKS / 4;                                 // X DMA instructions per wave
  static_assert(SPT * NT == BM * NCK && XI * 4 * 8 == BM * NKS, "tile shape");
  constexpr bool GF = EPI == 1 || EPI == 2, GB = EPI == 3 || EPI == 4;   // GELU forward / act backward
  constexpr int SPASS = (GF ? 2 : 1) * SPT;                            // stores per thread and tile
  constexpr int PL = GB ? SPT : 0;                                     // pre-activation loads per thread and tile
  // per tile, in issue order: PL pre loads, the DMA of a later tile (XI), SPASS stores
  constexpr int WAITN = (NBUF - 1) * SPASS + (NBUF - 2) * (XI + PL);  // issued after a tile's DMA
  static_assert(WAITN <= 63, "vmcnt");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[WB + NBUF * XB + OB + (GF ? kGeluEntries * 2 : 0)];
  unsigned char* sW = smem;
  unsigned char* sX = smem + WB;                                       // [NBUF][NKS][BM rows x 128 B]
  unsigned char* sO = smem + WB + NBUF * XB;
  unsigned short* sgelu = reinterpret_cast<unsigned short*>(sO + OB);
  const int rowB = K * 2;
  const int tilesM = (M + BM - 1) / BM, tilesN = (N + BN - 1) / BN;
  const int wg = xcd_swizzle(blockIdx.x, gridDim.x);
  const int tn = wg % tilesN, g0 = wg / tilesN, G = gridDim.x / tilesN;   // token tiles g0, g0 + G, ...
  if (g0 >= G || g0 >= tilesM) return;                                 // (uniform)
  const int ntl = (tilesM - g0 + G - 1) / G;                           // this workgroup's tiles
  const int n0 = tn * BN;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  // zero the X ring and W (the chunks past K stay zero), then W by LDS-DMA
  for (int i = threadIdx.x; i < (WB + NBUF * XB) / 16; i += NT) reinterpret_cast<uint4*>(smem)[i] = make_uint4(0, 0, 0, 0);
  if (GF)
    for (int i = threadIdx.x; i < kGeluEntries / 8; i += NT)
      reinterpret_cast<uint4*>(sgelu)[i] = reinterpret_cast<const uint4*>(kGeluTable)[i];
  __syncthreads();
  // W: NKS images of BN rows, 8 rows (1 KB) per wave instruction, lane L -> row 8j + L/8,
  // physical chunk L%8 (the swizzle applied to the source chunk)
  for (int blk = w; blk < NKS * BN / 8; blk += 4) {
    const int ks = blk / (BN / 8), row = (blk % (BN / 8)) * 8 + (l >> 3);
    const int chunk = (l & 7) ^ ((row >> 1) & 7), kb = ks * kRowB + chunk * 16;
    if (kb < rowB) glds16(reinterpret_cast<const unsigned char*>(Wt) + (size_t)min(n0 + row, N - 1) * rowB + kb,
                          sW + ks * WIMG + (blk % (BN / 8)) * 1024);
  }
  auto issue_x = [&](int j) {                                          // tile j of this workgroup
    const int tm = g0 + j * G;
    unsigned char* base = sX + (j % NBUF) * XB;
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int blk = w * XI + i, ks = blk / (BM / 8), rb = blk % (BM / 8);
      const int row = rb * 8 + (l >> 3);
      const int chunk = (l & 7) ^ ((row >> 1) & 7), kb = ks * kRowB + chunk * 16;
      if (kb < rowB)
        glds16(reinterpret_cast<const unsigned char*>(X) + (size_t)min(tm * BM + row, M - 1) * rowB + kb,
               base + ks * XIMG + rb * 1024);
    }
  };
  auto so_off = [](int row, int chunk) { return row * (BN * 2) + ((chunk ^ (row & 15)) << 4); };
  // this lane's bias values (features 32w + 8g + 4hh .. +3), once: a per-tile load from L2
  // sat in the epilogue's critical path
  bf16x4_t bvr[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int n = n0 + 32 * w + 8 * g + 4 * hh;
    bvr[g] = (bias && n < N) ? *reinterpret_cast<const bf16x4_t*>(bias + n) : bf16x4_t{0, 0, 0, 0};
  }
  for (int j = 0; j < NBUF - 1 && j < ntl; ++j) issue_x(j);
  wait_vm<0>();                                                        // W and the first tiles
  for (int j = 0; j < ntl; ++j) {
    if (j >= NBUF - 1) {                                               // (tiles < NBUF - 1: the prologue's wait)
      if (j + NBUF - 2 < ntl) wait_vm<WAITN>();                        // tile j landed; later ops may fly
      else wait_vm<0>();
    }
    raw_barrier();                                                     // every wave's DMA landed; ring slot free
    const int m0 = (g0 + j * G) * BM;
    uint4 pv[GB ? SPT : 1];                                            // GELU backward: this tile's pre-activations
    if (GB) {
#pragma unroll
      for (int i = 0; i < SPT; ++i) {
        const int idx = threadIdx.x + i * NT, row = idx / NCK, chunk = idx % NCK;
        const int m = min(m0 + row, M - 1), n = min(n0 + chunk * 8, N - 8);   // always a load: counted waits
        pv[i] = *reinterpret_cast<const uint4*>(Y2 + (size_t)m * N + n);
      }
    }
    if (j + NBUF - 1 < ntl) issue_x(j + NBUF - 1);                     // the slot of tile j - 1
    // W fragments are re-read from LDS per tile: hoisted out of the tile loop they took the
    // registers of a second wave per SIMD
    asm volatile("" ::: "memory");
    const unsigned char* xs = sX + (j % NBUF) * XB;
    f32x16_t acc[TM];
#pragma unroll
    for (int t = 0; t < TM; ++t) zero16(acc[t]);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        if (ks * 64 + kk * 16 >= K) break;                           // K % 8 == 0: whole 16-steps only
        const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(sW + ks * WIMG + tile_off(32 * w + r, 2 * kk + hh));
#pragma unroll
        for (int t = 0; t < TM; ++t)
          acc[t] = mfma16(a, *reinterpret_cast<const bf16x8_t*>(xs + ks * XIMG + tile_off(32 * t + r, 2 * kk + hh)),
                          acc[t]);
      }
    }
#pragma unroll
    for (int pass = 0; pass < (GF ? 2 : 1); ++pass) {
      if (pass) raw_barrier();                                         // pass 0's rows are stored
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        const int row = 32 * t + r;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int f = 32 * w + 8 * g + 4 * hh;
          const bf16x4_t bv = bvr[g];
          bf16x4_t o;
#pragma unroll
          for (int e2 = 0; e2 < 4; ++e2) {
            const short pre = bf16_bits(acc[t][4 * g + e2] + bf16_bits_to_f32((unsigned short)bv[e2]));
            o[e2] = (GF && pass == 0) ? (short)gelu_bits((unsigned short)pre, sgelu) : pre;
          }
          *reinterpret_cast<bf16x4_t*>(sO + so_off(row, f >> 3) + (f & 7) * 2) = o;
        }
      }
      raw_barrier();
      if (GB) {
        // the pre loads were issued before tile j + NBUF - 1's DMA: only that DMA may fly on
        if (j + NBUF - 1 < ntl) wait_vm<XI>();
        else wait_vm<0>();
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
          const int idx = threadIdx.x + i * NT, row = idx / NCK, chunk = idx % NCK;
          const int m = m0 + row, n = n0 + chunk * 8;
          if (m < M && n < N)
            *reinterpret_cast<uint4*>(Y + (size_t)m * N + n) =
                act_bwd8<EPI == 4>(*reinterpret_cast<const uint4*>(sO + so_off(row, chunk)), pv[i]);
        }
        continue;
      }
      bf16* out = pass == 0 ? Y : Y2;
#pragma unroll
      for (int i = 0; i < SPT; ++i) {
        const int idx = threadIdx.x + i * NT, row = idx / NCK, chunk = idx % NCK;
        const int m = m0 + row, n = n0 + chunk * 8;
        if (m < M && n < N)
          *reinterpret_cast<uint4*>(out + (size_t)m * N + n) = *reinterpret_cast<const uint4*>(sO + so_off(row, chunk));
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

// VS_TGEMM_STREAM_ROWS: the least M for the streaming kernel (0 = never; default 32768)
static int tgemm_stream_min_rows() {
  const char* e = getenv("VS_TGEMM_STREAM_ROWS");
  const int x = e ? atoi(e) : 32768;
  return x <= 0 ? (1 << 30) : x;
}

extern "C" int vs_token_gemm(int mode, const void* x, const void* x_scales, const void* w, const void* w_scales,
                             const void* bias, void* y, void* y_pre, void* y_q, void* y_qscales, int M, int N, int K,
                             void* stream) {
  const bool f8 = (mode & VS_TGEMM_FP8) != 0, gelu = (mode & VS_TGEMM_GELU) != 0;
  const bool gbwd = (mode & VS_TGEMM_GELU_BWD) != 0, rbwd = (mode & VS_TGEMM_RELU_BWD) != 0;
  VS_CHECK(x && w && y, "null pointer");
  VS_CHECK(!(gbwd && rbwd), "one activation backward");
  VS_CHECK(!(gbwd || rbwd) || (!f8 && !gelu && !(mode & VS_TGEMM_QOUT) && !bias && y_pre && N % 8 == 0),
           "activation backward: bf16, no bias / GELU / quantised output, y_pre (read) given, N % 8 == 0");
  VS_CHECK(M > 0 && N > 0 && K > 0, "empty GEMM");
  VS_CHECK(N % 4 == 0, "N must be a multiple of 4");
  VS_CHECK(f8 ? (K % 128 == 0 && x_scales && w_scales) : (K % 8 == 0), "fp8: K % 128 == 0 and scales; bf16: K % 8 == 0");
  VS_CHECK(!gelu || y_pre, "gelu needs the pre-activation output");
  // 16-B LDS-DMA row loads and epilogue stores, 8-B bias loads, 4-B scale loads
  VS_CHECK(((uintptr_t)x & 15) == 0 && ((uintptr_t)w & 15) == 0 && ((uintptr_t)y & 15) == 0 &&
               (!y_pre || ((uintptr_t)y_pre & 15) == 0) && (!bias || ((uintptr_t)bias & 7) == 0) &&
               (!x_scales || ((uintptr_t)x_scales & 3) == 0) && (!w_scales || ((uintptr_t)w_scales & 3) == 0) &&
               (!y_q || ((uintptr_t)y_q & 3) == 0),
           "alignment: x / w / y / y_pre 16 B, bias 8 B, scales / y_q 4 B");
  const bool qout = (mode & VS_TGEMM_QOUT) != 0;
  VS_CHECK(!qout || (gelu && y_q && y_qscales && N % 32 == 0), "quantised output: with gelu, N % 32 == 0, both buffers");
  if (!f8 && !qout && N % 8 == 0 && K <= 192 && M >= tgemm_stream_min_rows()) {
    // short rows, many tokens: the streaming kernel (W slice resident, token tiles streamed)
    hipStream_t sst = (hipStream_t)stream;
    // 32-row token tiles through a ring of 4 X buffers (3 tiles of prefetch), 2 workgroups
    // per CU; K-steps of 3 (K > 128): a ring of 2 keeps 2 workgroups per CU
    const int nks = (K * 2 + kRowB - 1) / kRowB;
    const int tilesN = (N + 127) / 128, tilesM = (M + 31) / 32;
    const int per_cu = (gelu && nks == 3) ? 1 : 2;                 // workgroups per CU (LDS)
    const int G = std::max(1, std::min(tilesM, 256 * per_cu / tilesN));
    const dim3 sgrid((unsigned)(G * tilesN));
#define VS_TGS(E_, NK_, NB_)                                                                                     \
  hipLaunchKernelGGL((token_gemm_stream_kernel<E_, NK_, 1, NB_>), sgrid, dim3(256), 0, sst, (const bf16*)x,      \
                     (const bf16*)w, (const bf16*)bias, (bf16*)y, (bf16*)y_pre, M, N, K)
    if (gelu) {
      if (nks == 1) VS_TGS(1, 1, 4);
      else if (nks == 2) VS_TGS(1, 2, 4);
      else VS_TGS(1, 3, 2);
    } else if (gbwd) {
      if (nks == 1) VS_TGS(3, 1, 4);
      else if (nks == 2) VS_TGS(3, 2, 4);
      else VS_TGS(3, 3, 2);
    } else if (rbwd) {
      if (nks == 1) VS_TGS(4, 1, 4);
      else if (nks == 2) VS_TGS(4, 2, 4);
      else VS_TGS(4, 3, 2);
    } else {
      // (K-steps 4-6 with one workgroup per CU were measured slower than the tile kernel:
      // profiles/r5_tgemm_stream_ab.txt)
      if (nks == 1) VS_TGS(0, 1, 4);
      else if (nks == 2) VS_TGS(0, 2, 4);
      else VS_TGS(0, 3, 2);
    }
#undef VS_TGS
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
  // the 256 x 256 tile where the product is MFMA-bound and fills the chip
  // (the activation-backward epilogues take the 128 x 128 tile: its pre-activation loads ride
  // with the last K-step, and two workgroups per CU overlap one's epilogue with the other's
  // loop -- 56.5 vs 66.6 us at the stage-3 fc2 dX, 135.7 vs 144.0 at the encoder FFN's,
  // profiles/r6_act_bwd_epilogue_ab.txt)
  const bool big = N >= 512 && K >= 256 && (long long)((M + 255) / 256) * ((N + 255) / 256) >= 256 &&
                   !(gbwd || rbwd);
  const int bm = big ? 256 : 128, bn = big ? 256 : 128;
  const long long tiles = (long long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  VS_CHECK(tiles < (1ll << 31), "too many tiles");
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)tiles);
#define VS_TG(F8_, E_)                                                                                               \
  do {                                                                                                               \
    if (big)                                                                                                         \
      hipLaunchKernelGGL((token_gemm_kernel<F8_, E_, 2, 4, 4, 2>), grid, dim3(512), 0, st, (const unsigned char*)x,  \
                         (const unsigned char*)x_scales, (const unsigned char*)w, (const unsigned char*)w_scales,     \
                         (const bf16*)bias, (bf16*)y, (bf16*)y_pre, (unsigned char*)y_q, (unsigned char*)y_qscales, M, N, K);                                         \
    else                                                                                                             \
      hipLaunchKernelGGL((token_gemm_kernel<F8_, E_, 2, 2, 2, 2>), grid, dim3(256), 0, st, (const unsigned char*)x,  \
                         (const unsigned char*)x_scales, (const unsigned char*)w, (const unsigned char*)w_scales,     \
                         (const bf16*)bias, (bf16*)y, (bf16*)y_pre, (unsigned char*)y_q, (unsigned char*)y_qscales, M, N, K);                                         \
  } while (0)
  if (f8 && qout) VS_TG(true, 2);
  else if (f8 && gelu) VS_TG(true, 1);
  else if (f8) VS_TG(true, 0);
  else if (qout) VS_TG(false, 2);
  else if (gelu) VS_TG(false, 1);
  else if (gbwd) VS_TG(false, 3);
  else if (rbwd) VS_TG(false, 4);
  else VS_TG(false, 0);
#undef VS_TG
  VS_LAUNCH_CHECK();
  return VS_OK;
}
