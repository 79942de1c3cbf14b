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

#include <type_traits>

#include "lds_dma.h"

namespace vs {
namespace {


// A workgroup: BO output rows x BI input columns of dW (BO, BI in {128, 256}), 8 waves in a
// WO x WI grid (WO = 4 for BI = 128, else 2): a wave owns BO / WO rows (TO MFMA tiles of 32) x
// 64 columns (2 tiles).  The bias column sums: wave (qo, qi) adds the ones-row MFMA for its
// o-tile qi (if it has one), so the extra MFMA is spread over the waves of the first input
// block.  part [S][N][K], pbias [S][N].
// NS-stage ring of TK-token chunk buffers: NS - 1 chunks in flight while one is multiplied
// (every wave issues the same PW DMA instructions per chunk, so a counted vmcnt wait retires
// exactly the oldest chunk).
// DBG (timing experiments only): 1 no MFMA, 2 no DMA, 3 neither and no LDS reads, 4 no chunk loop
template <int BO, int BI, int NS, int TK, int DBG = 0>
__global__ void __launch_bounds__(512) token_wgrad_kernel(const bf16* __restrict__ gy, const bf16* __restrict__ x,
                                                          float* __restrict__ part, float* __restrict__ pbias, int T,
                                                          int N, int K, long long ldg, long long ldx, int S) {
  constexpr int NH = BO / 128, NXH = BI / 128;          // gY / X half-images of 128 columns
  constexpr int IMG = TK * 256;                         // bytes of one half-image
  constexpr int GYB = NH * IMG, STG = (NH + NXH) * IMG;
  constexpr int RB = TK / 4;                            // 1-KB DMA blocks (4 rows) per image
  constexpr int NBLK = STG / 1024;                      // 1-KB DMA blocks per stage
  constexpr int PW = NBLK / 8;                          // DMA instructions per wave per chunk
  static_assert(NBLK % 8 == 0, "uniform DMA count per wave");
  constexpr int WO = BI == 128 ? 4 : 2, WI = 8 / WO;
  static_assert(WI * 64 == BI, "64 input columns per wave");
  constexpr int TO = BO / WO / 32;                      // o-tiles per wave
  static_assert(TO <= WI, "one bias o-tile per wave");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NS * STG];
  const int tiles_o = (N + BO - 1) / BO, tiles_i = (K + BI - 1) / BI, tiles = tiles_o * tiles_i;
  const int wg = xcd_swizzle(blockIdx.x, S * tiles);
  const int s = wg / tiles, tile = wg - s * tiles;      // a split's tiles are neighbours (one XCD)
  const int ob = tile / tiles_i, ib = tile - ob * tiles_i;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int qo = w % WO, qi = w / WO;
  const int wo = qo * (BO / WO), wi = qi * 64;
  const long long nchunk = ((long long)T + TK - 1) / TK;
  const long long cb = nchunk * s / S, ce = nchunk * (s + 1) / S;
  const int bt = __builtin_amdgcn_readfirstlane(qi);    // this wave's bias o-tile (if < TO)
  const bool do_bias = pbias != nullptr && ib == 0 && bt < TO;

  // per-lane DMA constants, hoisted out of the chunk loop: for the j-th piece, the element
  // offset of this lane's 16 B inside a chunk (row * ld + col), its row, and whether it reads
  // gY (else X) / lies inside the matrix width
  int doff[PW], drow[PW];
  unsigned dgy = 0, dok = 0;
#pragma unroll
  for (int j = 0; j < PW; ++j) {
    const int blk = w + 8 * j;
    const int img = blk / RB, row = (blk % RB) * 4 + (l >> 4), ch = (l & 15) ^ img_swz(row);
    drow[j] = row;
    if (img < NH) {
      const int col = ob * BO + img * 128 + ch * 8;
      doff[j] = (int)(row * ldg) + col;
      dgy |= 1u << j;
      if (col < N) dok |= 1u << j;
    } else {
      const int col = ib * BI + (img - NH) * 128 + ch * 8;
      doff[j] = (int)(row * ldx) + col;
      if (col < K) dok |= 1u << j;
    }
  }
  auto issue = [&](long long c, int st) {
    unsigned char* base = smem + st * STG;
    const bf16* cg = gy + c * TK * ldg;                 // the chunk's first rows (wave-uniform)
    const bf16* cx = x + c * TK * ldx;
    const long long left = (long long)T - c * TK;       // rows of the chunk inside the matrix
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      const int blk = w + 8 * j;
      const int ch = (l & 15) ^ img_swz(drow[j]);
      const bool ok = ((dok >> j) & 1u) && drow[j] < left;
      const unsigned char* src = ok ? reinterpret_cast<const unsigned char*>(((dgy >> j) & 1u ? cg : cx) + doff[j])
                                    : g_dma_zero_row + ch * 16;
      if (DBG != 2 && DBG != 3) glds16(src, base + blk * 1024);
    }
  };

  f32x16_t acc[TO][2], accb;
#pragma unroll
  for (int a = 0; a < TO; ++a) {
    zero16(acc[a][0]);
    zero16(acc[a][1]);
  }
  zero16(accb);
  const short one = (short)0x3f80;                      // bf16 1.0
  const bf16x8_t ones = {one, one, one, one, one, one, one, one};
#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (cb + j < ce) issue(cb + j, j);
  // the chunk loop, instantiated with and without the bias MFMAs (a wave-uniform choice made
  // once: a branch around them inside the loop made the compiler shuffle the accumulators)
  auto run = [&](auto bias_tag) {
    constexpr bool BIAS = decltype(bias_tag)::value;
    int st = 0;
    for (long long c = cb; c < ce; ++c) {
      if (c + NS - 2 < ce)
        wait_vm<(NS - 2) * PW>();                       // chunk c landed (NS - 2 younger in flight)
      else
        wait_vm<0>();
      raw_barrier();                                    // every wave's did; chunk c - 1 is consumed
      if (c + NS - 1 < ce) issue(c + NS - 1, st == 0 ? NS - 1 : st - 1);   // into chunk c - 1's stage
      const unsigned char* sg = smem + st * STG;
      st = st == NS - 1 ? 0 : st + 1;
      const unsigned char* sx = sg + GYB;
      // operands of 16-token step k (asm reads: see lds_dma.h), one step ahead of the MFMAs
      bf16x8_t a[2][2], b[2][TO];
      auto load = [&](int k, int p) {
        if (DBG == 3) return;
#pragma unroll
        for (int ti = 0; ti < 2; ++ti) {
          const int ic = wi + 32 * ti;                                                         // X^T: rows i
          a[p][ti] = tr_frag_asm(sx + (ic >> 7) * IMG, 16 * k, ic & 127, l);
        }
#pragma unroll
        for (int to = 0; to < TO; ++to) {
          const int oc = wo + 32 * to;                                                         // gY: cols o
          b[p][to] = tr_frag_asm(sg + (oc >> 7) * IMG, 16 * k, oc & 127, l);
        }
      };
      constexpr int RD = 2 * (2 + TO);                   // ds_read_tr per step
      // DB: step k + 1's operands in flight during step k's MFMAs (the 256 x 256 tile has no
      // registers for a second set: its co-resident wave hides the reads instead)
      constexpr bool DB = TO <= 2;
      if (DB) load(0, 0);
#pragma unroll
      for (int k = 0; k < TK / 16; ++k) {
        const int p = DB ? (k & 1) : 0;
        if (!DB) {
          load(k, 0);
          lgkm_wait<0>(a[p][0]);
        } else if (k + 1 < TK / 16) {
          load(k + 1, p ^ 1);
          lgkm_wait<RD>(a[p][0]);                        // step k's reads are the older RD
        } else {
          lgkm_wait<0>(a[p][0]);
        }
        lgkm_wait<RD>(a[p][1]);
#pragma unroll
        for (int to = 0; to < TO; ++to) lgkm_wait<RD>(b[p][to]);
#pragma unroll
        for (int to = 0; to < TO; ++to) {
#pragma unroll
          for (int ti = 0; ti < 2; ++ti)
            if (DBG != 1 && DBG != 3) acc[to][ti] = mfma16(a[p][ti], b[p][to], acc[to][ti]);
          if (BIAS && to == bt) accb = mfma16(ones, b[p][to], accb);   // bt: scalar, a branch
        }
      }
    }
  };
  if (DBG == 4) {
  } else if (do_bias) {
    run(std::true_type{});
  } else {
    run(std::false_type{});
  }
  // partials in FRAGMENT order (whole 1-KB stores: the [o][i] row layout wrote 16 B every
  // 32 B across 32 rows per instruction, ~2 TB/s): the workgroup's block of BO x BI floats is
  // [wave][to][ti][g][lane][4 registers]; token_wgrad_reduce_kernel maps (o, i) back
  float* pw = part + ((size_t)s * tiles + tile) * (BO * BI) + (size_t)w * (TO * 2 * 1024) + l * 4;
#pragma unroll
  for (int to = 0; to < TO; ++to)
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(pw + ((to * 2 + ti) * 4 + g) * 256) =
            make_float4(acc[to][ti][4 * g], acc[to][ti][4 * g + 1], acc[to][ti][4 * g + 2], acc[to][ti][4 * g + 3]);
  if (do_bias && hh == 0) {
    const int o = ob * BO + wo + 32 * bt + r;
    if (o < N) pbias[(size_t)s * N + o] = accb[0];
  }
}

// dW[o][i] = sum_s (fragment-order partial of (o, i) in split s), db[o] = sum_s pbias[s][o],
// fixed order.  A thread owns (o, 4 consecutive i): one float4 per split (the 4 registers of
// a lane's group), consecutive threads take consecutive o (= consecutive lanes: 16-B reads of
// one 1-KB block).  A 256-thread block = 64 items x 4 split groups (g, g + 4, ...), the group
// sums added in LDS in group order.
template <typename T>
__global__ void __launch_bounds__(256) token_wgrad_reduce_kernel(const float* __restrict__ part,
                                                                 const float* __restrict__ pbias, T* __restrict__ dw,
                                                                 T* __restrict__ db, int N, int K, int BO, int BI,
                                                                 int S) {
  __shared__ float4 sp[4][64];
  const int it = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const long long q = (long long)blockIdx.x * 64 + it;
  const long long nq = (long long)N * (K / 4), nqb = db ? N / 4 : 0;
  const bool isw = q < nq, isb = !isw && q - nq < nqb;
  const int WO = BI == 128 ? 4 : 2, TO = BO / WO / 32;
  const int tiles_i = (K + BI - 1) / BI, tiles = ((N + BO - 1) / BO) * tiles_i;
  const long long tstride = (long long)tiles * BO * BI;          // floats per split
  const float* src = part;
  long long stride = tstride;
  int o = 0, i = 0;
  if (isw) {
    o = (int)(q % N);
    i = (int)(q / N) * 4;
    const int ob = o / BO, ib = i / BI, oo = o - ob * BO, ii = i - ib * BI;
    const int qo = oo / (BO / WO), qi = ii >> 6, to = (oo % (BO / WO)) >> 5, r = oo & 31;
    const int ti = (ii & 63) >> 5, row = ii & 31;                // row % 4 == 0: registers 4g..4g+3
    const int g = row >> 3, hh = (row >> 2) & 1;
    const int w = qi * WO + qo;
    src = part + (long long)(ob * tiles_i + ib) * BO * BI + (long long)w * (TO * 2 * 1024) +
          ((to * 2 + ti) * 4 + g) * 256 + (hh * 32 + r) * 4;
  } else if (isb) {
    src = pbias + 4 * (q - nq);
    stride = N;
  }
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (isw || isb) {
    int s = grp;
    for (; s + 12 < S; s += 16) {
      const float4 v0 = *reinterpret_cast<const float4*>(src + s * stride);
      const float4 v1 = *reinterpret_cast<const float4*>(src + (s + 4) * stride);
      const float4 v2 = *reinterpret_cast<const float4*>(src + (s + 8) * stride);
      const float4 v3 = *reinterpret_cast<const float4*>(src + (s + 12) * stride);
      a.x += v0.x; a.y += v0.y; a.z += v0.z; a.w += v0.w;
      a.x += v1.x; a.y += v1.y; a.z += v1.z; a.w += v1.w;
      a.x += v2.x; a.y += v2.y; a.z += v2.z; a.w += v2.w;
      a.x += v3.x; a.y += v3.y; a.z += v3.z; a.w += v3.w;
    }
    for (; s < S; s += 4) {
      const float4 v = *reinterpret_cast<const float4*>(src + s * stride);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  sp[grp][it] = a;
  __syncthreads();
  if (grp == 0 && (isw || isb)) {
    const float4 b = sp[1][it], c = sp[2][it], d = sp[3][it];
    const float r0 = ((a.x + b.x) + c.x) + d.x, r1 = ((a.y + b.y) + c.y) + d.y;
    const float r2 = ((a.z + b.z) + c.z) + d.z, r3 = ((a.w + b.w) + c.w) + d.w;
    T* out = isw ? dw + (size_t)o * K + i : db + 4 * (q - nq);
    out[0] = from_f32<T>(r0);
    out[1] = from_f32<T>(r1);
    out[2] = from_f32<T>(r2);
    out[3] = from_f32<T>(r3);
  }
}

int wgrad_bo(int N) { return N > 128 ? 256 : 128; }

// VS_WGRAD_CFG: 0 (default) -> 64-token chunks; 1 -> 32-token chunks, twice the ring depth
// (same LDS): 0.737 vs 0.786 ms over the C2 shapes (profiles/r5_token_wgrad_ab.txt)
int wgrad_cfg() {
  static const int c = [] {
    const char* e = getenv("VS_WGRAD_CFG");
    return e ? atoi(e) : 0;
  }();
  return c;
}

// 256 input columns per workgroup (half the L2 -> LDS bytes per flop of 256 x 128) where the
// input is wide enough; VS_WGRAD_BI=128 forces the narrow tile
int wgrad_bi(int N, int K) {
  static const int force = [] {
    const char* e = getenv("VS_WGRAD_BI");
    return e ? atoi(e) : 0;
  }();
  if (force) return force;
  // measured: no gain from the 256-wide tile at the C2 shapes (the LDS-DMA issue rate, not
  // the L2 -> LDS bytes per flop, bounds the chunk loop: profiles/r5_token_wgrad_pmc.txt)
  (void)N;
  (void)K;
  return 128;
}

int wgrad_tok() { return wgrad_cfg() == 0 ? 64 : 32; }

int wgrad_splits(long long T, int N, int K) {
  const int BO = wgrad_bo(N), BI = wgrad_bi(N, K);
  const long long tiles = (long long)((N + BO - 1) / BO) * ((K + BI - 1) / BI);
  const long long nchunk = (T + wgrad_tok() - 1) / wgrad_tok();
  static const int target = [] {
    const char* e = getenv("VS_WGRAD_WGS");
    return e ? atoi(e) : 256;
  }();
  long long S = target / tiles;                        // ~one workgroup per CU (>= 128 KB of LDS)
  // at least 8 chunks a split: the per-split f32 partial block costs about as much traffic
  // as a few chunks of the operands
  if (S > nchunk / 8) S = nchunk / 8;
  if (S < 1) S = 1;
  return (int)S;
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" long long vs_token_wgrad_workspace_bytes(long long tokens, int N, int K) {
  if (tokens <= 0 || N <= 0 || K <= 0) return 0;
  const long long S = wgrad_splits(tokens, N, K);
  const int BO = wgrad_bo(N), BI = wgrad_bi(N, K);
  const long long padded = (long long)((N + BO - 1) / BO) * BO * (((K + BI - 1) / BI) * BI);
  return S * (padded + N) * 4;
}

extern "C" int vs_token_wgrad(int dtype, const void* grad_y, long long ld_grad_y, const void* x, long long ld_x,
                              void* dw, void* db, void* workspace, long long tokens, int N, int K, void* stream) {
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype (of dw / db) must be VS_F32 or VS_BF16");
  VS_CHECK(grad_y && x && dw && workspace, "null pointer");
  VS_CHECK(tokens > 0 && tokens < (1ll << 31) && N > 0 && K > 0 && N % 8 == 0 && K % 8 == 0,
           "0 < tokens < 2^31, N % 8 == 0, K % 8 == 0");
  VS_CHECK(ld_grad_y >= N && ld_x >= K && ld_grad_y % 8 == 0 && ld_x % 8 == 0, "row strides: >= width, % 8 == 0");
  VS_CHECK(64 * (ld_grad_y > ld_x ? ld_grad_y : ld_x) < (1ll << 31), "row strides too large");
  VS_CHECK(((uintptr_t)grad_y & 15) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)workspace & 15) == 0,
           "grad_y / x / workspace must be 16-B aligned");
  const int S = wgrad_splits(tokens, N, K);
  const int BO = wgrad_bo(N), BI = wgrad_bi(N, K);
  const long long tiles = (long long)((N + BO - 1) / BO) * ((K + BI - 1) / BI);
  VS_CHECK(S * tiles < (1ll << 31), "too many workgroups");
  float* part = (float*)workspace;
  float* pb = db ? part + (size_t)S * tiles * BO * BI : nullptr;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g((unsigned)(S * tiles));
#define VS_TW(BO_, BI_, NS_, TK_)                                                                                  \
  hipLaunchKernelGGL((token_wgrad_kernel<BO_, BI_, NS_, TK_>), g, dim3(512), 0, st, (const bf16*)grad_y,           \
                     (const bf16*)x, part, pb, (int)tokens, N, K, ld_grad_y, ld_x, S)
  const bool t64 = wgrad_cfg() == 0;
  if (BI == 256) {
    if (BO == 256) {
      if (t64) VS_TW(256, 256, 2, 64); else VS_TW(256, 256, 4, 32);
    } else {
      if (t64) VS_TW(128, 256, 3, 64); else VS_TW(128, 256, 6, 32);
    }
  } else {
    if (BO == 256) {
      if (t64) {
        static const int dbg = [] {
          const char* e = getenv("VS_WGRAD_DEBUG");
          return e ? atoi(e) : 0;
        }();
        if (dbg == 1)
          hipLaunchKernelGGL((token_wgrad_kernel<256, 128, 3, 64, 1>), g, dim3(512), 0, st, (const bf16*)grad_y,
                             (const bf16*)x, part, pb, (int)tokens, N, K, ld_grad_y, ld_x, S);
        else if (dbg == 2)
          hipLaunchKernelGGL((token_wgrad_kernel<256, 128, 3, 64, 2>), g, dim3(512), 0, st, (const bf16*)grad_y,
                             (const bf16*)x, part, pb, (int)tokens, N, K, ld_grad_y, ld_x, S);
        else if (dbg == 3)
          hipLaunchKernelGGL((token_wgrad_kernel<256, 128, 3, 64, 3>), g, dim3(512), 0, st, (const bf16*)grad_y,
                             (const bf16*)x, part, pb, (int)tokens, N, K, ld_grad_y, ld_x, S);
        else if (dbg == 4)
          hipLaunchKernelGGL((token_wgrad_kernel<256, 128, 3, 64, 4>), g, dim3(512), 0, st, (const bf16*)grad_y,
                             (const bf16*)x, part, pb, (int)tokens, N, K, ld_grad_y, ld_x, S);
        else
          VS_TW(256, 128, 3, 64);
      } else {
        VS_TW(256, 128, 6, 32);
      }
    } else {
      if (t64) VS_TW(128, 128, 4, 64); else VS_TW(128, 128, 8, 32);
    }
  }
#undef VS_TW
  VS_LAUNCH_CHECK();
  const long long items = (long long)N * (K / 4) + (db ? N / 4 : 0);
  const dim3 gr((unsigned)((items + 63) / 64));
  if (dtype == VS_BF16)
    hipLaunchKernelGGL(token_wgrad_reduce_kernel<bf16>, gr, dim3(256), 0, st, part, pb, (bf16*)dw, (bf16*)db, N, K,
                       BO, BI, S);
  else
    hipLaunchKernelGGL(token_wgrad_reduce_kernel<float>, gr, dim3(256), 0, st, part, pb, (float*)dw, (float*)db, N, K,
                       BO, BI, S);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
