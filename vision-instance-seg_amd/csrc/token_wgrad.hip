// Weight (and bias) gradient of token-major Linears: dW[o, i] = sum_t gY[t, o] X[t, i],
// db[o] = sum_t gY[t, o], for the token-heavy Linears of the Swin blocks and the pixel
// decoder (qkv, proj, fc1, fc2; the encoder's value / output / offset
// projections and FFN) -- one Linear per call, or a GROUP of independent Linears in one launch.
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
// input block.
//
// Splits: a Linear's output has few 256 x 128 tiles (18 at the C2 stage-3 fc1), so the
// tokens are split to fill the chip, and every split's f32 tile goes to memory and back
// through a reduction (~14 of a 33 us launch at that shape: one f32 block per CU).  A GROUP
// launch plans all its Linears together: with the tiles of many Linears filling the CUs,
// most of them run unsplit and write dW / db straight from the accumulators; a split is
// only used to balance the chunks per workgroup (the plan sizes every workgroup to about the
// same number of chunks).  Split partials are summed in a fixed order by a second kernel
// (deterministic, no atomics).
#include <stdlib.h>

#include <type_traits>

#include "lds_dma.h"

namespace vs {
namespace {

constexpr int kTK = 64;                      // tokens per chunk
constexpr int kMaxProbs = 20;                // Linears per group launch (kernel-argument space)

// one Linear of a launch, planned on the host
struct WgProb {
  const bf16* gy;
  const bf16* x;
  void* dw;
  void* db;
  long long ldg, ldx;
  long long part0;                           // first float of its split partial blocks (S > 1)
  long long pb0;                             // first float of its bias partials (S > 1)
  int T, N, K;
  int S;                                     // token splits
  int tiles_i, tiles;                        // tiles per split
  int wg0;                                   // first workgroup
  int item0;                                 // first reduction item (S > 1)
};

struct WgGroup {
  WgProb p[kMaxProbs];
  int n;
  int f32;                                   // dW / db dtype: 1 f32, 0 bf16
};

__device__ __forceinline__ void store4(void* base, size_t idx, bool f32, float a, float b, float c, float d) {
  if (f32) {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(base) + idx) = make_float4(a, b, c, d);
  } else {
    bf16x4_t v = {bf16_bits(a), bf16_bits(b), bf16_bits(c), bf16_bits(d)};
    *reinterpret_cast<bf16x4_t*>(reinterpret_cast<bf16*>(base) + idx) = v;
  }
}

// A workgroup: BO output rows x 128 input columns of one Linear's dW, 8 waves in a 4 x 2 grid:
// a wave owns BO / 4 rows (TO MFMA tiles of 32) x 64 columns (2 tiles).  The bias column
// sums: wave (qo, qi) adds the ones-row MFMA for its o-tile qi (if it has one).
// NS-stage ring of 64-token chunk buffers: NS - 1 chunks in flight while one is multiplied
// (every wave issues the same PW DMA instructions per chunk, so a counted vmcnt wait retires
// exactly the oldest chunk).
// DBG: the parts switched off in the round-5 timing split (tools/r5/wg4.sh; 1 no MFMA, 2 no DMA,
// 3 neither and no LDS reads, 4 no chunk loop); only DBG = 0 is instantiated
template <int BO, int BI, int WO, int WI, int NS, int DBG = 0>
__global__ void __launch_bounds__(64 * WO * WI) token_wgrad_kernel(const WgGroup grp, float* __restrict__ part,
                                                                   float* __restrict__ pbias, int spread) {
  constexpr int TK = kTK, NW = WO * WI;
  constexpr int NH = BO / 128, NXH = BI / 128;          // gY / X half-images of 128 columns
  constexpr int IMG = TK * 256;                         // bytes of one half-image
  constexpr int GYB = NH * IMG, STG = (NH + NXH) * IMG;
  constexpr int RB = TK / 4;                            // 1-KB DMA blocks (4 rows) per image
  constexpr int NBLK = STG / 1024;                      // 1-KB DMA blocks per stage
  constexpr int PW = NBLK / NW;                         // DMA instructions per wave per chunk
  static_assert(NBLK % NW == 0, "uniform DMA count per wave");
  constexpr int TO = BO / WO / 32, TI = BI / WI / 32;   // o- / i-tiles per wave
  constexpr int NB = TO / WI > 0 ? TO / WI : 1;         // bias o-tiles per wave (waves of one qo share)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NS * STG];
  const int wg = xcd_swizzle(blockIdx.x, gridDim.x);
  int pi = 0;                                           // this workgroup's Linear (scalar scan)
  for (int k = 1; k < grp.n; ++k)
    if (wg >= grp.p[k].wg0) pi = k;
  const WgProb& P = grp.p[pi];
  const bf16* __restrict__ gy = P.gy;
  const bf16* __restrict__ x = P.x;
  const int T = P.T, N = P.N, K = P.K, S = P.S, tiles_i = P.tiles_i, tiles = P.tiles;
  const long long ldg = P.ldg, ldx = P.ldx;
  const int local = wg - P.wg0;
  const int s = local / tiles, tile = local - s * tiles;   // a split's tiles are neighbours (one XCD)
  const int ob = tile / tiles_i, ib = tile - ob * tiles_i;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, hh = l >> 5;
  const int qo = w % WO, qi = w / WO;
  const int wo = qo * (BO / WO), wi = qi * (BI / WI);
  const long long nchunk = ((long long)T + TK - 1) / TK;
  const long long cb = nchunk * s / S, ce = nchunk * (s + 1) / S;
  const int bt = __builtin_amdgcn_readfirstlane(qi * NB);   // this wave's first bias o-tile (if < TO)
  const bool do_bias = P.db != nullptr && ib == 0 && bt < TO;

  // per-lane DMA constants, hoisted out of the chunk loop: for the j-th piece, the element
  // offset of this lane's 16 B inside a chunk (row * ld + col), its row, and whether it reads
  // gY (else X) / lies inside the matrix width
  int doff[PW], drow[PW];
  unsigned dgy = 0, dok = 0;
#pragma unroll
  for (int j = 0; j < PW; ++j) {
    const int blk = w + NW * j;
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
  // pieces [J0, J1) of chunk c into stage st
  auto issue_part = [&](long long c, int st, auto j0_tag, auto j1_tag) {
    constexpr int J0 = decltype(j0_tag)::value, J1 = decltype(j1_tag)::value;
    unsigned char* base = smem + st * STG;
    const bf16* cg = gy + c * TK * ldg;                 // the chunk's first rows (wave-uniform)
    const bf16* cx = x + c * TK * ldx;
    const long long left = (long long)T - c * TK;       // rows of the chunk inside the matrix
#pragma unroll
    for (int j = J0; j < J1; ++j) {
      const int blk = w + NW * j;
      const int ch = (l & 15) ^ img_swz(drow[j]);
      const bool ok = ((dok >> j) & 1u) && drow[j] < left;
      const unsigned char* src = ok ? reinterpret_cast<const unsigned char*>(((dgy >> j) & 1u ? cg : cx) + doff[j])
                                    : g_dma_zero_row + ch * 16;
      if (DBG != 2 && DBG != 3) glds16(src, base + blk * 1024);
    }
  };
  auto issue = [&](long long c, int st) {
    issue_part(c, st, std::integral_constant<int, 0>{}, std::integral_constant<int, PW>{});
  };

  f32x16_t acc[TO][TI], accb[NB];
#pragma unroll
  for (int a = 0; a < TO; ++a)
#pragma unroll
    for (int b = 0; b < TI; ++b) zero16(acc[a][b]);
#pragma unroll
  for (int a = 0; a < NB; ++a) zero16(accb[a]);
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
      // chunk c + NS - 1 goes into chunk c - 1's stage, its DMA pieces issued between the
      // MFMAs of chunk c's four steps (an LDS-DMA piece costs ~60-185 issue cycles: issued all
      // at once after the barrier, by every wave at the same time, they idled the MFMA pipe)
      const bool pre = spread && c + NS - 1 < ce;
      const int pst = st == 0 ? NS - 1 : st - 1;
      if (!spread && c + NS - 1 < ce) issue(c + NS - 1, pst);
      const unsigned char* sg = smem + st * STG;
      st = st == NS - 1 ? 0 : st + 1;
      const unsigned char* sx = sg + GYB;
      // operands of 16-token step k (asm reads: see lds_dma.h), one step ahead of the MFMAs
      bf16x8_t a[TO + TI <= 4 ? 2 : 1][TI], b[TO + TI <= 4 ? 2 : 1][TO];
      auto load = [&](int k, int p) {
        if (DBG == 3) return;
#pragma unroll
        for (int ti = 0; ti < TI; ++ti) {
          const int ic = wi + 32 * ti;                                                         // X^T: rows i
          a[p][ti] = tr_frag_asm(sx + (ic >> 7) * IMG, 16 * k, ic & 127, l);
        }
#pragma unroll
        for (int to = 0; to < TO; ++to) {
          const int oc = wo + 32 * to;                                                         // gY: cols o
          b[p][to] = tr_frag_asm(sg + (oc >> 7) * IMG, 16 * k, oc & 127, l);
        }
      };
      // ds_read_tr per step (the lgkmcnt field holds 15: a wait for "<= 15 outstanding" of 16
      // newer reads also retires one of them -- correct, marginally early)
      constexpr int RD = 2 * (TI + TO) > 15 ? 15 : 2 * (TI + TO);
      // DB: step k + 1's operands read during step k's MFMAs (the 256 x 256 tile's 256
      // accumulators leave no registers for a second set: one wave per SIMD, the next step's
      // reads are issued right after the MFMAs that free them)
      constexpr bool DB = TO + TI <= 4;
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
#pragma unroll
        for (int ti = 1; ti < TI; ++ti) lgkm_wait<RD>(a[p][ti]);
#pragma unroll
        for (int to = 0; to < TO; ++to) lgkm_wait<RD>(b[p][to]);
#pragma unroll
        for (int to = 0; to < TO; ++to) {
#pragma unroll
          for (int ti = 0; ti < TI; ++ti)
            if (DBG != 1 && DBG != 3) acc[to][ti] = mfma16(a[p][ti], b[p][to], acc[to][ti]);
          // bias: this wave's NB o-tiles from bt (a scalar: a uniform branch, compile-time slot)
          if (BIAS && to >= bt && to < bt + NB) accb[to % NB] = mfma16(ones, b[p][to], accb[to % NB]);
        }
        // this step's share of the next chunk's DMA pieces, behind the MFMAs just issued
        if (pre) {
          constexpr int NSTEP = TK / 16;
          if (k == 0)
            issue_part(c + NS - 1, pst, std::integral_constant<int, 0>{},
                       std::integral_constant<int, PW * 1 / NSTEP>{});
          else if (k == 1)
            issue_part(c + NS - 1, pst, std::integral_constant<int, PW * 1 / NSTEP>{},
                       std::integral_constant<int, PW * 2 / NSTEP>{});
          else if (k == 2)
            issue_part(c + NS - 1, pst, std::integral_constant<int, PW * 2 / NSTEP>{},
                       std::integral_constant<int, PW * 3 / NSTEP>{});
          else if (k == 3)
            issue_part(c + NS - 1, pst, std::integral_constant<int, PW * 3 / NSTEP>{},
                       std::integral_constant<int, PW>{});
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
  if (S > 1) {
    // split partials in FRAGMENT order (whole 1-KB stores): the workgroup's block of BO x BI
    // floats is [wave][to][ti][g][lane][4 registers]; token_wgrad_reduce_kernel maps (o, i) back
    float* pw = part + P.part0 + ((size_t)s * tiles + tile) * (BO * BI) + (size_t)w * (TO * TI * 1024) + l * 4;
#pragma unroll
    for (int to = 0; to < TO; ++to)
#pragma unroll
      for (int ti = 0; ti < TI; ++ti)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<float4*>(pw + ((to * TI + ti) * 4 + g) * 256) =
              make_float4(acc[to][ti][4 * g], acc[to][ti][4 * g + 1], acc[to][ti][4 * g + 2], acc[to][ti][4 * g + 3]);
    if (do_bias && hh == 0) {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int o = ob * BO + wo + 32 * (bt + j) + r;
        if (bt + j < TO && o < N) pbias[P.pb0 + (size_t)s * N + o] = accb[j][0];
      }
    }
    return;
  }
  // unsplit: dW / db straight from the accumulators (lane column = o, registers = 4 groups of
  // 4 consecutive i), rounded once to the parameter dtype
  const bool f32 = grp.f32 != 0;
#pragma unroll
  for (int to = 0; to < TO; ++to) {
    const int o = ob * BO + wo + 32 * to + r;
    if (o >= N) continue;
#pragma unroll
    for (int ti = 0; ti < TI; ++ti) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i = ib * BI + wi + 32 * ti + 8 * g + 4 * hh;
        if (i < K)
          store4(P.dw, (size_t)o * K + i, f32, acc[to][ti][4 * g], acc[to][ti][4 * g + 1], acc[to][ti][4 * g + 2],
                 acc[to][ti][4 * g + 3]);
      }
    }
  }
  if (do_bias && hh == 0) {
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int o = ob * BO + wo + 32 * (bt + j) + r;
      if (bt + j < TO && o < N) {
        if (f32)
          reinterpret_cast<float*>(P.db)[o] = accb[j][0];
        else
          reinterpret_cast<bf16*>(P.db)[o] = __float2bfloat16(accb[j][0]);
      }
    }
  }
}

// dW[o][i] = sum_s (fragment-order partial of (o, i) in split s), db[o] = sum_s pbias[s][o],
// fixed order, for the split Linears of a group.  A thread owns (o, 4 consecutive i): one
// float4 per split (the 4 registers of a lane's group), consecutive threads take consecutive
// o (= consecutive lanes: 16-B reads of one 1-KB block).  A block = 64 items x NG split
// groups (g, g + NG, ...), the group sums added in LDS in group order; a block's 64 items
// belong to one Linear (item0 is a multiple of 64).  NG = 16 when the items give few blocks
// (a 96 x 288 Linear: 108 blocks of 4 groups left most CUs idle and each thread ~40
// dependent-latency loads deep).
template <int BO, int BI, int WO, int WI, int NG>
__global__ void __launch_bounds__(64 * NG) token_wgrad_reduce_kernel(const WgGroup grp, const float* __restrict__ part,
                                                                     const float* __restrict__ pbias) {
  constexpr int TO = BO / WO / 32, TI = BI / WI / 32;
  __shared__ float4 sp[NG][64];
  const int it = threadIdx.x & 63, gq = threadIdx.x >> 6;
  const int item_blk = blockIdx.x * 64;
  int pi = -1;
  for (int k = 0; k < grp.n; ++k)
    if (grp.p[k].S > 1 && item_blk >= grp.p[k].item0) pi = k;
  if (pi < 0) return;
  const WgProb& P = grp.p[pi];
  const int N = P.N, K = P.K, S = P.S, tiles_i = P.tiles_i, tiles = P.tiles;
  const long long q = (long long)item_blk - P.item0 + it;
  const long long nq = (long long)N * (K / 4), nqb = P.db ? N / 4 : 0;
  const bool isw = q < nq, isb = !isw && q - nq < nqb;
  const long long tstride = (long long)tiles * BO * BI;          // floats per split
  const float* src = part + P.part0;
  long long stride = tstride;
  int o = 0, i = 0;
  if (isw) {
    o = (int)(q % N);
    i = (int)(q / N) * 4;
    const int ob = o / BO, ib = i / BI, oo = o - ob * BO, ii = i - ib * BI;
    const int qo = oo / (BO / WO), qi = ii / (BI / WI), to = (oo % (BO / WO)) >> 5, r = oo & 31;
    const int ti = (ii % (BI / WI)) >> 5, row = ii & 31;        // row % 4 == 0: registers 4g..4g+3
    const int g = row >> 3, hh = (row >> 2) & 1;
    const int w = qi * WO + qo;
    src += (long long)(ob * tiles_i + ib) * BO * BI + (long long)w * (TO * TI * 1024) + ((to * TI + ti) * 4 + g) * 256 +
           (hh * 32 + r) * 4;
  } else if (isb) {
    src = pbias + P.pb0 + 4 * (q - nq);
    stride = N;
  }
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (isw || isb) {
    int s = gq;
    for (; s + 3 * NG < S; s += 4 * NG) {
      const float4 v0 = *reinterpret_cast<const float4*>(src + s * stride);
      const float4 v1 = *reinterpret_cast<const float4*>(src + (s + NG) * stride);
      const float4 v2 = *reinterpret_cast<const float4*>(src + (s + 2 * NG) * stride);
      const float4 v3 = *reinterpret_cast<const float4*>(src + (s + 3 * NG) * stride);
      a.x += v0.x; a.y += v0.y; a.z += v0.z; a.w += v0.w;
      a.x += v1.x; a.y += v1.y; a.z += v1.z; a.w += v1.w;
      a.x += v2.x; a.y += v2.y; a.z += v2.z; a.w += v2.w;
      a.x += v3.x; a.y += v3.y; a.z += v3.z; a.w += v3.w;
    }
    for (; s < S; s += NG) {
      const float4 v = *reinterpret_cast<const float4*>(src + s * stride);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  sp[gq][it] = a;
  __syncthreads();
  if (gq == 0 && (isw || isb)) {
    float r0 = a.x, r1 = a.y, r2 = a.z, r3 = a.w;
#pragma unroll
    for (int k = 1; k < NG; ++k) {
      const float4 b = sp[k][it];
      r0 += b.x; r1 += b.y; r2 += b.z; r3 += b.w;
    }
    if (isw)
      store4(P.dw, (size_t)o * K + i, grp.f32 != 0, r0, r1, r2, r3);
    else
      store4(P.db, (size_t)(4 * (q - nq)), grp.f32 != 0, r0, r1, r2, r3);
  }
}


// Plan one launch: the Linears share BO.  Every workgroup gets about the same number of
// chunks C: C = max(8, total chunk-tiles / 256) (one workgroup per CU with 144 KB of LDS);
// a Linear is split into ceil(nchunk / C) token ranges.  Returns the workgroup count and the
// partial floats / reduction items it needs.
struct Plan {
  WgGroup g;
  long long wgs, tile_floats, part_floats, items;   // part_floats = tile partials + bias partials
};

void plan_group(const vs_wgrad_problem* probs, const int* idx, int n, int BO, int BI, int f32, Plan& pl) {
  constexpr int target = 256, minc = 8;        // one workgroup per CU; >= 8 chunks a workgroup
  long long total = 0;
  for (int k = 0; k < n; ++k) {
    const vs_wgrad_problem& q = probs[idx[k]];
    const long long tiles = (long long)((q.N + BO - 1) / BO) * ((q.K + BI - 1) / BI);
    total += tiles * ((q.tokens + kTK - 1) / kTK);
  }
  // the smallest C whose workgroups fit one round (ceil per Linear can push past the target:
  // a second, mostly idle round of workgroups)
  auto wgs_for = [&](long long c) {
    long long w = 0;
    for (int k = 0; k < n; ++k) {
      const vs_wgrad_problem& q = probs[idx[k]];
      const long long tiles = (long long)((q.N + BO - 1) / BO) * ((q.K + BI - 1) / BI);
      w += tiles * (((q.tokens + kTK - 1) / kTK + c - 1) / c);
    }
    return w;
  };
  long long C = (total + target - 1) / target;
  if (C < minc) C = minc;
  long long cmax = 1;
  for (int k = 0; k < n; ++k) {
    const long long nc = (probs[idx[k]].tokens + kTK - 1) / kTK;
    if (nc > cmax) cmax = nc;
  }
  while (wgs_for(C) > target && C < cmax) ++C;
  pl.g.n = n;
  pl.g.f32 = f32;
  pl.wgs = pl.tile_floats = pl.part_floats = pl.items = 0;
  long long pbf = 0;
  for (int k = 0; k < n; ++k) {
    const vs_wgrad_problem& q = probs[idx[k]];
    WgProb& P = pl.g.p[k];
    P.gy = (const bf16*)q.grad_y;
    P.x = (const bf16*)q.x;
    P.dw = q.dw;
    P.db = q.db;
    P.ldg = q.ld_grad_y;
    P.ldx = q.ld_x;
    P.T = (int)q.tokens;
    P.N = q.N;
    P.K = q.K;
    P.tiles_i = (q.K + BI - 1) / BI;
    P.tiles = ((q.N + BO - 1) / BO) * P.tiles_i;
    const long long nchunk = (q.tokens + kTK - 1) / kTK;
    long long S = (nchunk + C - 1) / C;
    if (S < 1) S = 1;
    P.S = (int)S;
    P.wg0 = (int)pl.wgs;
    pl.wgs += S * P.tiles;
    P.part0 = P.pb0 = 0;
    P.item0 = 0;
    if (S > 1) {
      P.part0 = pl.part_floats;
      pl.part_floats += S * P.tiles * BO * BI;
      P.item0 = (int)pl.items;
      const long long items = (long long)q.N * (q.K / 4) + (q.db ? q.N / 4 : 0);
      pl.items += (items + 63) / 64 * 64;
      if (q.db) pbf += S * q.N;
    }
  }
  // bias partials after all tile partials (pb0 relative to the bias region)
  pl.tile_floats = pl.part_floats;
  long long off = 0;
  for (int k = 0; k < n; ++k) {
    WgProb& P = pl.g.p[k];
    if (P.S > 1 && P.db) {
      P.pb0 = off;
      off += (long long)P.S * P.N;
    }
  }
  pl.part_floats += pbf;
}

// tile configurations: 0 = 256 x 128 (8 waves), 1 = 128 x 128 (8 waves, N <= 128).  (A
// 256 x 256 tile of 4 waves -- 128 x 128 per wave, half the operand reads per MFMA -- needs
// 256 accumulators per lane and spilled: not built.)
int wgrad_cfg_of(int N, int K) {
  (void)K;
  return N <= 128 ? 1 : 0;
}

// the launches of a call: problems grouped by tile configuration, in chunks of kMaxProbs
template <typename F>
int for_each_launch(const vs_wgrad_problem* probs, int n, int f32, F&& fn) {
  for (int cfg : {0, 1}) {
    const int BO = cfg == 1 ? 128 : 256, BI = 128;
    int idx[kMaxProbs];
    int m = 0;
    for (int k = 0; k < n; ++k) {
      if (wgrad_cfg_of(probs[k].N, probs[k].K) != cfg) continue;
      idx[m++] = k;
      if (m == kMaxProbs) {
        Plan pl;
        plan_group(probs, idx, m, BO, BI, f32, pl);
        const int rc = fn(cfg, pl);
        if (rc != VS_OK) return rc;
        m = 0;
      }
    }
    if (m) {
      Plan pl;
      plan_group(probs, idx, m, BO, BI, f32, pl);
      const int rc = fn(cfg, pl);
      if (rc != VS_OK) return rc;
    }
  }
  return VS_OK;
}

}  // namespace
}  // namespace vs

using namespace vs;

static int check_problems(const vs_wgrad_problem* probs, int n) {
  VS_CHECK(probs && n >= 0, "null problem list");
  for (int k = 0; k < n; ++k) {
    const vs_wgrad_problem& q = probs[k];
    VS_CHECK(q.grad_y && q.x && q.dw, "null pointer");
    VS_CHECK(q.tokens > 0 && q.tokens < (1ll << 31) && q.N > 0 && q.K > 0 && q.N % 8 == 0 && q.K % 8 == 0,
             "0 < tokens < 2^31, N % 8 == 0, K % 8 == 0");
    VS_CHECK(q.ld_grad_y >= q.N && q.ld_x >= q.K && q.ld_grad_y % 8 == 0 && q.ld_x % 8 == 0,
             "row strides: >= width, % 8 == 0");
    VS_CHECK(64 * (q.ld_grad_y > q.ld_x ? q.ld_grad_y : q.ld_x) < (1ll << 31), "row strides too large");
    VS_CHECK(((uintptr_t)q.grad_y & 15) == 0 && ((uintptr_t)q.x & 15) == 0, "grad_y / x must be 16-B aligned");
    VS_CHECK(((uintptr_t)q.dw & 15) == 0 && (!q.db || ((uintptr_t)q.db & 15) == 0), "dw / db must be 16-B aligned");
  }
  return VS_OK;
}

extern "C" long long vs_token_wgrad_grouped_workspace_bytes(const vs_wgrad_problem* probs, int n) {
  if (!probs || n <= 0) return 0;
  long long mx = 0;
  for_each_launch(probs, n, 1, [&](int, const Plan& pl) {
    if (pl.part_floats > mx) mx = pl.part_floats;
    return VS_OK;
  });
  return mx * 4 + 256;
}

extern "C" int vs_token_wgrad_grouped(int dtype, const vs_wgrad_problem* probs, int n, void* workspace,
                                      void* stream) {
  VS_CHECK(dtype == VS_BF16 || dtype == VS_F32, "dtype (of dw / db) must be VS_F32 or VS_BF16");
  const int rc = check_problems(probs, n);
  if (rc != VS_OK) return rc;
  if (n == 0) return VS_OK;
  const long long need = vs_token_wgrad_grouped_workspace_bytes(probs, n);
  VS_CHECK(need <= 256 || (workspace && ((uintptr_t)workspace & 15) == 0), "workspace: 16-B aligned, sized by "
           "vs_token_wgrad_grouped_workspace_bytes");
  hipStream_t st = (hipStream_t)stream;
  // the next chunk's DMA pieces are issued between the MFMA steps (all at once after the
  // barrier, every wave at the same time, they idled the MFMA pipe: round 5)
  const int spread = 1;
  return for_each_launch(probs, n, dtype == VS_F32, [&](int cfg, const Plan& pl) -> int {
    VS_CHECK(pl.wgs > 0 && pl.wgs < (1ll << 31), "bad workgroup count");
    float* part = (float*)workspace;
    float* pb = part ? part + pl.tile_floats : nullptr;
    const dim3 g((unsigned)pl.wgs);
    if (cfg == 0) {
      hipLaunchKernelGGL((token_wgrad_kernel<256, 128, 4, 2, 3>), g, dim3(512), 0, st, pl.g, part, pb, spread);
    } else {
      hipLaunchKernelGGL((token_wgrad_kernel<128, 128, 4, 2, 4>), g, dim3(512), 0, st, pl.g, part, pb, spread);
    }
    VS_LAUNCH_CHECK();
    if (pl.items > 0) {
      const dim3 gr((unsigned)(pl.items / 64));
      // 16 split groups per block below 512 blocks, else 4 (profiles/r5_wgrad_reduce_ab.txt)
      const bool wide = pl.items / 64 < 512;
      if (cfg == 0 && wide)
        hipLaunchKernelGGL((token_wgrad_reduce_kernel<256, 128, 4, 2, 16>), gr, dim3(1024), 0, st, pl.g,
                           (const float*)part, (const float*)pb);
      else if (cfg == 0)
        hipLaunchKernelGGL((token_wgrad_reduce_kernel<256, 128, 4, 2, 4>), gr, dim3(256), 0, st, pl.g,
                           (const float*)part, (const float*)pb);
      else if (wide)
        hipLaunchKernelGGL((token_wgrad_reduce_kernel<128, 128, 4, 2, 16>), gr, dim3(1024), 0, st, pl.g,
                           (const float*)part, (const float*)pb);
      else
        hipLaunchKernelGGL((token_wgrad_reduce_kernel<128, 128, 4, 2, 4>), gr, dim3(256), 0, st, pl.g,
                           (const float*)part, (const float*)pb);
      VS_LAUNCH_CHECK();
    }
    return VS_OK;
  });
}

extern "C" long long vs_token_wgrad_workspace_bytes(long long tokens, int N, int K) {
  if (tokens <= 0 || N <= 0 || K <= 0) return 0;
  vs_wgrad_problem q = {nullptr, nullptr, nullptr, (void*)1, N, K, tokens, N, K};
  return vs_token_wgrad_grouped_workspace_bytes(&q, 1);
}

extern "C" int vs_token_wgrad(int dtype, const void* grad_y, long long ld_grad_y, const void* x, long long ld_x,
                              void* dw, void* db, void* workspace, long long tokens, int N, int K, void* stream) {
  vs_wgrad_problem q = {grad_y, x, dw, db, ld_grad_y, ld_x, tokens, N, K};
  return vs_token_wgrad_grouped(dtype, &q, 1, workspace, stream);
}
