// Mask head: logits[b,q,n] = sum_c E[b,q,c] * P[b,n,c]  (HF:m2f:2040-2051 einsum
// 'bqc,bchw->bqhw' with the pixel embedding kept channels-last, P = [B, H*W, C]),
// and the masked-attention bitmask derived from it (HF:m2f:2049-2055, row fix
// HF:m2f:1912-1914).
//
// GEMM: per batch M = Q (queries, <=128 per workgroup z-slice), N = H*W pixels,
// K = C.  Both operands are K-contiguous (E row-major, P channels-last), so every MFMA
// fragment is a contiguous 16-B (bf16) / 4-B (f32) read: E for the workgroup's 128
// query rows is staged once in LDS (rows padded by 16 B -> conflict-free ds_read_b128),
// P fragments are loaded straight from HBM (each pixel row is read exactly once per
// launch: the kernel is HBM-bound, AI ~ 2Q flop per 4+2C/Q bytes).  bf16 path:
// v_mfma_f32_32x32x16_bf16; f32 path (parity mode): v_mfma_f32_32x32x2_f32 (exact
// f32 products, k-ordered f32 accumulation).  4 waves per workgroup, one 32-pixel
// column tile per wave per iteration, 4 query tiles of 32 per wave (64 acc VGPRs).
//
// Bitmask: one workgroup per (b, q): bilinear (align_corners=False, PyTorch's
// area_pixel_compute_source_index rule) resize of the logits row to (th, tw), blocked
// bit = sigmoid(v) < 0.5, 32 keys per u32 word (bit k%32 of word k/32); a row blocked
// at every key is written as all-zero (un-blocked), so the consumer needs no fix-up.
#include "common.h"

namespace vs {
namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

constexpr int kQT = 4;          // 32-row query tiles per workgroup (128 rows)
constexpr int kWaves = 4;

template <typename T, int KC>  // KC: compile-time channel count (0 = runtime K)
__global__ void __launch_bounds__(256) mask_head_fwd_kernel(const T* __restrict__ E, const T* __restrict__ P,
                                                            float* __restrict__ out, int Q, int N, int Kr) {
  const int K = KC > 0 ? KC : Kr;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* sE = reinterpret_cast<T*>(smem_raw);
  const int ldE = K + 16 / (int)sizeof(T);  // pad each row by 16 bytes
  const int b = blockIdx.y;
  const int q0 = blockIdx.z * 32 * kQT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, hh = lane >> 5;
  // ---- stage E rows [q0, q0+128) of batch b into LDS (zero rows past Q)
  {
    constexpr int V = 16 / sizeof(T);
    constexpr int kBatch = 8;   // loads in flight per thread before their LDS stores
    const int chunks = K / V;
    const int total = 32 * kQT * chunks;
    for (int base = 0; base < total; base += 256 * kBatch) {
      uint4 v[kBatch];
#pragma unroll
      for (int k = 0; k < kBatch; ++k) {
        const int idx = base + threadIdx.x + 256 * k;
        const int row = idx / chunks, c = (idx % chunks) * V;
        v[k] = make_uint4(0, 0, 0, 0);
        if (idx < total && q0 + row < Q) v[k] = *reinterpret_cast<const uint4*>(E + ((size_t)b * Q + q0 + row) * K + c);
      }
#pragma unroll
      for (int k = 0; k < kBatch; ++k) {
        const int idx = base + threadIdx.x + 256 * k;
        const int row = idx / chunks, c = (idx % chunks) * V;
        if (idx < total) *reinterpret_cast<uint4*>(sE + row * ldE + c) = v[k];
      }
    }
  }
  __syncthreads();
  const T* Pb = P + (size_t)b * N * K;
  float* Ob = out + (size_t)b * Q * N;
  const int tiles = (N + 31) / 32;
  for (int tile = blockIdx.x * kWaves + wave; tile < tiles; tile += gridDim.x * kWaves) {
    const int n0 = tile * 32;
    const int n = n0 + r;
    const bool nvalid = n < N;
    f32x16_t acc[kQT];
#pragma unroll
    for (int t = 0; t < kQT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
    const T* prow = Pb + (size_t)(nvalid ? n : 0) * K;
    if constexpr (sizeof(T) == 2) {
      for (int k0 = 0; k0 < K; k0 += 16) {
        bf16x8_t bfrag = *reinterpret_cast<const bf16x8_t*>(prow + k0 + 8 * hh);
        if (!nvalid) bfrag = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int t = 0; t < kQT; ++t) {
          const bf16x8_t afrag = *reinterpret_cast<const bf16x8_t*>(sE + (32 * t + r) * ldE + k0 + 8 * hh);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afrag, bfrag, acc[t], 0, 0, 0);
        }
      }
    } else {
      for (int k0 = 0; k0 < K; k0 += 2) {
        float bv = nvalid ? (float)prow[k0 + hh] : 0.f;
#pragma unroll
        for (int t = 0; t < kQT; ++t) {
          const float av = (float)sE[(32 * t + r) * ldE + k0 + hh];
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[t], 0, 0, 0);
        }
      }
    }
    if (nvalid) {
#pragma unroll
      for (int t = 0; t < kQT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int row = q0 + 32 * t + (i & 3) + 8 * (i >> 2) + 4 * hh;
          if (row < Q) Ob[(size_t)row * N + n] = acc[t][i];
        }
    }
  }
}


// bf16 forward with a compile-time channel count: each wave streams its pixel tiles with
// the NEXT tile's P fragments (KC/16 x 16 B per lane) in flight while the current tile's
// MFMAs run, so at one wave per SIMD the HBM latency stays hidden.
// GROUPED: logits row (b, q) is stored at row ((q / G) B + b) G + q % G of out (q / G by the
// multiply-shift gm = ceil(2^20 / G), exact for Q G < 2^20): the matched maps of S decoder
// steps x G targets land in (step, image, target) order straight from one launch.
template <int KC, bool GROUPED = false>
__global__ void __launch_bounds__(256) mask_head_fwd_bf16_kernel(const bf16* __restrict__ E, const bf16* __restrict__ P,
                                                                 float* __restrict__ out, int Q, int N, int G = 0,
                                                                 unsigned gm = 0) {
  constexpr int S = KC / 16;
  constexpr int ldE = KC + 8;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16* sE = reinterpret_cast<bf16*>(smem_raw);
  const int b = blockIdx.y;
  const int q0 = blockIdx.z * 32 * kQT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, hh = lane >> 5;
  {
    constexpr int CH = KC / 8;
    constexpr int EC = 32 * kQT * CH / 256;
    uint4 v[EC];
#pragma unroll
    for (int k = 0; k < EC; ++k) {
      const int idx = threadIdx.x + 256 * k;
      const int row = idx / CH, c = (idx % CH) * 8;
      v[k] = q0 + row < Q ? *reinterpret_cast<const uint4*>(E + ((size_t)b * Q + q0 + row) * KC + c) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < EC; ++k) {
      const int idx = threadIdx.x + 256 * k;
      const int row = idx / CH, c = (idx % CH) * 8;
      *reinterpret_cast<uint4*>(sE + row * ldE + c) = v[k];
    }
  }
  __syncthreads();
  const bf16* Pb = P + (size_t)b * N * KC;
  float* Ob = out + (size_t)b * Q * N;
  const int tiles = (N + 31) / 32;
  const int stride = gridDim.x * kWaves;
  bf16x8_t cur[S], nxt[S];
  auto load = [&](bf16x8_t* f, int tile) {
    const int n = tile * 32 + r;
    const bf16* prow = Pb + (size_t)(n < N ? n : 0) * KC + 8 * hh;
#pragma unroll
    for (int s = 0; s < S; ++s) f[s] = *reinterpret_cast<const bf16x8_t*>(prow + 16 * s);
  };
  int tile = blockIdx.x * kWaves + wave;
  if (tile < tiles) load(cur, tile);
  for (; tile < tiles; tile += stride) {
    if (tile + stride < tiles) load(nxt, tile + stride);
    const int n = tile * 32 + r;
    const bool nvalid = n < N;
    f32x16_t acc[kQT];
#pragma unroll
    for (int t = 0; t < kQT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      __builtin_amdgcn_sched_barrier(0);
      const bf16x8_t bfrag = nvalid ? cur[s] : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int t = 0; t < kQT; ++t) {
        const bf16x8_t afrag = *reinterpret_cast<const bf16x8_t*>(sE + (32 * t + r) * ldE + 16 * s + 8 * hh);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afrag, bfrag, acc[t], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (nvalid) {
#pragma unroll
      for (int t = 0; t < kQT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int row = q0 + 32 * t + (i & 3) + 8 * (i >> 2) + 4 * hh;
          if (row < Q) {
            if constexpr (GROUPED) {
              const unsigned d = (unsigned)(((unsigned long long)row * gm) >> 20);
              out[((size_t)(d * gridDim.y + b) * G + (row - d * G)) * N + n] = acc[t][i];
            } else {
              Ob[(size_t)row * N + n] = acc[t][i];
            }
          }
        }
    }
#pragma unroll
    for (int s = 0; s < S; ++s) cur[s] = nxt[s];
  }
}

// ---------------------------------------------------------------------------------
// Backward (bf16): one pass over the logits gradient produces both operand grads.
//   dP[b,n,:] = sum_q gL[b,q,n] E[b,q,:]          (M = pixels, N = C, K = Q)
//   dE[b,q,:] = sum_n gL[b,q,n] P[b,n,:]          (M = Q, N = C, K = pixels: split-K)
// A workgroup (4 waves) walks 32-pixel tiles of one image.  Everything is staged in LDS
// in its NATURAL layout with 16-B stores (E [q][C] once, the gL tile [q][32] as bf16,
// the P tile [32][C]); operands that the MFMA needs in the other orientation (gL^T and E
// for dP, P for dE) are read with the gfx950 transpose read ds_read_b64_tr_b16
// (cdna_hip_programming.md T10): a 16-lane group reads a 4-row x 16-column block and
// each lane receives one column.  Row pitches of 64 B mod 256 keep those reads in
// distinct banks.  The next tile's gL / P are loaded into registers while the current
// tile computes (one barrier pair per tile).  dE accumulates in registers across the
// workgroup's tiles and is written once as a per-workgroup f32 partial;
// `mask_head_bwd_reduce` sums the partials (deterministic).
// HBM traffic per call: gL (f32) + P read once, dP written once.
typedef short bf16x4v_t __attribute__((ext_vector_type(4)));

// MFMA operand (8 k-values of one column) from an LDS image whose ROWS are the k index:
// rows k0 + 8hh + {0..3} and k0 + 8hh + 4 + {0..3}, column cbase + (lane & 31)
__device__ __forceinline__ bf16x8_t tr_operand(const bf16* img, int pitch, int k0, int cbase, int lane) {
  const int hh = lane >> 5;
  const int row = k0 + 8 * hh + ((lane & 15) >> 2);
  const int col = cbase + (lane & 16) + 4 * (lane & 3);
  typedef __attribute__((address_space(3))) bf16x4v_t lds_v4;
  const bf16x4v_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(img + row * pitch + col));
  const bf16x4v_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(img + (row + 4) * pitch + col));
  bf16x8_t v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return v;
}

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  const bf16 x = __float2bfloat16(a), y = __float2bfloat16(b);
  return (uint32_t)(*reinterpret_cast<const uint16_t*>(&x)) | ((uint32_t)(*reinterpret_cast<const uint16_t*>(&y)) << 16);
}

// ACC: dP += (the pixel-embedding gradient summed over the decoder's mask-head calls in
// place, instead of autograd adding 10 [B, HW, C] tensors)
template <int CT, int TN, bool ACC = false>  // c-tiles (of 32) per wave (C = 128 * CT); pixels per tile (32 or 64)
__global__ void __launch_bounds__(256) mask_head_bwd_kernel(const float* __restrict__ gL, const bf16* __restrict__ E,
                                                            const bf16* __restrict__ P, bf16* __restrict__ dP,
                                                            float* __restrict__ dEpart, int Q, int N) {
  constexpr int C = 128 * CT;
  constexpr int NT = TN / 32;
  constexpr int EP = C + 32;      // E / P row pitch (elements): 2*EP bytes = 64 mod 256
  constexpr int GP = TN == 32 ? 32 : 96;   // gL tile row pitch: 64 / 192 B (4 rows -> distinct banks)
  constexpr int CH = C / 8;       // 16-B chunks per P row
  constexpr int PCH = TN * CH / 256;  // P chunks per thread per tile
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16* sE = reinterpret_cast<bf16*>(smem_raw);      // [128][EP]
  bf16* sG = sE + 128 * EP;                          // [128][GP]
  bf16* sP = sG + 128 * GP;                          // [TN][EP]
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, hh = lane >> 5;
  {  // all of this thread's E chunks in flight at once, then the LDS stores
    constexpr int EC = 128 * CH / 256;
    uint4 ue[EC];
#pragma unroll
    for (int k = 0; k < EC; ++k) {
      const int idx = threadIdx.x + 256 * k;
      const int q = idx / CH, c0 = (idx - q * CH) * 8;
      ue[k] = q < Q ? *reinterpret_cast<const uint4*>(E + ((size_t)b * Q + q) * C + c0) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < EC; ++k) {
      const int idx = threadIdx.x + 256 * k;
      const int q = idx / CH, c0 = (idx - q * CH) * 8;
      *reinterpret_cast<uint4*>(sE + q * EP + c0) = ue[k];
    }
  }
  f32x16_t accE[4][CT];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int u = 0; u < CT; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) accE[t][u][i] = 0.f;
  const float* gLb = gL + (size_t)b * Q * N;
  const bf16* Pb = P + (size_t)b * N * C;
  bf16* dPb = dP + (size_t)b * N * C;
  const int tiles = (N + TN - 1) / TN;
  // register staging of one tile: gL row q = tid/2, TN/2 pixels; PCH P chunks
  constexpr int GH = TN / 2;
  const int gq = threadIdx.x >> 1, gh = (threadIdx.x & 1) * GH;
  float4 rg[GH / 4];
  uint4 rp[PCH];
  auto load_tile = [&](int n0) {
    if (gq < Q && n0 + gh + GH <= N && (N & 3) == 0) {
      const float4* src = reinterpret_cast<const float4*>(gLb + (size_t)gq * N + n0 + gh);
#pragma unroll
      for (int i = 0; i < GH / 4; ++i) rg[i] = src[i];
    } else {
#pragma unroll
      for (int i = 0; i < GH / 4; ++i) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n0 + gh + 4 * i + j;
          v[j] = (gq < Q && n < N) ? gLb[(size_t)gq * N + n] : 0.f;
        }
        rg[i] = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
#pragma unroll
    for (int k = 0; k < PCH; ++k) {
      const int idx = threadIdx.x + k * 256;
      const int n = idx / CH, c0 = (idx - n * CH) * 8;
      rp[k] = (n0 + n < N) ? *reinterpret_cast<const uint4*>(Pb + (size_t)(n0 + n) * C + c0) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < GH / 8; ++i) {
      uint4 w;
      w.x = pack_bf16x2(rg[2 * i].x, rg[2 * i].y); w.y = pack_bf16x2(rg[2 * i].z, rg[2 * i].w);
      w.z = pack_bf16x2(rg[2 * i + 1].x, rg[2 * i + 1].y); w.w = pack_bf16x2(rg[2 * i + 1].z, rg[2 * i + 1].w);
      *reinterpret_cast<uint4*>(sG + gq * GP + gh + 8 * i) = w;
    }
#pragma unroll
    for (int k = 0; k < PCH; ++k) {
      const int idx = threadIdx.x + k * 256;
      const int n = idx / CH, c0 = (idx - n * CH) * 8;
      *reinterpret_cast<uint4*>(sP + n * EP + c0) = rp[k];
    }
  };
  int tile = blockIdx.x;
  if (tile < tiles) load_tile(tile * TN);
  for (; tile < tiles; tile += gridDim.x) {
    const int n0 = tile * TN;
    __syncthreads();                 // previous tile's LDS reads are done
    store_tile();
    __syncthreads();
    if (tile + gridDim.x < tiles) load_tile((tile + gridDim.x) * TN);   // in flight during the MFMAs
    // ---- dP tile [TN n][C]: A = gL^T (rows n, k = q), B = E (k = q, cols c).  The
    // fragments of k-step s+1 are read before the MFMAs of step s issue (one wave per
    // SIMD: nothing else hides the LDS latency); CT x NT independent accumulators.
    {
      f32x16_t acc[CT][NT];
#pragma unroll
      for (int u = 0; u < CT; ++u)
#pragma unroll
        for (int m = 0; m < NT; ++m)
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[u][m][i] = 0.f;
      bf16x8_t fa[2][NT], fb[2][CT];
#pragma unroll
      for (int m = 0; m < NT; ++m) fa[0][m] = tr_operand(sG, GP, 0, 32 * m, lane);
#pragma unroll
      for (int u = 0; u < CT; ++u) fb[0][u] = tr_operand(sE, EP, 0, (wave * CT + u) * 32, lane);
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int cur = s & 1, nxt = cur ^ 1;
        __builtin_amdgcn_sched_barrier(0);
        if (s + 1 < 8) {
#pragma unroll
          for (int m = 0; m < NT; ++m) fa[nxt][m] = tr_operand(sG, GP, 16 * (s + 1), 32 * m, lane);
#pragma unroll
          for (int u = 0; u < CT; ++u) fb[nxt][u] = tr_operand(sE, EP, 16 * (s + 1), (wave * CT + u) * 32, lane);
        }
        __builtin_amdgcn_sched_barrier(0);   // keep the next step's reads ahead of these MFMAs
#pragma unroll
        for (int u = 0; u < CT; ++u)
#pragma unroll
          for (int m = 0; m < NT; ++m)
            acc[u][m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[cur][u], fa[cur][m], acc[u][m], 0, 0, 0);
      }
      // acc[u][m] is the dP^T tile: lane column = pixel n0 + 32m + r, rows = channels
      // c0 + (i & 3) + 8 (i >> 2) + 4 hh -> four consecutive channels per 8-B store
#pragma unroll
      for (int m = 0; m < NT; ++m) {
        const int n = n0 + 32 * m + r;
        if (n < N) {
          bf16* dst = dPb + (size_t)n * C + wave * CT * 32 + 4 * hh;
#pragma unroll
          for (int u = 0; u < CT; ++u)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              float a0 = acc[u][m][4 * g], a1 = acc[u][m][4 * g + 1], a2 = acc[u][m][4 * g + 2],
                    a3 = acc[u][m][4 * g + 3];
              if constexpr (ACC) {
                const uint2 o = *reinterpret_cast<const uint2*>(dst + 32 * u + 8 * g);
                a0 += __uint_as_float(o.x << 16);
                a1 += __uint_as_float(o.x & 0xffff0000u);
                a2 += __uint_as_float(o.y << 16);
                a3 += __uint_as_float(o.y & 0xffff0000u);
              }
              uint2 w;
              w.x = pack_bf16x2(a0, a1);
              w.y = pack_bf16x2(a2, a3);
              *reinterpret_cast<uint2*>(dst + 32 * u + 8 * g) = w;
            }
        }
      }
    }
    // ---- dE partial [128 q][C] += gL_tile [128 x TN] . P_tile [TN x C]
    {
      bf16x8_t fa[2][4], fb[2][CT];
#pragma unroll
      for (int t = 0; t < 4; ++t) fa[0][t] = *reinterpret_cast<const bf16x8_t*>(sG + (32 * t + r) * GP + 8 * hh);
#pragma unroll
      for (int u = 0; u < CT; ++u) fb[0][u] = tr_operand(sP, EP, 0, (wave * CT + u) * 32, lane);
#pragma unroll
      for (int s = 0; s < 2 * NT; ++s) {
        const int cur = s & 1, nxt = cur ^ 1;
        __builtin_amdgcn_sched_barrier(0);
        if (s + 1 < 2 * NT) {
#pragma unroll
          for (int t = 0; t < 4; ++t)
            fa[nxt][t] = *reinterpret_cast<const bf16x8_t*>(sG + (32 * t + r) * GP + 16 * (s + 1) + 8 * hh);
#pragma unroll
          for (int u = 0; u < CT; ++u) fb[nxt][u] = tr_operand(sP, EP, 16 * (s + 1), (wave * CT + u) * 32, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int u = 0; u < CT; ++u)
            accE[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[cur][u], fa[cur][t], accE[t][u], 0, 0, 0);
      }
    }
  }
  // accE[t][u] is the dE^T tile: lane column = query 32t + r, rows = channels
  // (wave * CT + u) * 32 + (i & 3) + 8 (i >> 2) + 4 hh -> 16-B stores of 4 channels
  float* part = dEpart + ((size_t)blockIdx.x * gridDim.y + b) * Q * C;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int q = 32 * t + r;
    if (q < Q) {
#pragma unroll
      for (int u = 0; u < CT; ++u)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<float4*>(part + (size_t)q * C + (wave * CT + u) * 32 + 8 * g + 4 * hh) =
              make_float4(accE[t][u][4 * g], accE[t][u][4 * g + 1], accE[t][u][4 * g + 2], accE[t][u][4 * g + 3]);
    }
  }
}

__global__ void __launch_bounds__(256) mask_head_bwd_reduce(const float* __restrict__ part, bf16* __restrict__ dE,
                                                            int nparts, long long per_part) {
  // 4 consecutive elements per thread (per_part % 4 == 0: C is a multiple of 128), 8 parts
  // in flight; parts summed in index order (deterministic)
  const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= per_part) return;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  int p = 0;
  for (; p + 8 <= nparts; p += 8) {
    float4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const float4*>(part + (size_t)(p + k) * per_part + i);
#pragma unroll
    for (int k = 0; k < 8; ++k) { s.x += v[k].x; s.y += v[k].y; s.z += v[k].z; s.w += v[k].w; }
  }
  for (; p < nparts; ++p) {
    const float4 v = *reinterpret_cast<const float4*>(part + (size_t)p * per_part + i);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  uint2 w;
  w.x = pack_bf16x2(s.x, s.y);
  w.y = pack_bf16x2(s.z, s.w);
  *reinterpret_cast<uint2*>(dE + i) = w;
}

// PyTorch upsample_bilinear2d (align_corners=False) source index for one axis.
__device__ __forceinline__ void src_index(int dst, int in, int out, int& i0, int& i1, float& l0, float& l1) {
  const float scale = (float)in / (float)out;
  float s = scale * ((float)dst + 0.5f) - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = (int)s;
  i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  l1 = s - (float)i0;
  l0 = 1.f - l1;
}

__global__ void __launch_bounds__(1024) attn_bitmask_kernel(const float* __restrict__ logits,
                                                            uint32_t* __restrict__ words, int H, int W,
                                                            int th, int tw, int nwords) {
  // one workgroup (16 waves) per (b, q) row; a wave evaluates 64 consecutive keys and
  // its ballot IS two output words (bit k % 32 of word k / 32), written directly
  __shared__ int s_count;
  const long long row = blockIdx.x;
  const float* src = logits + row * (long long)H * W;
  uint32_t* dst = words + row * nwords;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_count = 0;
  __syncthreads();
  const int total = th * tw;
  int local = 0;
  for (int base = wave * 64; base < total; base += 1024) {
    const int k = base + lane;
    bool blocked = false;
    if (k < total) {
      const int y = k / tw, x = k - y * tw;
      int y0, y1, x0, x1;
      float ly0, ly1, lx0, lx1;
      src_index(y, H, th, y0, y1, ly0, ly1);
      src_index(x, W, tw, x0, x1, lx0, lx1);
      const float v = ly0 * (lx0 * src[y0 * W + x0] + lx1 * src[y0 * W + x1]) +
                      ly1 * (lx0 * src[y1 * W + x0] + lx1 * src[y1 * W + x1]);
      const float sg = 1.f / (1.f + expf(-v));
      blocked = sg < 0.5f;
    }
    const unsigned long long m = __ballot(blocked);
    if (lane == 0) {
      const int w0 = base >> 5;
      dst[w0] = (uint32_t)m;
      if (w0 + 1 < nwords) dst[w0 + 1] = (uint32_t)(m >> 32);
      local += __popcll(m);
    }
  }
  if (lane == 0) atomicAdd(&s_count, local);
  __syncthreads();
  // a row blocked at every key is written un-blocked (HF:m2f:1912-1914); words past the
  // last key (nwords * 32 > total) were written by the wave that covers them
  if (s_count == total)
    for (int i = threadIdx.x; i < nwords; i += blockDim.x) dst[i] = 0u;
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" int vs_mask_head_forward(int dtype, const void* E, const void* P, float* logits, int B, int Q,
                                    int C, int H, int W, void* stream) {
  VS_CHECK(E && P && logits, "null pointer");
  VS_CHECK(B > 0 && Q > 0 && C > 0 && H > 0 && W > 0, "bad sizes");
  const int N = H * W;
  hipStream_t st = (hipStream_t)stream;
  const int qz = (Q + 32 * kQT - 1) / (32 * kQT);
  const int tiles = (N + 31) / 32;
  int gx = (tiles + kWaves - 1) / kWaves;
  const int cap = (2048 + B * qz - 1) / (B * qz);
  if (gx > cap) gx = cap;
  dim3 grid(gx, B, qz);
  if (dtype == VS_BF16) {
    VS_CHECK(C % 16 == 0 && C <= 512, "bf16 mask head needs C % 16 == 0, C <= 512");
    const size_t lds = (size_t)32 * kQT * (C + 8) * 2;
    // pipelined kernel: one workgroup per CU (1 wave/SIMD by registers), tiles streamed
    dim3 pgrid(grid);
    const int pcap = (256 + B * qz - 1) / (B * qz);
    if ((int)pgrid.x > pcap) pgrid.x = pcap;
    if (C == 256)
      hipLaunchKernelGGL((mask_head_fwd_bf16_kernel<256>), pgrid, dim3(256), lds, st, (const bf16*)E,
                         (const bf16*)P, logits, Q, N);
    else if (C == 128)
      hipLaunchKernelGGL((mask_head_fwd_bf16_kernel<128>), pgrid, dim3(256), lds, st, (const bf16*)E,
                         (const bf16*)P, logits, Q, N);
    else
      hipLaunchKernelGGL((mask_head_fwd_kernel<bf16, 0>), grid, dim3(256), lds, st, (const bf16*)E,
                         (const bf16*)P, logits, Q, N, C);
  } else if (dtype == VS_F32) {
    VS_CHECK(C % 4 == 0 && C <= 256, "f32 mask head needs C % 4 == 0, C <= 256");
    const size_t lds = (size_t)32 * kQT * (C + 4) * 4;
    hipLaunchKernelGGL((mask_head_fwd_kernel<float, 0>), grid, dim3(256), lds, st, (const float*)E, (const float*)P,
                       logits, Q, N, C);
  } else {
    VS_CHECK(false, "dtype must be VS_F32 or VS_BF16");
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_mask_head_forward_grouped(const void* E, const void* P, float* logits, int B, int Q, int C, int H,
                                            int W, int group, void* stream) {
  VS_CHECK(E && P && logits, "null pointer");
  VS_CHECK(B > 0 && Q > 0 && H > 0 && W > 0, "bad sizes");
  VS_CHECK(C == 128 || C == 256, "grouped mask head: bf16, C in {128, 256}");
  VS_CHECK(group > 0 && Q % group == 0 && (long long)Q * group < (1LL << 20), "group must divide Q, Q * group < 2^20");
  const int N = H * W;
  const int qz = (Q + 32 * kQT - 1) / (32 * kQT);
  const int tiles = (N + 31) / 32;
  int gx = (tiles + kWaves - 1) / kWaves;
  const int pcap = (256 + B * qz - 1) / (B * qz);
  if (gx > pcap) gx = pcap;
  const unsigned gm = (unsigned)(((1u << 20) + group - 1) / group);
  const size_t lds = (size_t)32 * kQT * (C + 8) * 2;
  hipStream_t st = (hipStream_t)stream;
  if (C == 256)
    hipLaunchKernelGGL((mask_head_fwd_bf16_kernel<256, true>), dim3(gx, B, qz), dim3(256), lds, st, (const bf16*)E,
                       (const bf16*)P, logits, Q, N, group, gm);
  else
    hipLaunchKernelGGL((mask_head_fwd_bf16_kernel<128, true>), dim3(gx, B, qz), dim3(256), lds, st, (const bf16*)E,
                       (const bf16*)P, logits, Q, N, group, gm);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_attn_bitmask(const float* logits, uint32_t* words, int rows, int H, int W, int th, int tw,
                               void* stream) {
  VS_CHECK(logits && words, "null pointer");
  VS_CHECK(rows > 0 && H > 0 && W > 0 && th > 0 && tw > 0, "bad sizes");
  const int nwords = (th * tw + 31) / 32;
  VS_CHECK(nwords * 4 <= 64 * 1024, "target too large");
  hipLaunchKernelGGL(attn_bitmask_kernel, dim3(rows), dim3(1024), 0, (hipStream_t)stream, logits, words,
                     H, W, th, tw, nwords);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

static int mask_head_bwd_parts(int B) { return B >= 64 ? 1 : (256 + B - 1) / B; }

// ---------------------------------------------------------------------------------
// Point scatter: the adjoint of the mask losses' bilinear point sampling into dense maps.
// One workgroup per (pair, band of RB map rows): the band lives in LDS (<= 64 KB), every
// point of the pair is visited and the corners inside the band are added there (LDS f32
// atomics: a pair's 12544 points land on distinct cells mostly), then the band is written
// out once with 16-B stores -- no zero-fill pass and no global atomics (torch's
// grid_sampler_2d_backward: one global f32 atomic per corner, one lane per row).
constexpr int kScatterLds = 16384;    // floats per band

__global__ void __launch_bounds__(256) point_scatter_kernel(const float* __restrict__ gp,
                                                            const float* __restrict__ grid, float* __restrict__ maps,
                                                            int S, int B, int K, int n, int H, int W, int RB) {
  __shared__ __attribute__((aligned(16))) float band[kScatterLds];
  const int pair = blockIdx.x;                       // (s, b, k)
  const int r0 = blockIdx.y * RB;
  const int rows = min(RB, H - r0);
  const int k = pair % K, b = (pair / K) % B, s = pair / (K * B);
  for (int i = threadIdx.x; i < rows * W; i += 256) band[i] = 0.f;
  __syncthreads();
  const float* g = gp + (size_t)pair * n;
  const float2* xy = reinterpret_cast<const float2*>(grid) + (size_t)pair * n;
  const float fW = (float)W, fH = (float)H;
  for (int p = threadIdx.x; p < n; p += 256) {
    const float go = g[p];
    const float2 c = xy[p];
    // grid_sampler_compute_source_index, align_corners = false
    const float ix = ((c.x + 1.f) * fW - 1.f) / 2.f;
    const float iy = ((c.y + 1.f) * fH - 1.f) / 2.f;
    const float ix_nw = floorf(ix), iy_nw = floorf(iy);
    const float ix_se = ix_nw + 1.f, iy_se = iy_nw + 1.f;
    const float w_nw = (ix_se - ix) * (iy_se - iy);
    const float w_ne = (ix - ix_nw) * (iy_se - iy);
    const float w_sw = (ix_se - ix) * (iy - iy_nw);
    const float w_se = (ix - ix_nw) * (iy - iy_nw);
    const int x0 = (int)ix_nw, y0 = (int)iy_nw;
    const float wts[4] = {w_nw, w_ne, w_sw, w_se};
#pragma unroll
    for (int cnr = 0; cnr < 4; ++cnr) {
      const int yy = y0 + (cnr >> 1), xx = x0 + (cnr & 1);
      const int ry = yy - r0;
      if (xx >= 0 && xx < W && yy >= 0 && yy < H && ry >= 0 && ry < rows) atomicAdd(&band[ry * W + xx], wts[cnr] * go);
    }
  }
  __syncthreads();
  float* out = maps + (((size_t)b * S + s) * K + k) * H * W + (size_t)r0 * W;
  const int nv = rows * W;
  if ((nv & 3) == 0) {
    for (int i = threadIdx.x; i < nv / 4; i += 256)
      reinterpret_cast<float4*>(out)[i] = reinterpret_cast<const float4*>(band)[i];
  } else {
    for (int i = threadIdx.x; i < nv; i += 256) out[i] = band[i];
  }
}

// Point gather: out[n, p] = bilinear sample of maps[rows[n]] at coords[n, p] in [0, 1]
// (point_sample = grid_sample with align_corners=False, zero padding: ATen's unnormalisation
// ((2c - 1 + 1) W - 1) / 2 and corner weights), one thread per point -- the MaskDINO mask
// losses' labels, each query's OWN target map sampled at its points, without materialising
// the per-query maps or sampling every target channel.
// a map element as a sample value: f32 as is; u8 is a bool mask (any non-zero byte is True:
// torch's bool tensors made by views / casts of byte data may hold 0xFF, not 0x01)
__device__ __forceinline__ float map_value(float v) { return v; }
__device__ __forceinline__ float map_value(unsigned char v) { return v != 0 ? 1.f : 0.f; }

template <typename T, bool GRID>
__global__ void __launch_bounds__(256) point_sample_rows_kernel(const T* __restrict__ maps,
                                                                const long long* __restrict__ rows,
                                                                const float* __restrict__ coords,
                                                                float* __restrict__ out, int H, int W, long long total,
                                                                int P, int sets_per_coord) {
  // XCD-aware block order (common.h xcd_swizzle): consecutive points of one map stay on one
  // XCD, so each XCD's L2 holds only its share of the maps.  Round-robin placement made every
  // XCD gather from every map (80 x 256^2 f32 = 21 MB against a 4 MB L2): 85 us per call at
  // the criterion's 37 632 uncertainty points per map, one L2 miss per corner
  const long long i = (long long)xcd_swizzle(blockIdx.x, gridDim.x) * 256 + threadIdx.x;
  if (i >= total) return;
  const long long n = i / P;
  const T* m = maps + (rows ? rows[n] : n) * (long long)H * W;
  // GRID: coords already in grid_sample's [-1, 1] space, one point set per sets_per_coord rows
  const long long ci = GRID ? (n / sets_per_coord) * P + (i - n * P) : i;
  const float2 c = reinterpret_cast<const float2*>(coords)[ci];
  const float gx = GRID ? c.x : 2.f * c.x - 1.f, gy = GRID ? c.y : 2.f * c.y - 1.f;
  const float ix = ((gx + 1.f) * (float)W - 1.f) / 2.f;
  const float iy = ((gy + 1.f) * (float)H - 1.f) / 2.f;
  const float fx = floorf(ix), fy = floorf(iy);
  const int x0 = (int)fx, y0 = (int)fy;
  const float w_nw = (fx + 1.f - ix) * (fy + 1.f - iy), w_ne = (ix - fx) * (fy + 1.f - iy);
  const float w_sw = (fx + 1.f - ix) * (iy - fy), w_se = (ix - fx) * (iy - fy);
  float v = 0.f;
  const bool xi0 = x0 >= 0 && x0 < W, xi1 = x0 + 1 >= 0 && x0 + 1 < W;
  const bool yi0 = y0 >= 0 && y0 < H, yi1 = y0 + 1 >= 0 && y0 + 1 < H;
  if (yi0 && xi0) v += map_value(m[(size_t)y0 * W + x0]) * w_nw;
  if (yi0 && xi1) v += map_value(m[(size_t)y0 * W + x0 + 1]) * w_ne;
  if (yi1 && xi0) v += map_value(m[(size_t)(y0 + 1) * W + x0]) * w_sw;
  if (yi1 && xi1) v += map_value(m[(size_t)(y0 + 1) * W + x0 + 1]) * w_se;
  out[i] = v;
}

extern "C" int vs_point_sample_rows(const float* maps, const long long* rows, const float* coords, float* out,
                                    int num_maps, int height, int width, int num_sets, int num_points,
                                    void* stream) {
  VS_CHECK(num_maps > 0 && height > 0 && width > 0 && num_sets >= 0 && num_points > 0, "bad sizes");
  const long long total = (long long)num_sets * num_points;
  if (total == 0) return VS_OK;
  VS_CHECK(maps && coords && out, "null pointer");
  VS_CHECK(rows || num_sets <= num_maps, "without rows, set n reads map n");
  VS_CHECK(((uintptr_t)coords & 7) == 0, "coords must be 8-B aligned");
  hipLaunchKernelGGL((point_sample_rows_kernel<float, false>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, maps, rows, coords, out, height, width, total, num_points, 1);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

// The set criterion's target labels at points straight from the bool (u8) target masks:
// no f32 copy of the full-resolution masks, one launch per point set (replaces
// grid_sample(masks.float(), ...) at HF:m2f:453-459 (matcher) and 700-724 (loss labels)).
extern "C" int vs_point_sample_masks(const unsigned char* masks, const long long* rows, const float* coords,
                                     float* out, int num_maps, int height, int width, int num_sets, int num_points,
                                     int grid_space, int sets_per_coord, void* stream) {
  VS_CHECK(num_maps > 0 && height > 0 && width > 0 && num_sets >= 0 && num_points > 0, "bad sizes");
  VS_CHECK(grid_space == 0 || sets_per_coord > 0, "sets_per_coord must be positive");
  const long long total = (long long)num_sets * num_points;
  if (total == 0) return VS_OK;
  VS_CHECK(masks && coords && out, "null pointer");
  VS_CHECK(rows || num_sets <= num_maps, "without rows, set n reads mask n");
  VS_CHECK(((uintptr_t)coords & 7) == 0, "coords must be 8-B aligned");
  const dim3 grid((unsigned)((total + 255) / 256));
  if (grid_space)
    hipLaunchKernelGGL((point_sample_rows_kernel<unsigned char, true>), grid, dim3(256), 0, (hipStream_t)stream,
                       masks, rows, coords, out, height, width, total, num_points, sets_per_coord);
  else
    hipLaunchKernelGGL((point_sample_rows_kernel<unsigned char, false>), grid, dim3(256), 0, (hipStream_t)stream,
                       masks, rows, coords, out, height, width, total, num_points, 1);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" long long vs_mask_head_backward_workspace_bytes(int B, int Q, int C) {
  return (long long)mask_head_bwd_parts(B) * B * Q * C * 4;
}

static int mask_head_backward_impl(int dtype, const float* grad_logits, const void* E, const void* P, void* grad_E,
                                   void* grad_P, void* workspace, int B, int Q, int C, int H, int W, bool acc,
                                   void* stream);

extern "C" int vs_mask_head_backward(int dtype, const float* grad_logits, const void* E, const void* P, void* grad_E,
                                     void* grad_P, void* workspace, int B, int Q, int C, int H, int W,
                                     void* stream) {
  return mask_head_backward_impl(dtype, grad_logits, E, P, grad_E, grad_P, workspace, B, Q, C, H, W, false, stream);
}

extern "C" int vs_mask_head_backward_ex(int dtype, const float* grad_logits, const void* E, const void* P,
                                        void* grad_E, void* grad_P, void* workspace, int B, int Q, int C, int H, int W,
                                        int accumulate_grad_P, void* stream) {
  return mask_head_backward_impl(dtype, grad_logits, E, P, grad_E, grad_P, workspace, B, Q, C, H, W,
                                 accumulate_grad_P != 0, stream);
}

static int mask_head_backward_impl(int dtype, const float* grad_logits, const void* E, const void* P, void* grad_E,
                                   void* grad_P, void* workspace, int B, int Q, int C, int H, int W, bool acc,
                                   void* stream) {
  VS_CHECK(grad_logits && E && P && grad_E && grad_P && workspace, "null pointer");
  VS_CHECK(dtype == VS_BF16, "the fused mask-head backward is the bf16 path (f32 parity mode uses vendor GEMMs)");
  VS_CHECK(B > 0 && Q > 0 && Q <= 128 && H > 0 && W > 0, "need 0 < Q <= 128");
  VS_CHECK(C == 128 || C == 256, "channels must be 128 or 256");
  const int N = H * W;
  const int parts = mask_head_bwd_parts(B);
  constexpr int TN = 64;
  const int tiles = (N + TN - 1) / TN;
  const int gx = parts < tiles ? parts : tiles;
  hipStream_t st = (hipStream_t)stream;
  const size_t lds = ((size_t)128 * (C + 32) + 128 * 96 + (size_t)TN * (C + 32)) * 2;
  float* part = (float*)workspace;
  if (gx < parts) VS_HIP(hipMemsetAsync(part + (size_t)gx * B * Q * C, 0, (size_t)(parts - gx) * B * Q * C * 4, st));
#define VS_MHB(CT_, ACC_)                                                                                 \
  hipLaunchKernelGGL((mask_head_bwd_kernel<CT_, TN, ACC_>), dim3(gx, B), dim3(256), lds, st, grad_logits, \
                     (const bf16*)E, (const bf16*)P, (bf16*)grad_P, part, Q, N)
  if (C == 256 && acc)
    VS_MHB(2, true);
  else if (C == 256)
    VS_MHB(2, false);
  else if (acc)
    VS_MHB(1, true);
  else
    VS_MHB(1, false);
#undef VS_MHB
  VS_LAUNCH_CHECK();
  const long long per = (long long)B * Q * C;
  hipLaunchKernelGGL(mask_head_bwd_reduce, dim3((int)((per / 4 + 255) / 256)), dim3(256), 0, st, part, (bf16*)grad_E,
                     parts, per);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_point_scatter(const float* grad_points, const float* grid, float* maps, int S, int B, int K, int n,
                                int H, int W, void* stream) {
  VS_CHECK(S > 0 && B > 0 && K > 0 && n >= 0 && H > 0 && W > 0, "bad sizes");
  VS_CHECK(W <= kScatterLds, "map rows wider than the LDS band");
  VS_CHECK(maps && (n == 0 || (grad_points && grid)), "null pointer");
  VS_CHECK(((uintptr_t)grid & 7) == 0 && ((uintptr_t)maps & 15) == 0, "grid must be 8-B and maps 16-B aligned");
  const int RB = kScatterLds / W < H ? kScatterLds / W : H;
  const long long pairs = (long long)S * B * K;
  VS_CHECK(pairs <= 0x7fffffff, "too many pairs");
  hipLaunchKernelGGL(point_scatter_kernel, dim3((unsigned)pairs, (H + RB - 1) / RB), dim3(256), 0,
                     (hipStream_t)stream, grad_points, grid, maps, S, B, K, n, H, W, RB);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
