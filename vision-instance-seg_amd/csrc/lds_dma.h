// LDS-DMA staging and transposed-read helpers shared by the pixel-major weight-gradient
// kernels (conv3x3.hip, token_wgrad.hip) and the implicit-GEMM conv.
//
// Images are [row][128 x bf16] with 256-B rows and the 16-B chunks XOR-swizzled so that both
// the DMA's lane-linear 1-KB writes and the 32x32x16 transposed operand reads
// (ds_read_b64_tr_b16) are conflict-free (cdna_hip_programming.md T10, image (b)).  The DMA
// writes lane-linear, so the swizzle is applied to the GLOBAL source address of each lane.
#pragma once
#include "mfma_util.h"

namespace vs {
namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef short bf16x4v_t __attribute__((ext_vector_type(4)));

// the DMA source of padding taps, rows past the end and columns past the width: never written
__device__ __attribute__((aligned(256))) unsigned char g_dma_zero_row[256];

__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (lds_void*)lds_wave_base, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// barrier that keeps outstanding DMA in flight (no vmcnt drain): the caller waits for its
// own DMA with wait_vm first
__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ int img_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// byte offset of (row, 16-B chunk) in a [row][128 x bf16] image
__device__ __forceinline__ int woff(int row, int ch) { return 256 * row + 16 * (ch ^ img_swz(row)); }

// MFMA operand from an image: k = rows row0 + 8hh + 0..7, m/n = columns col0 + (lane & 31)
__device__ __forceinline__ bf16x8_t tr_frag(const unsigned char* img, int row0, int col0, int lane) {
  const int hh = lane >> 5;
  const int row = row0 + 8 * hh + ((lane & 15) >> 2);
  const int col = col0 + (lane & 16) + 4 * (lane & 3);
  typedef __attribute__((address_space(3))) bf16x4v_t lds_v4;
  const int within = (col & 7) * 2;
  const bf16x4v_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(img + woff(row, col >> 3) + within));
  const bf16x4v_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(img + woff(row + 4, col >> 3) + within));
  bf16x8_t v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return v;
}

// The same operand read from inline asm.  The compiler's waitcnt pass models the
// ds_read_tr intrinsic as possibly reading LDS that an in-flight LDS-DMA writes, so it drains
// vmcnt(0) in front of it -- the next chunk's prefetch is then waited for before the current
// chunk is multiplied (every chunk serialised behind its own DMA).  Hidden in asm, the read is
// ordered only by what the kernel states: the buffer it reads was retired by a counted
// wait_vm + barrier.  The pass does not track the asm's result either: lgkm_wait below must
// sit between the reads and the first use, carrying the fragments as operands so that no use
// (and no copy) is scheduled above it.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

__device__ __forceinline__ bf16x4v_t ds_tr16_asm(unsigned addr) {
  bf16x4v_t v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}

__device__ __forceinline__ bf16x8_t tr_frag_asm(const unsigned char* img, int row0, int col0, int lane) {
  const int hh = lane >> 5;
  const int row = row0 + 8 * hh + ((lane & 15) >> 2);
  const int col = col0 + (lane & 16) + 4 * (lane & 3);
  const int within = (col & 7) * 2;
  const unsigned a = lds_addr(img);
  const bf16x4v_t lo = ds_tr16_asm(a + woff(row, col >> 3) + within);
  const bf16x4v_t hi = ds_tr16_asm(a + woff(row + 4, col >> 3) + within);
  bf16x8_t v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return v;
}

// wait until at most N LDS operations of this wave are outstanding; v is carried through
template <int N>
__device__ __forceinline__ void lgkm_wait(bf16x8_t& v) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "n"(N) : "memory");
}

// ---- 64-B-row images ([token][32 x bf16], one attention head's rows): the 16-B chunk c of
// row t sits at chunk c ^ ((t >> 2) & 3), so a row-major read of one chunk column by 16
// lanes and a 4-row transposed read both cover all 64 banks.  Offsets in shorts.
__device__ __forceinline__ int swz64(int t, int c) { return 32 * t + 8 * (c ^ ((t >> 2) & 3)); }

// MFMA operand m = channel lane & 31, k = 8hh + j from rows t_lo + e (j = e < 4) and
// t_hi + e (j = 4 + e), e = (lane & 15) >> 2 chosen by the caller per lane half
__device__ __forceinline__ bf16x8_t tr64_rows(const short* img, int t_lo, int t_hi, int lane) {
  typedef __attribute__((address_space(3))) bf16x4v_t lds_v4;
  const int col = (lane & 16) + 4 * (lane & 3);
  const bf16x4v_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_v4*)(img + 32 * t_lo + 8 * ((col >> 3) ^ ((t_lo >> 2) & 3)) + (col & 7)));
  const bf16x4v_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_v4*)(img + 32 * t_hi + 8 * ((col >> 3) ^ ((t_hi >> 2) & 3)) + (col & 7)));
  bf16x8_t v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return v;
}

// permuted token order (k = 8hh + j <-> token base + (j&3) + 8(j>>2) + 4hh: a C tile's rows)
__device__ __forceinline__ bf16x8_t tr_perm64(const short* img, int base, int lane) {
  const int t0 = base + 4 * (lane >> 5) + ((lane & 15) >> 2);
  return tr64_rows(img, t0, t0 + 8, lane);
}

// natural token order (k = 8hh + j <-> token base + 8hh + j)
__device__ __forceinline__ bf16x8_t tr_nat64(const short* img, int base, int lane) {
  const int t0 = base + 8 * (lane >> 5) + ((lane & 15) >> 2);
  return tr64_rows(img, t0, t0 + 4, lane);
}

}  // namespace
}  // namespace vs
