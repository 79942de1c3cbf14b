// Swin pad + cyclic shift + window partition, and the exact inverse
// (window reverse + roll back + crop).  HF:swin:486-505 (partition/reverse),
// HF:swin:609-626 (pad, roll), order HF:swin:546-566.
//
// Pure data movement: one lane moves one `Unit` (16/8/4/2 bytes) of the channel row,
// so a pixel's channel row is copied by consecutive lanes with the widest aligned
// access the element size and channel count allow.  Padded source pixels read as
// zero.  HBM-bound: 2 x activation bytes per pass.
#include "common.h"

namespace vs {
namespace {

template <typename Unit>
__global__ void __launch_bounds__(256) partition_kernel(const Unit* __restrict__ x, Unit* __restrict__ win,
                                                        int H, int W, int Cu, int ws, int shift,
                                                        int Hp, int Wp, long long total) {
  const int nWw = Wp / ws, nWh = Hp / ws;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (; i < total; i += stride) {
    long long t = i;
    const int cu = (int)(t % Cu); t /= Cu;
    const int tx = (int)(t % ws); t /= ws;
    const int ty = (int)(t % ws); t /= ws;
    const int wx = (int)(t % nWw); t /= nWw;
    const int wy = (int)(t % nWh);
    const long long b = t / nWh;
    int sy = wy * ws + ty + shift; if (sy >= Hp) sy -= Hp;
    int sx = wx * ws + tx + shift; if (sx >= Wp) sx -= Wp;
    Unit v;
    if (sy < H && sx < W) {
      v = x[((b * H + sy) * W + sx) * Cu + cu];
    } else {
      v = Unit{};
    }
    win[i] = v;
  }
}

template <typename Unit>
__global__ void __launch_bounds__(256) reverse_kernel(const Unit* __restrict__ win, Unit* __restrict__ x,
                                                      int H, int W, int Cu, int ws, int shift,
                                                      int Hp, int Wp, long long total) {
  const int nWw = Wp / ws, nWh = Hp / ws;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (; i < total; i += stride) {
    long long t = i;
    const int cu = (int)(t % Cu); t /= Cu;
    const int xx = (int)(t % W); t /= W;
    const int yy = (int)(t % H);
    const long long b = t / H;
    int py = yy - shift; if (py < 0) py += Hp;   // padded-grid position of this pixel
    int px = xx - shift; if (px < 0) px += Wp;
    const int wy = py / ws, ty = py - wy * ws;
    const int wx = px / ws, tx = px - wx * ws;
    const long long src = ((((b * nWh + wy) * nWw + wx) * ws + ty) * ws + tx) * Cu + cu;
    x[i] = win[src];
  }
}

struct alignas(16) U16 { uint32_t a, b, c, d; };
struct alignas(8) U8 { uint32_t a, b; };

template <typename T> struct PK { static constexpr auto f = partition_kernel<T>; };
template <typename T> struct RK { static constexpr auto f = reverse_kernel<T>; };

template <template <typename> class K>
int launch(const void* src, void* dst, int esize, int B, int H, int W, int C, int ws, int shift,
            bool partition, hipStream_t st) {
  const int Hp = H + (ws - H % ws) % ws, Wp = W + (ws - W % ws) % ws;
  const long long rowbytes = (long long)C * esize;
  const long long pixels = partition ? (long long)B * Hp * Wp : (long long)B * H * W;
  const uintptr_t al = (uintptr_t)src | (uintptr_t)dst;
  int unit = 1;
  for (int u : {16, 8, 4, 2}) {
    if (rowbytes % u == 0 && al % u == 0) { unit = u; break; }
  }
  const int Cu = (int)(rowbytes / unit);
  const long long total = pixels * Cu;
  if (total == 0) return VS_OK;
  const int block = 256;
  const int grid = grid_for(total, block, 256 * 32);
#define VS_WIN_LAUNCH(T)                                                                        \
  hipLaunchKernelGGL(K<T>::f, dim3(grid), dim3(block), 0, st, (const T*)src, (T*)dst, H, W, Cu, \
                     ws, shift, Hp, Wp, total)
  switch (unit) {
    case 16: VS_WIN_LAUNCH(U16); break;
    case 8: VS_WIN_LAUNCH(U8); break;
    case 4: VS_WIN_LAUNCH(uint32_t); break;
    case 2: VS_WIN_LAUNCH(uint16_t); break;
    default: VS_WIN_LAUNCH(uint8_t); break;
  }
#undef VS_WIN_LAUNCH
  VS_LAUNCH_CHECK();
  return VS_OK;
}
}  // namespace
}  // namespace vs

using namespace vs;

extern "C" int vs_window_partition(const void* x, void* windows, int esize, int B, int H, int W,
                                   int C, int ws, int shift, void* stream) {
  VS_CHECK(x && windows, "null pointer");
  VS_CHECK(esize >= 1 && esize <= 8 && B > 0 && H > 0 && W > 0 && C > 0 && ws > 0, "bad sizes");
  VS_CHECK(shift >= 0 && shift < ws, "shift must be in [0, window)");
  return launch<PK>(x, windows, esize, B, H, W, C, ws, shift, true, (hipStream_t)stream);
}

extern "C" int vs_window_reverse(const void* windows, void* x, int esize, int B, int H, int W,
                                 int C, int ws, int shift, void* stream) {
  VS_CHECK(x && windows, "null pointer");
  VS_CHECK(esize >= 1 && esize <= 8 && B > 0 && H > 0 && W > 0 && C > 0 && ws > 0, "bad sizes");
  VS_CHECK(shift >= 0 && shift < ws, "shift must be in [0, window)");
  return launch<RK>(windows, x, esize, B, H, W, C, ws, shift, false, (hipStream_t)stream);
}
