"""Probe: the vendor fp8 GEMM paths of torch._scaled_mm on gfx950 (hipBLASLt) at the C5
Swin-L token-Linear shapes, against bf16 F.linear and the hand-written MX token GEMM.

For each scaling recipe (tensorwise f32, rowwise f32, MX e8m0 per 1x32 block) it checks
the numerics against the dequantised product computed in f32 and times the GEMM (HIP events,
median of 20).  MX scale layout: hipBLASLt's VEC32_UE8M0 wants [rows, K/32] row-major; the
probe tries that (and reports a mismatch if the layout is swizzled instead)."""
import sys
import time

import torch
import torch.nn.functional as F

DEV = "cuda"
SHAPES = [  # (name, M tokens, N out, K in) -- C5 Swin-L @1536^2, batch 4
    ("s1 qkv", 589824, 576, 192), ("s1 fc1", 589824, 768, 192), ("s1 fc2", 589824, 192, 768),
    ("s2 qkv", 147456, 1152, 384), ("s2 fc1", 147456, 1536, 384), ("s2 fc2", 147456, 384, 1536),
    ("s3 qkv", 36864, 2304, 768), ("s3 fc1", 36864, 3072, 768), ("s3 fc2", 36864, 768, 3072),
    ("s4 fc1", 9216, 6144, 1536), ("s4 fc2", 9216, 1536, 6144),
    ("s2 proj", 147456, 384, 384), ("s3 proj", 36864, 768, 768), ("s4 qkv", 9216, 4608, 1536),
    ("s4 proj", 9216, 1536, 1536),
]
E4 = torch.float8_e4m3fn


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    ev = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ev.append((a, b))
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in ev)[n // 2]


def mx_quant(x):
    """x [R, K] f32 -> (e4m3 [R, K], e8m0 scales [R, K/32]) with scale = 2^(floor(log2 amax) - 8)."""
    R, K = x.shape
    xb = x.view(R, K // 32, 32)
    amax = xb.abs().amax(-1).clamp(min=2.0 ** -100)
    e = torch.floor(torch.log2(amax)) - 8
    s = torch.exp2(e)
    q = (xb / s[..., None]).clamp(-448, 448).to(E4).view(R, K)
    kb = K // 32
    Rp, kbp = -(-R // 128) * 128, -(-kb // 4) * 4          # the padded scale shape torch checks
    sb = torch.full((Rp, kbp), 127, dtype=torch.uint8, device=x.device)
    sb[:R, :kb] = (e + 127).to(torch.uint8)
    return q, sb.view(torch.float8_e8m0fnu), s


def main():
    torch.manual_seed(0)
    print(torch.__version__, torch.version.hip, torch.cuda.get_device_name(0), flush=True)
    for name, M, N, K in SHAPES:
        x = torch.randn(M, K, device=DEV)
        w = torch.randn(N, K, device=DEV) / K ** 0.5
        xb, wb = x.bfloat16(), w.bfloat16()
        t_bf16 = timeit(lambda: F.linear(xb, wb))
        fl = 2.0 * M * N * K
        line = f"{name:7s} M={M:6d} N={N:5d} K={K:5d}: bf16 {t_bf16:.4f} ms ({fl / t_bf16 / 1e9:6.1f} TF/s)"
        # tensorwise
        try:
            sx = (x.abs().max() / 448).float()
            sw = (w.abs().max() / 448).float()
            xq, wq = (x / sx).to(E4), (w / sw).to(E4)
            out = torch._scaled_mm(xq, wq.t(), scale_a=sx.view(1), scale_b=sw.view(1), out_dtype=torch.bfloat16)
            ref = (xq.float() * sx) @ (wq.float() * sw).t()
            err = float((out.float() - ref).norm() / ref.norm())
            t = timeit(lambda: torch._scaled_mm(xq, wq.t(), scale_a=sx.view(1), scale_b=sw.view(1),
                                                out_dtype=torch.bfloat16))
            line += f" | tensor {t:.4f} ({fl / t / 1e9:6.1f}) err {err:.1e}"
        except Exception as e:  # noqa: BLE001
            line += f" | tensor FAIL {type(e).__name__}: {str(e)[:80]}"
        # rowwise
        try:
            sxr = (x.abs().amax(1, keepdim=True) / 448).float()
            swr = (w.abs().amax(1, keepdim=True) / 448).float()
            xq, wq = (x / sxr).to(E4), (w / swr).to(E4)
            out = torch._scaled_mm(xq, wq.t(), scale_a=sxr, scale_b=swr.t(), out_dtype=torch.bfloat16)
            ref = (xq.float() * sxr) @ (wq.float() * swr).t()
            err = float((out.float() - ref).norm() / ref.norm())
            t = timeit(lambda: torch._scaled_mm(xq, wq.t(), scale_a=sxr, scale_b=swr.t(), out_dtype=torch.bfloat16))
            line += f" | row {t:.4f} ({fl / t / 1e9:6.1f}) err {err:.1e}"
            bias = torch.randn(N, device=DEV).bfloat16()
            outb = torch._scaled_mm(xq, wq.t(), scale_a=sxr, scale_b=swr.t(), bias=bias, out_dtype=torch.bfloat16)
            errb = float((outb.float() - out.float() - bias.float()).abs().max())
            tb = timeit(lambda: torch._scaled_mm(xq, wq.t(), scale_a=sxr, scale_b=swr.t(), bias=bias,
                                                 out_dtype=torch.bfloat16))
            line += f" +bias {tb:.4f} (d {errb:.1e})"
        except Exception as e:  # noqa: BLE001
            line += f" | row FAIL {type(e).__name__}: {str(e)[:80]}"
        if "--mx" not in sys.argv:
            print(line, flush=True)
            continue
        # MX 1x32 e8m0
        try:
            xq, xs, xsf = mx_quant(x)
            wq, ws, wsf = mx_quant(w)
            out = torch._scaled_mm(xq, wq.t(), scale_a=xs.contiguous(), scale_b=ws.contiguous(),
                                   out_dtype=torch.bfloat16)
            ref = (xq.float().view(M, K // 32, 32) * xsf[..., None]).view(M, K) @ \
                (wq.float().view(N, K // 32, 32) * wsf[..., None]).view(N, K).t()
            err = float((out.float() - ref).norm() / ref.norm())
            t = timeit(lambda: torch._scaled_mm(xq, wq.t(), scale_a=xs, scale_b=ws, out_dtype=torch.bfloat16))
            line += f" | mx {t:.4f} ({fl / t / 1e9:6.1f}) err {err:.1e}"
        except Exception as e:  # noqa: BLE001
            line += f" | mx FAIL {type(e).__name__}: {str(e)[:100]}"
        print(line, flush=True)
        del x, w, xb, wb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    sys.exit(main())
