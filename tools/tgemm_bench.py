"""Token GEMM microbenchmark (csrc/token_gemm.hip) at the Swin block shapes of C2
(Swin-T, 4 x 1024^2) and C5 (Swin-L, 4 x 1536^2): the vendor GEMM (F.linear: hipBLASLt
with the shipped TunableOp table), the hand-written bf16 kernel, the MX-fp8 kernel (the
activation quantisation timed separately; weights are quantised once per step), and fc1
with GELU: F.linear + F.gelu vs the fused epilogue.  HIP-event timing, median of --iters.

    python tools/tgemm_bench.py [--configs C2,C5] [--iters 20]
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.environ.get("VS_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-instance-seg_amd")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from visionseg import ops  # noqa: E402
from visionseg.linear import load_gemm_table  # noqa: E402

CONFIGS = {"C2": (96, 1024, (2, 2, 6, 2)), "C5": (192, 1536, (2, 2, 18, 2))}


def bench(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2,C5")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    load_gemm_table()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    for cname in a.configs.split(","):
        C0, img, depths = CONFIGS[cname]
        tot = {}
        for st in range(4):
            C = C0 * 2 ** st
            M = 4 * (img // 4 // 2 ** st) ** 2
            x = torch.randn(M, 4 * C, device=dev, generator=g).to(torch.bfloat16)
            for name, (N, K) in {"qkv": (3 * C, C), "proj": (C, C), "fc1": (4 * C, C), "fc2": (C, 4 * C)}.items():
                xi = x[:, :K].contiguous()
                w = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).to(torch.bfloat16)
                b = torch.randn(N, device=dev, generator=g).to(torch.bfloat16)
                fl = 2.0 * M * N * K
                r = {"vendor": bench(lambda: F.linear(xi, w, b), a.iters),
                     "tgemm_bf16": bench(lambda: ops.token_gemm(xi, w, b), a.iters)}
                if K % 128 == 0:
                    xq, xs = ops.mx_quantize(xi)
                    wq, ws = ops.mx_quantize(w)
                    r["tgemm_fp8"] = bench(lambda: ops.token_gemm(xq, wq, b, x_scales=xs, w_scales=ws), a.iters)
                    r["quant_x"] = bench(lambda: ops.mx_quantize(xi), a.iters)
                if name == "fc1":
                    r["vendor+gelu"] = bench(lambda: F.gelu(F.linear(xi, w, b)), a.iters)
                    r["tgemm_gelu"] = bench(lambda: ops.token_gemm(xi, w, b, gelu=True), a.iters)
                    if K % 128 == 0:
                        r["tgemm_fp8_gelu"] = bench(lambda: ops.token_gemm(xq, wq, b, gelu=True, x_scales=xs,
                                                                           w_scales=ws), a.iters)
                line = "  ".join(f"{k} {v:7.4f} ms ({fl / v / 1e9:6.1f} TF/s)" for k, v in r.items())
                print(f"{cname} stage{st + 1} {name:4s} M={M:6d} N={N:5d} K={K:5d}: {line}", flush=True)
                for k, v in r.items():
                    tot[k] = tot.get(k, 0.0) + v * depths[st] * (1 if k != "quant_x" else 1)
        print(f"{cname} forward Linears per step (x blocks): " +
              "  ".join(f"{k} {v:.3f} ms" for k, v in sorted(tot.items())), flush=True)


if __name__ == "__main__":
    main()
