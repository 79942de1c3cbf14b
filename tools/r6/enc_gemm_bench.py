"""Encoder input-projection GEMMs at the C2 shape (B = 4, 21504 tokens per image): token GEMM
vs F.linear (hipBLASLt) for value (256 -> 256) and offset / attention-weight proj (256 -> 288)
forwards, and the dX GEMMs of their backward.  HIP graph of 10 calls, median of 20."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-instance-seg_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from visionseg import ops  # noqa: E402


def timeit(fn, n=20):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(10):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 10)
    return sorted(ts)[n // 2] * 1e3


def main():
    dev, bf = "cuda", torch.bfloat16
    M = 4 * 21504
    h = torch.randn(M, 256, device=dev).to(bf)
    pos = torch.randn(M, 256, device=dev).to(bf)
    for name, N, K in (("value fwd", 256, 256), ("proj fwd", 288, 256), ("fc1 fwd", 1024, 256),
                       ("fc2 fwd", 256, 1024)):
        x = torch.randn(M, K, device=dev).to(bf)
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(bf)
        b = torch.randn(N, device=dev).to(bf)
        tv = timeit(lambda: F.linear(x, w, b))
        tt = timeit(lambda: ops.token_gemm(x, w, b))
        e = float((ops.token_gemm(x, w, b).float() - F.linear(x, w, b).float()).abs().max())
        by = M * (N + K) * 2
        print(f"{name:10s} M={M} N={N:5d} K={K:5d}: vendor {tv:6.1f} us  token_gemm {tt:6.1f} us "
              f"({by / tt / 1e3:5.0f} GB/s)  max|diff| {e:.3g}", flush=True)
    # fc1 + bias + ReLU: hipBLASLt RELU_BIAS epilogue vs the token GEMM's (VS_TGEMM_RELU)
    x = torch.randn(M, 256, device=dev).to(bf)
    w = (torch.randn(1024, 256, device=dev) * 256 ** -0.5).to(bf)
    b = torch.randn(1024, device=dev).to(bf)
    tv = timeit(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=False))
    tt = timeit(lambda: ops.token_gemm(x, w, b, relu=True))
    print(f"fc1+relu   M={M} N= 1024 K=  256: vendor {tv:6.1f} us  token_gemm(relu) {tt:6.1f} us", flush=True)
    # dX: dh = gp Wp + gv Wv (K = 288 / 256 -> 256)
    for name, Nred in (("proj dX", 288), ("value dX", 256), ("fc2 dX", 1024)):
        g = torch.randn(M, Nred, device=dev).to(bf)
        w = (torch.randn(Nred, 256, device=dev) * Nred ** -0.5).to(bf)   # [N_red, 256]
        wt = w.t().contiguous()
        tv = timeit(lambda: g @ w)
        tt = timeit(lambda: ops.token_gemm(g, wt))
        print(f"{name:10s} M={M} Nred={Nred}: vendor {tv:6.1f} us  token_gemm(W^T) {tt:6.1f} us", flush=True)
    ta = timeit(lambda: h + pos)
    print(f"h + pos add: {ta:6.1f} us")


if __name__ == "__main__":
    main()
