"""Token-Linear weight gradient at the C2 shapes (Swin-T stages 1-4, the pixel-decoder
encoder): csrc/token_wgrad.hip (bias fused) vs the vendor batched GEMM + splitk_sum +
column_sum.  HIP events, median of 20; TF/s of the 2 T N K flops and GB/s of the operands."""
import sys

import torch

sys.path.insert(0, "vision-instance-seg_amd")
from visionseg import linear as lin, ops  # noqa: E402

DEV = "cuda"
QUICK = "--quick" in sys.argv
DGRAD_ONLY = "--dgrad-only" in sys.argv
SHAPES = [  # (name, tokens, N out, K in)
    ("s1 qkv", 262144, 288, 96), ("s1 proj", 262144, 96, 96), ("s1 fc1", 262144, 384, 96),
    ("s1 fc2", 262144, 96, 384), ("s2 qkv", 65536, 576, 192), ("s2 fc1", 65536, 768, 192),
    ("s2 fc2", 65536, 192, 768), ("s3 qkv", 16384, 1152, 384), ("s3 fc1", 16384, 1536, 384),
    ("s3 fc2", 16384, 384, 1536), ("s4 fc1", 4096, 3072, 768), ("s4 fc2", 4096, 768, 3072),
    ("enc val", 87040, 256, 256), ("enc off", 87040, 288, 256), ("enc fc1", 87040, 1024, 256),
    ("enc fc2", 87040, 256, 1024),
]


def timeit(fn, n=20):
    """Median GPU time of one call: 10 calls captured in a HIP graph and replayed (no host
    enqueue cost in the measurement)."""
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
    return sorted(ts)[n // 2]


def timeit_eager(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[n // 2]


def main():
    lin.load_gemm_table()
    tot_a = tot_b = 0.0
    for name, T, N, K in ([] if DGRAD_ONLY else SHAPES):
        gy = torch.randn(T, N, device=DEV).to(torch.bfloat16)
        x = torch.randn(T, K, device=DEV).to(torch.bfloat16)
        ta = timeit(lambda: ops.token_wgrad(gy, x, torch.bfloat16, bias=True))
        tb = ta if QUICK else timeit(lambda: (lin._vendor_weight_grad(gy, x, torch.bfloat16), ops.column_sum(gy)))
        d1, b1 = ops.token_wgrad(gy, x, torch.bfloat16, bias=True)
        d0 = lin._vendor_weight_grad(gy, x, torch.bfloat16)
        err = float((d1.float() - d0.float()).norm() / d0.float().norm())
        fl = 2.0 * T * N * K
        by = T * (N + K) * 2
        tot_a += ta
        tot_b += tb
        print(f"{name:8s} T={T:6d} N={N:5d} K={K:5d}: token_wgrad {ta * 1e3:7.1f} us ({fl / ta / 1e9:6.1f} TF/s, "
              f"{by / ta / 1e6:6.0f} GB/s)  vendor+colsum {tb * 1e3:7.1f} us ({fl / tb / 1e9:6.1f} TF/s)  rel {err:.1e}",
              flush=True)
        del gy, x
    print(f"total: token_wgrad {tot_a:.3f} ms, vendor {tot_b:.3f} ms", flush=True)
    if QUICK:
        return 0
    # input gradient dX = dY W ([T, N] x [N, K]): the token GEMM on W^T vs the vendor GEMM
    tot_a = tot_b = 0.0
    for name, T, N, K in SHAPES:
        gy = torch.randn(T, N, device=DEV).to(torch.bfloat16)
        w = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
        ta = timeit(lambda: ops.token_gemm(gy, w.t().contiguous()))
        tb = timeit(lambda: gy @ w)
        fl = 2.0 * T * N * K
        tot_a += ta
        tot_b += tb
        print(f"dgrad {name:8s}: token_gemm(+W^T) {ta * 1e3:7.1f} us ({fl / ta / 1e9:6.1f} TF/s)  vendor {tb * 1e3:7.1f} us "
              f"({fl / tb / 1e9:6.1f} TF/s)  rule {lin._use_token_gemm(T, K, N)}", flush=True)
        del gy, w
    print(f"dgrad total: token_gemm {tot_a:.3f} ms, vendor {tot_b:.3f} ms", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
