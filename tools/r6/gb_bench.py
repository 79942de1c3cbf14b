"""Activation-backward dX GEMMs (token_gemm gelu_pre / relu_out) at the C2 shapes vs the plain dX
GEMM + the activation backward kernel, HIP events (median of 20)."""
import os
import sys

ROOT = os.environ.get("VS_ROOT") or os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-instance-seg_amd")]
import torch  # noqa: E402
from visionseg import ops, _lib as L  # noqa: E402


def bench(fn, iters=20):
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
    return ts[len(ts) // 2] * 1e3


def main():
    dev = "cuda"
    for name, M, N, K, act in (("s1 fc2 dX", 262144, 384, 96, "gelu"), ("s2 fc2 dX", 65536, 768, 192, "gelu"),
                               ("s3 fc2 dX", 16384, 1536, 384, "gelu"), ("s4 fc2 dX", 4096, 3072, 768, "gelu"),
                               ("enc fc2 dX", 86016, 1024, 256, "relu")):
        gy = torch.randn(M, K, device=dev).to(torch.bfloat16)
        wt = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        pre = torch.randn(M, N, device=dev).to(torch.bfloat16)
        if act == "relu":
            pre = pre.clamp_min(0)
        kw = {"gelu_pre": pre} if act == "gelu" else {"relu_out": pre}
        dh = ops.token_gemm(gy, wt)
        out = torch.empty_like(dh)
        cs = torch.empty(N, device=dev, dtype=torch.bfloat16)
        ws = torch.empty(int(L.lib().vs_column_sum_workspace_bytes(M, N)), device=dev, dtype=torch.uint8)

        def act_bwd():
            L.check(L.lib().vs_act_backward_colsum(L.VS_BF16, 1 if act == "gelu" else 0, L.ptr(dh), L.ptr(pre),
                                                   L.ptr(out), L.ptr(cs), L.ptr(ws), M, N, L.stream(dh)), "act")
        tf = bench(lambda: ops.token_gemm(gy, wt, **kw))
        tp = bench(lambda: ops.token_gemm(gy, wt))
        ta = bench(act_bwd)
        mb = (M * K + N * K + 2 * M * N) * 2 / 1e6
        print(f"{name:10s} M={M:6d} N={N:5d} K={K:4d} {act}: fused {tf:7.1f} us ({mb / tf:5.2f} TB/s)  "
              f"plain dX {tp:7.1f} + act bwd {ta:7.1f} = {tp + ta:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
