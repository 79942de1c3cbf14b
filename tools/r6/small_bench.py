"""Decoder small Linears (csrc/small_linear.hip) at the C2 decoder shapes (B x Q = 400
tokens), forward and backward through the C ABI, HIP events over 50 launches."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "vision-instance-seg_amd"))
import torch
from visionseg import _lib as L


def bench(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    lib = L.lib()
    dev = "cuda"
    st = L.stream(torch.empty(1, device=dev))
    T = 400
    for O, I, relu in ((256, 256, 0), (2048, 256, 1), (256, 2048, 0)):
        x = torch.randn(T, I, device=dev).to(torch.bfloat16)
        w = (torch.randn(O, I, device=dev) * 0.05).to(torch.bfloat16)
        b = torch.randn(O, device=dev).to(torch.bfloat16)
        y = torch.empty(T, O, device=dev, dtype=torch.bfloat16)
        gy = torch.randn(T, O, device=dev).to(torch.bfloat16)
        gx = torch.empty(T, I, device=dev, dtype=torch.bfloat16)
        gw = torch.empty(O, I, device=dev, dtype=torch.bfloat16)
        gb = torch.empty(O, device=dev, dtype=torch.bfloat16)

        def fwd():
            L.check(lib.vs_small_linear_forward(L.VS_BF16, L.ptr(x), None, 0, L.ptr(w), L.ptr(b), relu, L.ptr(y), T, O, I,
                                                st), "fwd")

        def bwd():
            L.check(lib.vs_small_linear_backward(L.VS_BF16, L.ptr(gy), L.ptr(x), None, 0, L.ptr(w),
                                                 L.ptr(y) if relu else None, None, L.ptr(gx), None, 0, L.ptr(gw),
                                                 L.ptr(gb), T, O, I, st), "bwd")

        fwd()
        tf, tb = bench(fwd), bench(bwd)
        fl = 2.0 * T * O * I
        print(f"T={T} out={O:5d} in={I:5d} relu={relu}: fwd {tf:6.2f} us ({fl / tf / 1e6:6.1f} TF/s)  "
              f"bwd {tb:6.2f} us ({2 * fl / tb / 1e6:6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
