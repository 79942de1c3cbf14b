"""LayerNorm forward (residual-add form) and backward (ADD + CS form) at the C2 shapes,
through the C ABI, timed with HIP events; 3 rotating input sets so a launch does not find its
operands in the Infinity Cache from the previous one.  GB/s = algorithmic bytes / time."""
import os
import sys

sys.path.insert(0, os.path.join(os.environ.get("VS_ROOT") or os.path.join(os.path.dirname(__file__), "..", ".."),
                                "vision-instance-seg_amd"))
import torch
from visionseg import _lib as L

SHAPES = [(262144, 96), (65536, 192), (16384, 384), (4096, 768), (86016, 256), (400, 256)]


def bench(fn, n=30):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(n):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3        # us


def main():
    lib = L.lib()
    dev = "cuda"
    st = L.stream(torch.empty(1, device=dev))
    for M, C in SHAPES:
        sets = []
        for k in range(3):
            g = torch.Generator(device=dev).manual_seed(k)
            t = lambda: torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16)
            sets.append(dict(x=t(), r=t(), s=torch.empty(M, C, device=dev, dtype=torch.bfloat16),
                             y=torch.empty(M, C, device=dev, dtype=torch.bfloat16), dy=t(), dres=t(),
                             dx=torch.empty(M, C, device=dev, dtype=torch.bfloat16),
                             mean=torch.empty(M, device=dev), rstd=torch.empty(M, device=dev)))
        w = torch.randn(C, device=dev).to(torch.bfloat16)
        b = torch.randn(C, device=dev).to(torch.bfloat16)
        dw, db, cs = (torch.empty(C, device=dev, dtype=torch.bfloat16) for _ in range(3))
        ws = torch.empty(int(lib.vs_layer_norm_backward_workspace_bytes(M, C)), device=dev, dtype=torch.uint8)

        def fwd(i):
            d = sets[i % 3]
            L.check(lib.vs_add_layer_norm_forward(L.VS_BF16,
                                                  L.ptr(d["x"]), L.ptr(d["r"]), L.ptr(w), L.ptr(b), L.ptr(d["s"]),
                                                  L.ptr(d["y"]), L.ptr(d["mean"]), L.ptr(d["rstd"]), M, C, 1e-5, st),
                    "fwd")

        def bwd(i):
            d = sets[i % 3]
            L.check(lib.vs_layer_norm_backward_ex(L.dtype_code(d["x"]), L.ptr(d["dy"]), L.ptr(d["s"]), L.ptr(w),
                                                  L.ptr(d["mean"]), L.ptr(d["rstd"]), L.ptr(d["dres"]), L.ptr(d["dx"]),
                                                  L.ptr(dw), L.ptr(db), L.ptr(cs), L.ptr(ws), M, C, st), "bwd")

        tf = bench(fwd)
        tb = bench(bwd)
        nb = M * C * 2
        print(f"M={M:6d} C={C:4d}  fwd {tf:7.2f} us {4 * nb / tf / 1e3:6.0f} GB/s   bwd(+add,cs) {tb:7.2f} us "
              f"{4 * nb / tb / 1e3:6.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
