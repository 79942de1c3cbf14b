"""LayerNorm backward A/B at the Swin stage shapes of C2 / C5 (bf16, residual-add and
column-sum variant as the Swin blocks call it): VS_LN_BWD_PARTS workgroup caps."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-instance-seg_amd")]
import torch  # noqa: E402

from visionseg import ops  # noqa: E402

DEV = "cuda"


def main():
    bf = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(0)
    for M, C in ((4 * 65536, 96), (4 * 16384, 192), (4 * 147456, 192), (4 * 36864, 384)):
        x = torch.randn(M, C, device=DEV, generator=g).to(bf).requires_grad_(True)
        r = torch.randn(M, C, device=DEV, generator=g).to(bf).requires_grad_(True)
        w = (1 + 0.1 * torch.randn(C, device=DEV, generator=g)).to(bf).requires_grad_(True)
        b = (0.1 * torch.randn(C, device=DEV, generator=g)).to(bf).requires_grad_(True)
        gy = torch.randn(M, C, device=DEV, generator=g).to(bf)
        gs = torch.randn(M, C, device=DEV, generator=g).to(bf)
        s, y = ops.add_layer_norm(x, r, w, b)
        for parts in [int(v) for v in os.environ.get("LNB_PARTS", "256,512,1024,2048").split(",")]:
            os.environ["VS_LN_BWD_PARTS"] = str(parts)
            for _ in range(3):
                torch.autograd.backward([y, s], [gy, gs], retain_graph=True)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            n = 20
            for _ in range(n):
                torch.autograd.backward([y, s], [gy, gs], retain_graph=True)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / n
            byt = M * C * 2 * 4          # dy, gs, x read + dx written (bf16)
            print(f"M {M} C {C} parts {parts}: add_layer_norm backward {ms:.4f} ms ({byt / ms / 1e6:.0f} GB/s incl. "
                  f"the colsum pass)", flush=True)
        with torch.no_grad():                # forward launches for the kernel trace (23 per shape)
            for _ in range(23):
                ops.add_layer_norm(x, r, w, b)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
