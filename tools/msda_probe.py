"""Per-sub-kernel timing of the encoder-mode MSDA backward (tile / scatter / geom) on
smooth and iid offsets at several R0, via VS_MSDA_SKIP (C2 shapes, bf16)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "vision-instance-seg_amd"))
import torch

from visionseg import ops


def main():
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    B, H, L, P = 4, 8, 3, 4
    shapes = [(32, 32), (64, 64), (128, 128)]
    S = sum(h * w for h, w in shapes)
    ys = [torch.linspace(0.5, h - 0.5, h, device=dev) / h for h, w in shapes]
    xs = [torch.linspace(0.5, w - 0.5, w, device=dev) / w for h, w in shapes]
    ref = torch.cat([torch.stack(torch.meshgrid(x, y, indexing="xy"), -1).reshape(-1, 2) for x, y in zip(xs, ys)])
    norm = torch.tensor([[w, h] for h, w in shapes], device=dev, dtype=torch.float32)
    w = torch.softmax(torch.randn(B, S, H, L * P, device=dev, generator=g), -1).view(B, S, H, L, P)
    v = torch.randn(B, S, H, 32, device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
    go = torch.randn(B, S, H * 32, device=dev, generator=g).to(torch.bfloat16)
    offs = {"const": (torch.randn(1, 1, H, L, P, 2, device=dev, generator=g) * 2).expand(B, S, H, L, P, 2),
            "smooth": (torch.randn(1, 1, H, L, P, 2, device=dev, generator=g) * 2
                       + 0.3 * torch.randn(B, S, H, L, P, 2, device=dev, generator=g))}
    for oname, off in offs.items():
        loc = (ref[None, :, None, None, None, :] + off / norm[None, None, None, :, None, :]).contiguous()
        locr, wr = loc.clone().requires_grad_(True), w.clone().requires_grad_(True)
        for r0 in ("0", "3", "5"):
            for skip, what in (("6", "tile"), ("5", "scatter"), ("3", "geom"), ("0", "all")):
                os.environ["VS_MSDA_NEAR_R"], os.environ["VS_MSDA_SKIP"] = r0, skip

                def fb():
                    o = ops.ms_deform_attn(v, shapes, locr, wr, encoder=True)
                    o.backward(go)
                for _ in range(3):
                    fb()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                # the forward runs too: time it alone and subtract
                e0.record()
                for _ in range(10):
                    fb()
                e1.record()
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) / 10
                print(f"{oname:7s} R0={r0} {what:8s} fwd+bwd {t:7.3f} ms", flush=True)
    os.environ.pop("VS_MSDA_SKIP")


if __name__ == "__main__":
    main()
