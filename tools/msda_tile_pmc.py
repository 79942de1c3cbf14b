"""Encoder-mode MSDA backward sub-kernels at the C2 shapes (const offsets), few
iterations: a short program for rocprofv3 --pmc / --kernel-trace passes.
    python tools/msda_tile_pmc.py [R0] [skip] [encoder 0/1]
(VS_MSDA_BWD=tiled|carry|sorted selects the general-path variant when encoder=0)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "vision-instance-seg_amd"))
import torch  # noqa: E402

from visionseg import ops  # noqa: E402


def main():
    r0 = sys.argv[1] if len(sys.argv) > 1 else "5"
    skip = sys.argv[2] if len(sys.argv) > 2 else "6"
    enc = (sys.argv[3] if len(sys.argv) > 3 else "1") == "1"
    os.environ["VS_MSDA_NEAR_R"], os.environ["VS_MSDA_SKIP"] = r0, skip
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
    off = (torch.randn(1, 1, H, L, P, 2, device=dev, generator=g) * 2).expand(B, S, H, L, P, 2)
    loc = (ref[None, :, None, None, None, :] + off / norm[None, None, None, :, None, :]).contiguous()
    locr, wr = loc.clone().requires_grad_(True), w.clone().requires_grad_(True)
    for _ in range(4):
        o = ops.ms_deform_attn(v, shapes, locr, wr, encoder=enc)
        o.backward(go)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
