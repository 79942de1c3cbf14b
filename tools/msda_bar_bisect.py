"""Which of the MSDA backward's band-walk barriers may order LDS only (VS_MSDA_LDSBAR
bit mask, csrc/msda.hip bar()): per mask, the fused MFMA backward's grad_value /
grad_loc / grad_attn vs the mask-0 (__syncthreads everywhere) result on (a) a small
forced-split problem with many bands per tile and (b) the far-tap encoder case, and the
time per launch at the C2 encoder shape."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-instance-seg_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from visionseg import ops  # noqa: E402
from visionseg.profiling import KernelTimer  # noqa: E402
from oracle import ref_ops as R  # noqa: E402

DEV = "cuda"


def inputs(B, shapes, H, spread, seed):
    g = torch.Generator().manual_seed(seed)
    S = sum(h * w for h, w in shapes)
    L = len(shapes)
    ref = R.reference_points(shapes, B)
    off = (torch.rand(B, S, H, L, 4, 2, generator=g) * 2 - 1) * spread
    norm = torch.tensor([[w, h] for h, w in shapes], dtype=torch.float32)[None, None, None, :, None, :]
    loc = (ref[:, :, None, :, None, :] + off / norm).to(DEV)
    value = torch.randn(B, S, H, 32, generator=g).to(torch.bfloat16).to(DEV)
    w = torch.softmax(torch.randn(B, S, H, L * 4, generator=g), -1).view(B, S, H, L, 4).to(DEV)
    go = torch.randn(B, S, H * 32, generator=g).to(torch.bfloat16).to(DEV)
    return value, loc, w, go


def grads(case, mask):
    os.environ["VS_MSDA_LDSBAR"] = str(mask)
    value, loc, w, go, shapes = case
    v, l_, w_ = value.clone().requires_grad_(True), loc.clone().requires_grad_(True), w.clone().requires_grad_(True)
    ops.ms_deform_attn(v, shapes, l_, w_).backward(go)
    torch.cuda.synchronize()
    return v.grad.float(), l_.grad, w_.grad


def main():
    ops._MSDA_BWD = "carry"
    os.environ["VS_MSDA_RUN"] = "16"
    os.environ["VS_MSDA_MFMA"] = "1"
    os.environ["VS_MSDA_GEOM"] = "1"
    small = [(8, 8), (16, 16), (32, 32)]
    far = [(16, 16), (32, 32), (64, 64)]
    cases = {"small": (*inputs(2, small, 4, 3.0, 13), small), "far": (*inputs(1, far, 8, 12.0, 31), far)}
    c2 = [(32, 32), (64, 64), (128, 128)]
    big = (*inputs(4, c2, 8, 2.0, 5), c2)
    masks = [0, 1, 2, 4, 8, 16, 32, 64, 2 | 16, 1 | 2 | 4 | 8, 16 | 32 | 64, 127]
    base = {k: grads(c, 0) for k, c in cases.items()}
    for m in masks:
        errs = []
        for k, c in cases.items():
            for a, b in zip(grads(c, m), base[k]):
                errs.append(float((a - b).abs().max()) / max(float(b.abs().max()), 1e-30))
        os.environ["VS_MSDA_LDSBAR"] = str(m)
        value, loc, w, go, shapes = big
        v, l_, w_ = value.clone().requires_grad_(True), loc.clone().requires_grad_(True), w.clone().requires_grad_(True)
        for _ in range(3):
            ops.ms_deform_attn(v, shapes, l_, w_).backward(go)
        torch.cuda.synchronize()
        with KernelTimer() as t:
            for _ in range(10):
                ops.ms_deform_attn(v, shapes, l_, w_).backward(go)
        torch.cuda.synchronize()
        ms = t.summary()["msda_bwd"]["mean_ms"]
        print(f"mask {m:3d}: max rel diff vs mask 0 {max(errs):.2e} ({' '.join(f'{e:.1e}' for e in errs)}); "
              f"C2 encoder bwd {ms:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
