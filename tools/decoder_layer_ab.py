"""One masked-attention decoder layer (visionseg.model.DecoderLayer, B = 2, Q = 100, a
32 x 32 memory level) in bf16 with the small-token HIP kernels on and off, each against
the same layer in fp32 on the device: relative L2 error of the output and of every
gradient.  Separates a kernel defect (one setting far off) from rounding noise (both alike).
    python tools/decoder_layer_ab.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-instance-seg_amd")]
import torch  # noqa: E402

from visionseg import linear  # noqa: E402
from visionseg.model import DecoderLayer  # noqa: E402

DEV = "cuda"


def run(layer, dtype, h, table, mem, gy, fused):
    linear._SMALL_FUSED = linear._QKV_FUSED = fused
    lay = layer.to(dtype)
    for p in lay.parameters():
        p.grad = None
    hh = h.detach().to(dtype).clone().requires_grad_(True)
    tt = table.detach().to(dtype).clone().requires_grad_(True)
    mm = mem.detach().to(dtype).clone().requires_grad_(True)
    B, Q, D = hh.shape
    qpos = tt.unsqueeze(0).expand(B, -1, -1)
    words = torch.zeros(B, Q, (mm.shape[1] + 31) // 32, dtype=torch.int32, device=DEV)
    out = lay(hh, qpos, mm, mm * 1.0, words)
    out.backward(gy.to(dtype))
    res = {"out": out.detach().float(), "dh": hh.grad.float(), "dpos": tt.grad.float(), "dmem": mm.grad.float()}
    for n, p in lay.named_parameters():
        res[n] = p.grad.float()
    return res


def compare():
    """{tensor name: (fused rel-L2 error, library rel-L2 error)} against the fp32 layer."""
    torch.manual_seed(0)
    D = 256
    base = DecoderLayer(D, 2048, 8).to(DEV)
    with torch.no_grad():
        for n, p in base.named_parameters():
            p.copy_(torch.randn_like(p) * (0.02 if p.dim() == 1 else p.shape[-1] ** -0.5))
            if "norm" in n and n.endswith("weight"):
                p.fill_(1.0)
    B, Q = 2, 100
    h = torch.randn(B, Q, D, device=DEV).to(torch.bfloat16).float()
    table = torch.randn(Q, D, device=DEV).to(torch.bfloat16).float()
    mem = torch.randn(B, 1024, D, device=DEV).to(torch.bfloat16).float()
    gy = torch.randn(B, Q, D, device=DEV).to(torch.bfloat16).float()
    sd = {k: v.clone() for k, v in base.state_dict().items()}
    results = {}
    for name, dtype, fused in (("fp32", torch.float32, True), ("bf16 fused", torch.bfloat16, True),
                               ("bf16 unfused", torch.bfloat16, False)):
        lay = DecoderLayer(D, 2048, 8).to(DEV)
        lay.load_state_dict(sd)
        results[name] = run(lay, dtype, h, table, mem, gy, fused)
    ref = results["fp32"]
    return {k: tuple(float((results[name][k] - ref[k]).norm() / ref[k].norm().clamp_min(1e-12))
                     for name in ("bf16 fused", "bf16 unfused")) for k in ref}


def main():
    errs = compare()
    print(f"{'tensor':45s} {'fused':>10s} {'unfused':>10s}")
    for k, (a, b) in errs.items():
        print(f"{k:45s} {a:10.3e} {b:10.3e}")
    print("worst fused / unfused error ratio "
          f"{max(a / max(b, 1e-12) for k, (a, b) in errs.items() if k != 'self_attn.k_proj.bias'):.2f} "
          "(self_attn.k_proj.bias: analytically zero gradient, rounding noise on both paths)")


if __name__ == "__main__":
    main()
