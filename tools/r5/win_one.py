"""One window-attention shape (default: C5 stage 1, Swin-L 1536^2, 4 images) forward +
backward, HIP-event timed -- a short driver for rocprofv3 counter passes and A/B runs.
    python tools/r5/win_one.py [--bw 4096 --heads 6 --ws 12 --iters 5 --fp8 0]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vision-instance-seg_amd"))

import torch  # noqa: E402

from visionseg import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--bw", type=int, default=4096)
ap.add_argument("--heads", type=int, default=6)
ap.add_argument("--ws", type=int, default=12)
ap.add_argument("--nw", type=int, default=32)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--fp8", type=int, default=0)
a = ap.parse_args()
g = torch.Generator(device="cuda").manual_seed(0)
N, C = a.ws * a.ws, a.heads * 32
qkv = torch.randn(a.bw, N, 3 * C, device="cuda", generator=g).to(torch.bfloat16).requires_grad_(True)
tab = torch.randn((2 * a.ws - 1) ** 2, a.heads, device="cuda", generator=g).requires_grad_(True)
go = torch.randn(a.bw, N, C, device="cuda", generator=g).to(torch.bfloat16)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for it in range(a.iters + 2):
    if it == 2:
        ev[0].record()
    o = ops.window_attention(qkv, tab, a.heads, a.ws, a.ws // 2, a.nw, a.nw, fp8=bool(a.fp8))
    o.backward(go)
ev[1].record()
torch.cuda.synchronize()
print(f"bw={a.bw} heads={a.heads} ws={a.ws} fp8={a.fp8} fwd+bwd {ev[0].elapsed_time(ev[1]) / a.iters:.4f} ms/iter")
