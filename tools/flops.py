"""Forward matmul/conv FLOPs per image of the PRODUCT models, counted with
torch.utils.flop_counter.FlopCounterMode on the GPU (the product ops need HIP).

    python tools/flops.py [--arch mask2former|maskdino] [--model swin_t] [--size 1024] [--queries 100]

BASELINE.md §2's per-image figures were counted on the HF oracle (matmul / conv / bmm /
SDPA; grid_sample, i.e. the deformable sampling, counts 0).  The product runs its
attention cores as torch.ops.visionseg.* custom ops, which FlopCounterMode prices at 0
unless told otherwise; the formulas registered here give them the FLOPs of the matmuls
they replace (window attention QK^T + PV per head and window, masked cross-attention
QK^T + PV over every key, the mask-head einsum), so the product's Mask2Former count
reproduces the HF figure and the same method prices MaskDINO (C4: its training forward,
denoising queries included), for which no HF model exists.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-instance-seg_amd")]
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

import torch  # noqa: E402
from torch.utils.flop_counter import FlopCounterMode, register_flop_formula  # noqa: E402


def _register():
    from visionseg import _lib as L
    ops = L.tops()

    @register_flop_formula(ops.win_attn_fwd)
    def _win(qkv_shape, table_shape, heads, *args, out_shape=None, **kw):
        Bw, N = qkv_shape[0], qkv_shape[1]
        return 4 * Bw * heads * N * N * 32

    @register_flop_formula(ops.masked_xattn_fwd)
    def _xattn(q_shape, k_shape, v_shape, words_shape, heads, *args, out_shape=None, **kw):
        B, Q, S = q_shape[0], q_shape[1], k_shape[1]
        return 4 * B * heads * Q * S * 32

    @register_flop_formula(ops.mask_head_fwd)
    def _mask(e_shape, p_shape, height, width, *args, out_shape=None, **kw):
        B, Q, C = e_shape
        return 2 * B * Q * C * height * width


def count(arch, model, size, queries, batch=1):
    from visionseg.data import synthetic_batch
    dev = torch.device("cuda", 0)
    imgs, ml, cl = synthetic_batch(batch, size, seed=42, device=dev)
    if arch == "maskdino":
        from visionseg.criterion import PaddedTargets
        from visionseg.maskdino import MaskDINO, MaskDINOConfig, masks_to_boxes
        cfg = MaskDINOConfig.preset(model, num_queries=queries)
        m = MaskDINO(cfg).init_weights(0).to(dev).to(torch.bfloat16).train()
        tg = PaddedTargets.from_lists(ml, cl, device=dev)
        args = (imgs, tg, masks_to_boxes(tg.masks))
    else:
        from visionseg.model import M2FConfig, Mask2Former
        cfg = M2FConfig.preset(model, num_queries=queries)
        m = Mask2Former(cfg).init_weights(0).to(dev).to(torch.bfloat16).train()
        args = (imgs,)
    for p in m.parameters():          # no autograd state: FlopCounterMode's module tracker
        p.requires_grad_(False)       # hooks every grad-requiring input otherwise
    with torch.no_grad(), FlopCounterMode(display=False) as fc:
        m(*args)
    per_op = {str(k): v for k, v in fc.get_flop_counts().get("Global", {}).items()}
    return fc.get_total_flops() / batch, per_op


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="mask2former")
    ap.add_argument("--model", default="swin_t")
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--queries", type=int, default=0)
    a = ap.parse_args()
    _register()
    q = a.queries or (300 if a.arch == "maskdino" else 100)
    tot, per_op = count(a.arch, a.model, a.size, q)
    print(json.dumps({"arch": a.arch, "model": a.model, "size": a.size, "queries": q,
                      "forward_gflop_per_image": round(tot / 1e9, 1),
                      "per_op_gflop": {k: round(v / 1e9, 2) for k, v in sorted(per_op.items())}}))


if __name__ == "__main__":
    main()
