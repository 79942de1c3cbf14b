"""CPU emulation of csrc/optim.hip vs_flat_step over a visionseg.optim.FlatOptimizer's
buffers (test infrastructure: the product step is HIP-only).  Per parameter:
clip_grad_norm_ (detectron2 "norm") or one global norm, then torch.optim SGD / AdamW
arithmetic — the same formulas as oracle/ref_solver.py's torch optimisers; parameters
whose gradient flag is clear are skipped (torch.optim: .grad None), AdamW's bias
correction counts each parameter's own steps."""
from __future__ import annotations

import math

import torch


@torch.no_grad()
def flat_step_reference(opt):
    s = opt.solver
    lay = opt.layout
    g = opt.reduced_grads().double() / opt.world
    has = (opt.flags.float() > 0.5).tolist()          # torch.optim skips parameters without .grad
    opt.step_count += 1
    for i, h in enumerate(has):
        if h:
            opt.param_steps[i] += 1
    views = [(o, n) for (o, n) in lay.offsets]
    scale = [1.0] * len(views)
    if s.clip_type == "norm":
        scale = [min(1.0, s.clip_value / (float(g[o:o + n].norm()) + 1e-6)) for o, n in views]
    elif s.clip_type == "full_model":
        tot = math.sqrt(sum(float(g[o:o + n].pow(2).sum()) for (o, n), h in zip(views, has) if h))
        scale = [min(1.0, s.clip_value / (tot + 1e-6))] * len(views)
    for i, ((o, n), (_, _, lrm, wd)) in enumerate(zip(views, lay.entries)):
        if not has[i]:
            continue
        t = float(opt.param_steps[i])
        gi = g[o:o + n] * scale[i]
        p = opt.master[o:o + n].double()
        lr = float(opt.lr) * lrm
        if s.optimizer == "sgd":
            d = gi + wd * p
            m = d if t <= 1 else s.momentum * opt.state1[o:o + n].double() + d
            p = p - lr * m
            opt.state1[o:o + n] = m.float()
        else:
            b1, b2 = s.betas
            p = p * (1 - lr * wd)
            m = opt.state1[o:o + n].double() * b1 + (1 - b1) * gi
            v = opt.state2[o:o + n].double() * b2 + (1 - b2) * gi * gi
            denom = v.sqrt() / math.sqrt(1 - b2 ** t) + s.eps
            p = p - lr / (1 - b1 ** t) * m / denom
            opt.state1[o:o + n] = m.float()
            opt.state2[o:o + n] = v.float()
        opt.master[o:o + n] = p.float()
    if opt.master is not opt.weights:
        opt.weights.copy_(opt.master)
