"""ORACLE (test infrastructure only) — CPU restatement of the reference's solver step.

The reference trains through detectron2's `DefaultTrainer` (training/maskdino/
train_full.py:153-167; `MaskDINOTrainer` does not override `build_optimizer`), so its
optimizer is detectron2's default (upstream detectron2/solver/build.py, not in the
container):

* parameter groups from `get_default_optimizer_params(model, base_lr,
  weight_decay_norm=SOLVER.WEIGHT_DECAY_NORM (0.0), bias_lr_factor=1.0,
  weight_decay_bias=None)`: every parameter of a normalisation module (BatchNorm,
  GroupNorm, LayerNorm, ...) gets weight decay 0, every other parameter
  SOLVER.WEIGHT_DECAY (0.05 in MaskDINO's base config);
* `torch.optim.SGD(momentum=SOLVER.MOMENTUM 0.9, nesterov=False)`;
* `maybe_add_gradient_clipping` with CLIP_TYPE "norm", CLIP_VALUE 0.01, NORM_TYPE 2.0
  (train_full.py:266-271): `clip_grad_norm_(p, 0.01, 2.0)` for EVERY parameter on its
  own, before the update;
* the lr of WarmupMultiStepLR (BASE_LR 1e-4, train_full.py:251-254).

Upstream Mask2Former / MaskDINO `train_net.py` (not what the reference runs, but what
their configs' SOLVER.OPTIMIZER "ADAMW" means there) use AdamW with decay 0 for norm and
embedding parameters and the relative-position tables, and lr x BACKBONE_MULTIPLIER 0.1
for backbone parameters; `ref_param_groups(..., optimizer="adamw")` restates that.

The update itself is torch's own CPU single-tensor SGD / AdamW (what detectron2 calls).
"""
from __future__ import annotations

import torch
import torch.nn as nn

NORM_TYPES = (nn.BatchNorm1d, nn.BatchNorm2d, nn.BatchNorm3d, nn.SyncBatchNorm, nn.GroupNorm,
              nn.InstanceNorm1d, nn.InstanceNorm2d, nn.InstanceNorm3d, nn.LayerNorm, nn.LocalResponseNorm)


def ref_param_groups(model: nn.Module, lr: float, weight_decay: float, optimizer: str = "sgd",
                     backbone_multiplier: float = 0.1):
    """[{"params": [p], "lr": .., "weight_decay": .., "name": n}] in model.named_modules
    order, one group per parameter (detectron2 get_default_optimizer_params)."""
    groups, seen = [], set()
    for mname, module in model.named_modules():
        for pname, p in module.named_parameters(recurse=False):
            if not p.requires_grad or id(p) in seen:
                continue
            seen.add(id(p))
            name = f"{mname}.{pname}" if mname else pname
            wd, plr = weight_decay, lr
            if isinstance(module, NORM_TYPES):
                wd = 0.0
            if optimizer == "adamw":
                if isinstance(module, nn.Embedding) or "rel_table" in pname or "absolute_pos_embed" in pname:
                    wd = 0.0
                if name.startswith("backbone."):
                    plr = lr * backbone_multiplier
            groups.append({"params": [p], "lr": plr, "weight_decay": wd, "name": name})
    return groups


@torch.no_grad()
def ref_clip_per_parameter(params, max_norm: float, norm_type: float = 2.0):
    """detectron2 CLIP_TYPE "norm": clip_grad_norm_(p, max_norm) for each parameter."""
    for p in params:
        if p.grad is not None:
            torch.nn.utils.clip_grad_norm_([p], max_norm, norm_type)


@torch.no_grad()
def ref_clip_full_model(params, max_norm: float, norm_type: float = 2.0):
    """detectron2 / MaskDINO CLIP_TYPE "full_model": one global norm."""
    torch.nn.utils.clip_grad_norm_([p for p in params if p.grad is not None], max_norm, norm_type)


def ref_optimizer(groups, optimizer: str = "sgd", momentum: float = 0.9, betas=(0.9, 0.999), eps: float = 1e-8):
    """torch's single-tensor CPU implementation of the update the reference calls."""
    gs = [{k: v for k, v in g.items() if k != "name"} for g in groups]
    if optimizer == "sgd":
        return torch.optim.SGD(gs, lr=gs[0]["lr"], momentum=momentum, nesterov=False, foreach=False)
    if optimizer == "adamw":
        return torch.optim.AdamW(gs, lr=gs[0]["lr"], betas=betas, eps=eps, foreach=False)
    raise ValueError(optimizer)
