"""Mask2Former set criterion on the GPU (semantics of HF:m2f:378-794 / upstream
SetCriterion + HungarianMatcher).

Same losses and weights as the oracle (CE with no-object weight 0.1, point-sampled
sigmoid-BCE and dice on 12544 importance-sampled points, Hungarian matching on
uniformly sampled points; class 2 / mask 5 / dice 5; every decoder step supervised),
restructured for the device:

* the matching costs of ALL decoder steps and ALL images are computed in a few
  batched kernels, and the assignments are solved ON THE DEVICE (csrc/match.hip, one
  wave per (step, image) Hungarian problem): the reference's per-image, per-layer
  `linear_sum_assignment(cost.cpu())` is 10 x B host syncs per step, here there is none,
  so the host keeps enqueueing the loss and the backward while the GPU runs the forward;
* the mask/dice/CE losses of all decoder steps are evaluated as one batch over the
  matched (query, target) pairs;
* targets are carried PADDED (`PaddedTargets`: masks [B, Kc, H, W], classes [B, Kc],
  per-image counts [B] on the device, Kc = the batch's largest count): no shape or launch
  depends on the individual counts, so a captured HIP graph of the training step
  (train.Trainer(graphs=True)) serves every batch with the same Kc, and the padded
  columns / pairs are masked out of the matching and the losses.

`matcher="host"` keeps scipy's `linear_sum_assignment` (the reference's choice); both
return the same optimum (unique for generic costs).  The random points come from the
device generator; the `point_source` hook feeds both this criterion and the oracle's the
same keyed draws, which is how tests/test_gpu_train_parity.py compares the GPU loss and
gradients with the oracle's.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import ops


# A/B switch: the fused matcher-cost kernel (default) or the torch formulation below it
_FUSED_COST = os.environ.get("VS_MATCH_FUSED", "1") == "1"
# A/B switch: target labels at points from the bool masks on the HIP kernel (default) or
# grid_sample on an f32 copy
_MASK_SAMPLE_KERNEL = os.environ.get("VS_MASK_SAMPLE", "1") == "1"


def _sample(feat, coords):
    """point_sample (HF:m2f:245-275): feat [N,1,H,W], coords [N,P,2] in [0,1] -> [N,P]
    (ops.point_sample: the HIP point gather on the device)."""
    return ops.point_sample(feat, coords)


def _target_points(tg, grid):
    """The padded target masks sampled at the matcher's points (HF:m2f:453-459):
    grid [B,P,1,2] in [-1,1] (one point set per image) -> [B,Kc,P] f32.  On the device the
    bool masks are read as they are (ops.point_sample_masks), not copied to f32 first."""
    B, Kc = tg.masks.shape[:2]
    if tg.masks.is_cuda and _MASK_SAMPLE_KERNEL:
        H, W = tg.masks.shape[-2:]
        return ops.point_sample_masks(tg.masks.view(B * Kc, H, W), grid.squeeze(2), grid_space=True,
                                      sets_per_coord=Kc).view(B, Kc, -1)
    return F.grid_sample(tg.masks.float(), grid, align_corners=False).squeeze(3)


class PaddedTargets:
    """Per-image instance targets padded to the batch's largest count Kc.

    masks [B, Kc, H, W] (bool/uint8, zero past the count), classes int64 [B, Kc] (0 past
    the count), counts int32 [B] on the device.  `kc` is a host int (a shape); the counts
    themselves never reach the host."""

    def __init__(self, masks, classes, counts):
        self.masks, self.classes, self.counts = masks, classes, counts
        self.kc = int(classes.shape[1])

    @classmethod
    def from_lists(cls, mask_labels, class_labels, kc=None, device=None):
        """The reference's per-image lists ([K_i, H, W] masks, [K_i] classes) -> padded."""
        B = len(class_labels)
        ks = [int(t.shape[0]) for t in class_labels]
        kc = max(ks + [0]) if kc is None else int(kc)
        if any(k > kc for k in ks):
            raise ValueError(f"an image has {max(ks)} targets, more than the padded capacity {kc}")
        dev = device if device is not None else (mask_labels[0].device if B else "cpu")
        H, W = (int(mask_labels[0].shape[-2]), int(mask_labels[0].shape[-1])) if B else (0, 0)
        masks = torch.zeros(B, kc, H, W, dtype=torch.bool, device=dev)
        classes = torch.zeros(B, kc, dtype=torch.int64, device=dev)
        for i, (m, c) in enumerate(zip(mask_labels, class_labels)):
            if ks[i]:
                masks[i, :ks[i]] = m.to(dev)
                classes[i, :ks[i]] = c.to(dev)
        counts = torch.tensor(ks, dtype=torch.int32).to(dev)
        return cls(masks, classes, counts)

    def copy_from_lists(self, mask_labels, class_labels):
        """Refill in place (static buffers of a captured graph): eager copies, no reallocation."""
        ks = [int(t.shape[0]) for t in class_labels]
        if len(ks) != self.masks.shape[0] or max(ks + [0]) > self.kc:
            raise ValueError("targets do not fit the padded buffers")
        with torch.no_grad():
            self.masks.zero_()
            self.classes.zero_()
            for i, (m, c) in enumerate(zip(mask_labels, class_labels)):
                if ks[i]:
                    self.masks[i, :ks[i]].copy_(m)
                    self.classes[i, :ks[i]].copy_(c)
            self.counts.copy_(torch.tensor(ks, dtype=torch.int32), non_blocking=False)

    def valid(self):
        """bool [B, Kc]: target k of image b exists."""
        return torch.arange(self.kc, device=self.counts.device)[None, :] < self.counts[:, None]


def as_padded(mask_labels, class_labels, device):
    if isinstance(mask_labels, PaddedTargets):
        return mask_labels
    return PaddedTargets.from_lists(mask_labels, class_labels, device=device)


class SetCriterion:
    # reads ops.FactoredLogits (the matcher and the matched maps from the mask head's
    # factors): train.Trainer switches the decoder's factored output on for it
    accepts_factored_logits = True

    def __init__(self, cfg, matcher: str = "device", point_source=None):
        """matcher: "device" (csrc/match.hip, no host sync) or "host" (scipy, the
        reference's linear_sum_assignment).  point_source: None (device RNG) or a parity
        hook with `match_points(B, P, device) -> [B,P,2]` and `loss_points(S, B, Kc, n,
        kind, device) -> [S,B,Kc,n,2]` in [0,1) (kind "over": the oversampled candidates,
        "rand": the uniform remainder), draws keyed by (step, image, target) so the
        oracle criterion (oracle/ref_model.RefCriterion) can be fed the same points."""
        if matcher not in ("device", "host"):
            raise ValueError(matcher)
        self.cfg = cfg
        self.num_labels = cfg.num_labels
        self.matcher = matcher
        self.point_source = point_source
        self._ew = {}
        self._rows = {}

    def _loss_points(self, S, B, Kc, n, kind, dev):
        if self.point_source is None:
            return torch.rand(S * B * Kc, n, 2, device=dev)
        return self.point_source.loss_points(S, B, Kc, n, kind, dev).reshape(S * B * Kc, n, 2).to(dev)

    # --------------------------------------------------------------- matching
    @torch.no_grad()
    def match(self, masks_list, classes, mask_labels, class_labels=None):
        """masks_list: S x [B,Q,H,W] (S decoder steps), classes [S,B,Q,K+1], targets as
        lists or PaddedTargets -> int32 [S, B, Kc] on the device: the query matched to
        each target (-1 past the image's count).  Costs as HF:m2f:434-481 (HungarianMatcher:
        class -prob, sigmoid-BCE and dice on `train_num_points` uniform points)."""
        c = self.cfg
        S = len(masks_list)
        B, Q = masks_list[0].shape[:2]
        dev = masks_list[0].device
        tg = as_padded(mask_labels, class_labels, dev)
        Kc = max(1, tg.kc)
        if tg.kc > Q:
            raise ValueError(f"an image has more targets ({tg.kc}) than queries ({Q})")
        probs = classes.float().softmax(-1)                                              # [S,B,Q,C+1]
        # one uniform point set per image, shared by its queries, targets and the S steps:
        # queries / targets are grid_sample CHANNELS (one call per step, one for all targets)
        P = c.train_num_points
        u = (self.point_source.match_points(B, P, dev).to(dev) if self.point_source is not None
             else torch.rand(B, P, 2, device=dev))
        grid = (2.0 * u - 1.0).unsqueeze(2)                                              # [B,P,1,2]
        if ops.factored(masks_list):
            m0 = masks_list[0]
            if (self.matcher == "device" and 1 <= tg.kc <= 16 and Kc <= ops.lsa_max_targets(Q)
                    and m0.E.dtype == torch.bfloat16 and m0.E.shape[-1] in (64, 128, 256)):
                # the point logits are E_s . F(p): F sampled once at the points (hi | lo
                # bf16 pair), the costs from the factors (csrc/match_factors.hip) -- no
                # full-resolution logits of the S steps are made or read
                fp = ops.feature_sample_hilo(m0.F, m0.H, m0.W, grid.squeeze(2))
                tp = _target_points(tg, grid)                                              # [B,Kc,P]
                cost = ops.match_cost_factors(m0.E, fp, probs, tg.classes, tp, c.mask_weight, c.class_weight,
                                              c.dice_weight)
                return ops.linear_sum_assignment_padded(cost, tg.counts)
            masks_list = ops.materialize_masks(masks_list)
        if (self.matcher == "device" and dev.type == "cuda" and 1 <= tg.kc <= 16 and S <= 16
                and Kc <= ops.lsa_max_targets(Q) and _FUSED_COST):
            # one kernel: point-sampled logits, BCE / dice / class costs (csrc/match.hip).
            # The points are taken in pixel-row order (the cost sums over them): each
            # wave's taps then share cache lines and a logit map streams through L2 once
            H, W = masks_list[0].shape[-2:]
            key = (((grid[..., 0, 1] + 1) * (H / 2)).floor() * W + ((grid[..., 0, 0] + 1) * (W / 2)).floor())
            grid = torch.gather(grid, 1, key.argsort(dim=1)[:, :, None, None].expand(B, P, 1, 2))
            tp = _target_points(tg, grid)                                                  # [B,Kc,P]
            cost = ops.match_cost(masks_list, probs, tg.classes, grid.squeeze(2), tp, c.mask_weight,
                                  c.class_weight, c.dice_weight)
            return ops.linear_sum_assignment_padded(cost, tg.counts)
        pp = torch.stack([F.grid_sample(m.float(), grid, align_corners=False).squeeze(3)
                          for m in masks_list])                                          # [S,B,Q,P]
        if tg.kc:
            tp = _target_points(tg, grid)                                                  # [B,Kc,P]
        else:
            tp = torch.zeros(B, 1, P, device=dev)
        tpt = tp.transpose(1, 2)[None]                                                   # [1,B,P,Kc]
        Pn = pp.shape[-1]
        pos = F.softplus(-pp)          # BCE(x, 1)
        neg = F.softplus(pp)           # BCE(x, 0)
        cm = torch.matmul(pos / Pn, tpt) + torch.matmul(neg / Pn, 1 - tpt)              # [S,B,Q,Kc]
        sg = pp.sigmoid()
        num = 2 * torch.matmul(sg, tpt)
        den = sg.sum(-1)[..., None] + tp.sum(-1)[None, :, None, :]
        cd = 1 - (num + 1) / (den + 1)
        cls = (tg.classes if tg.kc else torch.zeros(B, 1, dtype=torch.int64, device=dev))
        cc = -torch.gather(probs, 3, cls[None, :, None, :].expand(S, B, Q, Kc))
        cost = c.mask_weight * cm + c.class_weight * cc + c.dice_weight * cd
        cost = torch.nan_to_num(cost.clamp(-1e10, 1e10), 0.0)
        if self.matcher == "device" and cost.is_cuda and Kc <= ops.lsa_max_targets(Q):
            return ops.linear_sum_assignment_padded(cost, tg.counts)                    # csrc/match.hip, no sync
        # scipy on the host (the reference's matcher): one device->host sync
        host = cost.cpu().numpy()
        ks = tg.counts.cpu().tolist()
        from scipy.optimize import linear_sum_assignment
        out = np.full((S, B, Kc), -1, dtype=np.int32)
        for s in range(S):
            for i in range(B):
                if ks[i]:
                    a, b = linear_sum_assignment(host[s, i, :, :ks[i]])
                    out[s, i, b] = a
        return torch.from_numpy(out).to(dev)

    # --------------------------------------------------------------- losses
    def _num_masks(self, tg, device):
        tot = getattr(self, "num_masks_total", None)
        if tot is not None:       # global count supplied by the trainer (graph-replayed steps)
            ws = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
            return torch.clamp(tot / ws, min=1)
        n = tg.counts.sum().float()                                   # on the device, no sync
        ws = 1
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(n)
            ws = dist.get_world_size()
        return torch.clamp(n / ws, min=1)

    def __call__(self, masks_list, classes_list, mask_labels, class_labels=None):
        """masks_list: per decoder step [B,Q,H,W] logits; classes_list: per step [B,Q,K+1];
        targets as the reference's per-image lists or a PaddedTargets.  Returns (total
        loss, dict of weighted components; keys as HF: final step un-suffixed, aux steps
        `_{i}`)."""
        c = self.cfg
        classes = torch.stack(classes_list)      # [S,B,Q,K+1]
        S, B, Q = classes.shape[:3]
        dev = classes.device
        tg = as_padded(mask_labels, class_labels, dev)
        Kc = tg.kc
        assign = self.match([m.detach() for m in masks_list], classes.detach(), tg)
        forced = getattr(self.point_source, "forced_assign", None)
        if forced is not None:      # parity hook: another run's matching decisions (tests/_draws.py)
            assign = forced(assign)
        nm = self._num_masks(tg, dev)
        ew = self._ew.get(dev)
        if ew is None:        # made once: a scalar store is a host->device copy (not capturable)
            ew = torch.ones(self.num_labels + 1, device=dev)
            ew[-1] = c.no_object_weight
            self._ew[dev] = ew
        # target class per query (no-object where unmatched): matched pairs scatter their
        # class; padded pairs go to a spare column Q that is dropped
        tc = torch.full((S, B, Q + 1), self.num_labels, dtype=torch.int64, device=dev)
        if Kc:
            valid = tg.valid()                                                           # [B,Kc]
            qs = assign[..., :Kc].long()                                                 # [S,B,Kc]
            qidx = torch.where(valid[None] & (qs >= 0), qs, torch.full_like(qs, Q))
            tc.scatter_(2, qidx, tg.classes[None].expand(S, B, Kc))
        tc = tc[..., :Q].contiguous()
        ce = F.cross_entropy(classes.float().reshape(S * B, Q, -1).transpose(1, 2), tc.view(S * B, Q),
                             weight=ew, reduction="none")                                  # [S*B, Q]
        # weighted mean per step, as nn.CrossEntropyLoss(weight) does
        wsum = ew[tc.view(S * B, Q)].view(S, B * Q).sum(-1)
        loss_ce = ce.view(S, B * Q).sum(-1) / wsum                                         # [S]
        if Kc:
            # every (step, image, target slot) pair; padded slots point at query 0 and are
            # masked out of the sums
            qsel = qidx.clamp(max=Q - 1)                                                 # [S,B,Kc]
            # the matched maps [S*B*Kc, 1, H, W]; when the logits came from the mask head the
            # loss differentiates through its factors (ops.MatchedPointLogitsFunction: no
            # full-size logits gradient, one adjoint GEMM pair for all steps)
            pred, fac = ops.matched_maps(masks_list, qsel)
            NP = B * Kc
            with torch.no_grad():
                npts = c.train_num_points
                ns = int(npts * c.oversample_ratio)
                nu = int(c.importance_sample_ratio * npts)
                coords = self._loss_points(S, B, Kc, ns, "over", dev)
                unc = -torch.abs(_sample(pred.detach().float(), coords))
                select = getattr(self.point_source, "select", None)
                if select is None:
                    top = ops.topk_rows(unc, nu) if unc.is_cuda else torch.topk(unc, k=nu, dim=1)[1]
                else:              # parity hook, rows keyed (step, image, target slot)
                    keys = (torch.arange(S).repeat_interleave(B * Kc), torch.arange(B).repeat_interleave(Kc).repeat(S),
                            torch.arange(Kc).repeat(S * B))
                    top = select(unc, nu, *keys)
                coords = torch.gather(coords, 1, top[..., None].expand(-1, -1, 2))
                if npts - nu > 0:
                    coords = torch.cat([coords, self._loss_points(S, B, Kc, npts - nu, "rand", dev)], 1)
                # the target labels at the points: pair (s, i) reads target mask i
                if dev.type == "cuda" and _MASK_SAMPLE_KERNEL:     # straight from the bool masks
                    rows = self._rows.get((S, NP, dev))
                    if rows is None:
                        rows = self._rows[(S, NP, dev)] = torch.arange(S * NP, device=dev) % NP
                    plab = ops.point_sample_masks(tg.masks.reshape(NP, *tg.masks.shape[-2:]), coords, rows=rows)
                else:
                    by_t = coords.view(S, NP, npts, 2).transpose(0, 1)                     # [NP,S,P,2]
                    tgt = tg.masks.reshape(NP, 1, *tg.masks.shape[-2:]).float()
                    lab_t = _sample(tgt, by_t.reshape(NP, S * npts, 2)).view(NP, S, npts)
                    plab = lab_t.transpose(0, 1).reshape(S * NP, npts)
            plog = ops.point_logits(pred, coords, qsel, fac)
            keep = valid.reshape(1, NP).expand(S, NP).reshape(S * NP)
            bce = F.binary_cross_entropy_with_logits(plog, plab, reduction="none").mean(1)  # [S*NP]
            zero = torch.zeros((), device=dev)
            loss_mask = torch.where(keep, bce, zero).view(S, NP).sum(-1) / nm
            pr = plog.sigmoid()
            dice = 1 - (2 * (pr * plab).sum(-1) + 1) / (pr.sum(-1) + plab.sum(-1) + 1)
            loss_dice = torch.where(keep, dice, zero).view(S, NP).sum(-1) / nm
        else:
            fac = ops.mask_head_factors(masks_list)
            anchor = (fac[0].float().sum() + fac[1].float().sum()) if fac is not None else sum(m.sum() for m in masks_list)
            loss_mask = anchor * 0.0 + torch.zeros(S, device=dev)
            loss_dice = torch.zeros(S, device=dev)
        losses = {}
        for s in range(S):
            suf = "" if s == S - 1 else f"_{s}"
            losses[f"loss_cross_entropy{suf}"] = c.class_weight * loss_ce[s]
            losses[f"loss_mask{suf}"] = c.mask_weight * loss_mask[s]
            losses[f"loss_dice{suf}"] = c.dice_weight * loss_dice[s]
        total = c.class_weight * loss_ce.sum() + c.mask_weight * loss_mask.sum() + c.dice_weight * loss_dice.sum()
        return total, losses
