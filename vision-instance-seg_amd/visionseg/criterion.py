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
  matched (query, target) pairs, ordered by target.

`matcher="host"` keeps scipy's `linear_sum_assignment` (the reference's choice); both
return the same optimum (unique for generic costs).  The random points come from the
device generator, so a GPU loss is not bit-comparable with the CPU oracle's (documented
in DESIGN.md; the oracle's loss is pinned to HF).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import ops


def _sample(feat, coords):
    """point_sample (HF:m2f:245-275): feat [N,1,H,W], coords [N,P,2] in [0,1] -> [N,P]."""
    return F.grid_sample(feat, 2.0 * coords.unsqueeze(2) - 1.0, align_corners=False).squeeze(3).squeeze(1)


class SetCriterion:
    def __init__(self, cfg, matcher: str = "device"):
        """matcher: "device" (csrc/match.hip, no host sync) or "host" (scipy, the
        reference's linear_sum_assignment)."""
        if matcher not in ("device", "host"):
            raise ValueError(matcher)
        self.cfg = cfg
        self.num_labels = cfg.num_labels
        self.matcher = matcher
        self._pairs = {}
        self._ew = {}

    # --------------------------------------------------------------- matching
    @torch.no_grad()
    def match(self, masks_list, classes, mask_labels, class_labels):
        """masks_list: S x [B,Q,H,W] (S decoder steps), classes [S,B,Q,K+1] -> int32
        [S, B, Kmax] on the device: the query matched to each target (-1 padding)."""
        c = self.cfg
        S = len(masks_list)
        B, Q = masks_list[0].shape[:2]
        dev = masks_list[0].device
        kmax = max(1, max(int(t.shape[0]) for t in class_labels))
        cost = torch.zeros(S, B, Q, kmax, device=dev)
        probs = classes.float().softmax(-1)
        # one uniform point set per image, shared by its queries and the S decoder steps:
        # the queries are grid_sample CHANNELS, so one call per step samples all B x Q masks
        P = c.train_num_points
        grid = (2.0 * torch.rand(B, P, 2, device=dev) - 1.0).unsqueeze(2)              # [B,P,1,2]
        pp_all = torch.stack([F.grid_sample(m.float(), grid, align_corners=False).squeeze(3)
                              for m in masks_list])                                      # [S,B,Q,P]
        for i in range(B):
            K = int(class_labels[i].shape[0])
            if K == 0:
                continue
            tp = F.grid_sample(mask_labels[i].float()[None], grid[i:i + 1], align_corners=False)
            tp = tp.squeeze(3)[0][None].expand(S, -1, -1)                                  # [S,K,P]
            pp = pp_all[:, i]                                                            # [S,Q,P]
            P = pp.shape[-1]
            pos = F.softplus(-pp)          # BCE(x, 1)
            neg = F.softplus(pp)           # BCE(x, 0)
            cm = torch.bmm(pos / P, tp.transpose(1, 2)) + torch.bmm(neg / P, (1 - tp).transpose(1, 2))
            sg = pp.sigmoid()
            num = 2 * torch.bmm(sg, tp.transpose(1, 2))
            den = sg.sum(-1)[:, :, None] + tp.sum(-1)[:, None, :]
            cd = 1 - (num + 1) / (den + 1)
            cc = -probs[:, i][:, :, class_labels[i]]
            cost[:, i, :, :K] = c.mask_weight * cm + c.class_weight * cc + c.dice_weight * cd
        cost = torch.nan_to_num(cost.clamp(-1e10, 1e10), 0.0)
        ks = [int(t.shape[0]) for t in class_labels]
        if any(k > Q for k in ks):
            raise ValueError(f"an image has more targets ({max(ks)}) than queries ({Q})")
        if self.matcher == "device" and cost.is_cuda and max(ks) <= ops.lsa_max_targets(Q):
            return ops.linear_sum_assignment_batch(cost, ks)           # csrc/match.hip, no host sync
        # scipy on the host (the reference's matcher): one device->host sync
        host = cost.cpu().numpy()
        from scipy.optimize import linear_sum_assignment
        out = np.full((S, B, kmax), -1, dtype=np.int32)
        for s in range(S):
            for i in range(B):
                if ks[i]:
                    a, b = linear_sum_assignment(host[s, i, :, :ks[i]])
                    out[s, i, b] = a
        return torch.from_numpy(out).to(dev)

    # --------------------------------------------------------------- losses
    def _num_masks(self, class_labels, device):
        tot = getattr(self, "num_masks_total", None)
        if tot is not None:       # global count supplied by the trainer (graph-replayed steps)
            ws = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
            return torch.clamp(tot / ws, min=1)
        n = torch.full((), float(sum(int(t.shape[0]) for t in class_labels)), device=device)   # fill, no copy
        ws = 1
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(n)
            ws = dist.get_world_size()
        return torch.clamp(n / ws, min=1)

    def __call__(self, masks_list, classes_list, mask_labels, class_labels):
        """masks_list: per decoder step [B,Q,H,W] logits; classes_list: per step [B,Q,K+1].
        Returns (total loss, dict of weighted components; keys as HF: final step
        un-suffixed, aux steps `_{i}`)."""
        c = self.cfg
        classes = torch.stack(classes_list)      # [S,B,Q,K+1]
        S, B, Q = classes.shape[:3]
        dev = classes.device
        assign = self.match([m.detach() for m in masks_list], classes.detach(), mask_labels, class_labels)
        nm = self._num_masks(class_labels, dev)
        # matched pairs of every step, ordered by target t (image-major): image bs[t], the
        # target's index k within its image, its query qs[s, t]; all on the device
        ks = tuple(int(t.shape[0]) for t in class_labels)
        N = sum(ks)
        if (ks, dev) not in self._pairs:
            img = [torch.full((k,), i, device=dev, dtype=torch.int64) for i, k in enumerate(ks) if k]
            kin = [torch.arange(k, device=dev) for k in ks if k]
            self._pairs[(ks, dev)] = (torch.cat(img), torch.cat(kin)) if N else (None, None)
        bt, kt = self._pairs[(ks, dev)]
        tgt_all = torch.cat([m.float() for m in mask_labels], 0) if N else None
        tc = torch.full((S, B, Q), self.num_labels, dtype=torch.int64, device=dev)
        if N:
            qs = assign[:, bt, kt].long()                                                  # [S, N]
            bs = bt.expand(S, N)
            cls_all = torch.cat([t.to(dev) for t in class_labels]).long()
            tc[torch.arange(S, device=dev)[:, None], bs, qs] = cls_all.expand(S, N)
        ew = self._ew.get(dev)
        if ew is None:        # made once: a scalar store is a host->device copy (not capturable)
            ew = torch.ones(self.num_labels + 1, device=dev)
            ew[-1] = c.no_object_weight
            self._ew[dev] = ew
        ce = F.cross_entropy(classes.float().reshape(S * B, Q, -1).transpose(1, 2), tc.view(S * B, Q),
                             weight=ew, reduction="none")                                  # [S*B, Q]
        # weighted mean per step, as nn.CrossEntropyLoss(weight) does
        wsum = ew[tc.view(S * B, Q)].view(S, B * Q).sum(-1)
        loss_ce = ce.view(S, B * Q).sum(-1) / wsum                                         # [S]
        if N:
            pred = torch.stack([masks_list[k][bs[k], qs[k]] for k in range(S)])           # [S,N,H,W]
            H, W = pred.shape[-2:]
            pred = pred.reshape(S * N, 1, H, W)
            with torch.no_grad():
                npts = c.train_num_points
                ns = int(npts * c.oversample_ratio)
                nu = int(c.importance_sample_ratio * npts)
                coords = torch.rand(S * N, ns, 2, device=dev)
                unc = -torch.abs(_sample(pred.detach().float(), coords))
                top = torch.topk(unc, k=nu, dim=1)[1]
                coords = torch.gather(coords, 1, top[..., None].expand(-1, -1, 2))
                if npts - nu > 0:
                    coords = torch.cat([coords, torch.rand(S * N, npts - nu, 2, device=dev)], 1)
                # sample each full-resolution target once, with the coordinates of the S
                # predictions it is matched to (pairs are target-ordered in every step)
                by_t = coords.view(S, N, npts, 2).transpose(0, 1)                          # [N,S,P,2]
                lab_t = _sample(tgt_all[:, None], by_t.reshape(N, S * npts, 2)).view(N, S, npts)
                plab = lab_t.transpose(0, 1).reshape(S * N, npts)
            plog = _sample(pred.float(), coords)
            bce = F.binary_cross_entropy_with_logits(plog, plab, reduction="none").mean(1)  # [S*N]
            loss_mask = bce.view(S, N).sum(-1) / nm
            pr = plog.sigmoid()
            dice = 1 - (2 * (pr * plab).sum(-1) + 1) / (pr.sum(-1) + plab.sum(-1) + 1)
            loss_dice = dice.view(S, N).sum(-1) / nm
        else:
            loss_mask = sum(m.sum() for m in masks_list) * 0.0 + torch.zeros(S, device=dev)
            loss_dice = torch.zeros(S, device=dev)
        losses = {}
        for s in range(S):
            suf = "" if s == S - 1 else f"_{s}"
            losses[f"loss_cross_entropy{suf}"] = c.class_weight * loss_ce[s]
            losses[f"loss_mask{suf}"] = c.mask_weight * loss_mask[s]
            losses[f"loss_dice{suf}"] = c.dice_weight * loss_dice[s]
        total = c.class_weight * loss_ce.sum() + c.mask_weight * loss_mask.sum() + c.dice_weight * loss_dice.sum()
        return total, losses
