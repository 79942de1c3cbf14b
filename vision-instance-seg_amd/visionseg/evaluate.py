"""COCO-style mask AP for the training seam's metrics dict.

The reference evaluates with detectron2 COCOEvaluator / pycocotools
(training/maskdino/evaluate.py:120-132), neither of which is installed here; this is a
restatement of the COCO protocol for segm: per class, detections sorted by score
(maxDets 100), greedy matching at each IoU threshold 0.50:0.05:0.95, 101-point
interpolated precision, AP averaged over thresholds and classes (no area ranges, no
crowd regions).  `precision` / `recall` (train_template.py:139-145 keys) are taken at
IoU 0.5 over detections with score >= `score_thresh`.
"""
from __future__ import annotations

import numpy as np
import torch

IOU_THRS = np.linspace(0.5, 0.95, 10)
REC_THRS = np.linspace(0.0, 1.0, 101)


def mask_iou(pred: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
    """bool [N,H,W] x bool [K,H,W] -> IoU [N,K]."""
    if pred.shape[0] == 0 or gt.shape[0] == 0:
        return torch.zeros(pred.shape[0], gt.shape[0])
    p = pred.flatten(1).float()
    g = gt.flatten(1).float()
    inter = p @ g.t()
    union = p.sum(1)[:, None] + g.sum(1)[None, :] - inter
    return (inter / union.clamp(min=1)).cpu()


class MaskAPEvaluator:
    def __init__(self, num_classes: int = 1, max_dets: int = 100, score_thresh: float = 0.5):
        self.nc, self.max_dets, self.score_thresh = num_classes, max_dets, score_thresh
        self.dets = {c: [] for c in range(num_classes)}   # (score, tp[T]) per detection
        self.npos = {c: 0 for c in range(num_classes)}
        self.pr = [0, 0, 0]                                # tp, fp, npos at IoU .5 and score >= thr

    def add(self, scores, labels, masks, gt_masks, gt_labels):
        scores = scores.detach().float().cpu()
        labels = labels.detach().cpu()
        gt_labels = gt_labels.detach().cpu()
        for c in range(self.nc):
            pi = (labels == c).nonzero().flatten()
            gi = (gt_labels == c).nonzero().flatten()
            self.npos[c] += int(gi.numel())
            if pi.numel() == 0:
                self.pr[2] += int(gi.numel())
                continue
            order = pi[torch.argsort(scores[pi], descending=True)][: self.max_dets]
            iou = mask_iou(masks[order.to(masks.device)].bool(), gt_masks[gi.to(gt_masks.device)].bool()).numpy()
            tps = np.zeros((len(order), len(IOU_THRS)), dtype=bool)
            for t, thr in enumerate(IOU_THRS):
                used = np.zeros(len(gi), dtype=bool)
                for d in range(len(order)):
                    best, bj = thr - 1e-10, -1
                    for j in range(len(gi)):
                        if not used[j] and iou[d, j] >= best:
                            best, bj = iou[d, j], j
                    if bj >= 0:
                        used[bj] = True
                        tps[d, t] = True
            sc = scores[order].numpy()
            for d in range(len(order)):
                self.dets[c].append((float(sc[d]), tps[d]))
            keep = sc >= self.score_thresh
            self.pr[0] += int(tps[keep, 0].sum())
            self.pr[1] += int((~tps[keep, 0]).sum())
            self.pr[2] += int(gi.numel())

    def summarize(self) -> dict:
        aps = np.full((len(IOU_THRS), self.nc), np.nan)
        for c in range(self.nc):
            if self.npos[c] == 0:
                continue
            if not self.dets[c]:
                aps[:, c] = 0.0
                continue
            d = sorted(self.dets[c], key=lambda x: -x[0])
            tp = np.stack([x[1] for x in d]).astype(np.float64)     # [D, T]
            fp = 1.0 - tp
            ctp, cfp = np.cumsum(tp, 0), np.cumsum(fp, 0)
            for t in range(len(IOU_THRS)):
                rc = ctp[:, t] / self.npos[c]
                pr = ctp[:, t] / np.maximum(ctp[:, t] + cfp[:, t], np.finfo(np.float64).eps)
                pr = np.maximum.accumulate(pr[::-1])[::-1]          # precision envelope
                inds = np.searchsorted(rc, REC_THRS, side="left")
                q = np.array([pr[i] if i < len(pr) else 0.0 for i in inds])
                aps[t, c] = q.mean()
        def m(x):
            x = x[~np.isnan(x)]
            return float(x.mean()) if x.size else 0.0
        tp, fp, npos = self.pr
        return {"mAP50": m(aps[0]), "mAP75": m(aps[5]), "mAP": m(aps),
                "precision": tp / max(1, tp + fp), "recall": tp / max(1, npos)}
