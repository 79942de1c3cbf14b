"""MaskDINO on the MI355X path (BASELINE config C4: Swin-L + MaskDINO, 300 queries).

The reference trains MaskDINO (training/maskdino/train_full.py:228-232, base config
`maskdino_R50_bs16_50ep_4s_dowsample1_2048.yaml`, trainer :308-310) from an un-vendored
upstream checkout (MaskDINO, Li et al. CVPR 2023).  No MaskDINO source is
present in the container, so this restates the published architecture (upstream
maskdino/modeling/transformer_decoder/maskdino_decoder.py, dino_decoder.py,
pixel_decoder/maskdino_encoder.py, criterion.py, matcher.py) on the build's kernels --
**parity unpinned** (no oracle; the tests check structural properties instead):

* pixel decoder: visionseg.model.PixelDecoder with 4 levels ("4s": res5 downsampled by a
  stride-2 conv as a 1/64 level) and a 2048-wide encoder FFN ("_2048");
* two-stage query selection: the encoder memory through enc_output + LayerNorm, class
  and box heads on every token (boxes relative to per-level anchor proposals), the top
  `num_queries` tokens by class score become the decoder's content queries (detached)
  and their boxes its reference boxes (detached); those tokens' own predictions are the
  "interm" outputs;
* denoising (DN, "seg"): noised ground-truth boxes and labels as extra queries (label
  flips with probability noise_scale/2, box jitter of noise_scale), dn_num // K groups
  of K slots (K = the batch's largest target count, read on the device), an attention
  mask keeping the matching queries from the DN queries and the DN groups from each
  other;
* 9 deformable decoder layers (self-attention with the DN mask -> MSDA cross-attention
  to the 4-level memory with box reference points: loc = c + off / P * wh / 2 ->
  ReLU FFN 2048, post-norm), query positions from the sine embedding of the box through
  a 2-layer MLP, iterative box refinement (shared bbox head, reference detached per
  layer);
* predictions after the selection and every layer (initial_pred): classes (sigmoid,
  no "no-object" column), masks (the hand-written mask-head kernel: Q = 300 + DN), boxes.

Hot ops on the HIP kernels: window attention (backbone), MSDA sampling + prologue
(encoder and decoder cross-attention, 4 levels), mask head, LayerNorms; the rest is
vendor GEMMs and torch.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .linear import SmallLinear, TokenLayerNorm, TokenLinear, linear_tokens
from .model import M2FConfig, PixelDecoder, SwinBackbone, _compute_dtype, self_attention_core


@dataclass
class MaskDINOConfig(M2FConfig):
    n_levels: int = 4
    enc_ffn: int = 2048
    dec_ffn: int = 2048
    dec_layers: int = 9               # decoder layers (predictions: 1 + dec_layers steps)
    num_queries: int = 300
    dn: bool = True
    dn_num: int = 100
    noise_scale: float = 0.4
    focal_alpha: float = 0.25
    class_weight: float = 4.0
    box_weight: float = 5.0
    giou_weight: float = 2.0

    @staticmethod
    def preset(name: str, **kw) -> "MaskDINOConfig":
        base = M2FConfig.preset(name).to_dict()
        keep = {k: base[k] for k in ("embed_dim", "depths", "num_heads", "window_size")}
        keep.update(kw)
        return MaskDINOConfig.from_dict(keep)

    @staticmethod
    def from_dict(d):
        d = dict(d)
        for k in ("depths", "num_heads"):
            if k in d:
                d[k] = tuple(d[k])
        return MaskDINOConfig(**{k: v for k, v in d.items() if k in MaskDINOConfig.__dataclass_fields__})


def inverse_sigmoid(x, eps: float = 1e-5):
    x = x.clamp(min=0.0, max=1.0)
    return torch.log(x.clamp(min=eps) / (1 - x).clamp(min=eps))


def box_cxcywh_to_xyxy(b):
    cx, cy, w, h = b.unbind(-1)
    return torch.stack((cx - 0.5 * w, cy - 0.5 * h, cx + 0.5 * w, cy + 0.5 * h), -1)


def generalized_box_iou(a, b):
    """Pairwise GIoU of xyxy boxes a [..., N, 4] and b [..., M, 4] -> [..., N, M]."""
    area_a = (a[..., 2] - a[..., 0]) * (a[..., 3] - a[..., 1])
    area_b = (b[..., 2] - b[..., 0]) * (b[..., 3] - b[..., 1])
    lt = torch.maximum(a[..., :, None, :2], b[..., None, :, :2])
    rb = torch.minimum(a[..., :, None, 2:], b[..., None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    union = area_a[..., :, None] + area_b[..., None, :] - inter
    iou = inter / union.clamp(min=1e-7)
    lt2 = torch.minimum(a[..., :, None, :2], b[..., None, :, :2])
    rb2 = torch.maximum(a[..., :, None, 2:], b[..., None, :, 2:])
    wh2 = (rb2 - lt2).clamp(min=0)
    area = wh2[..., 0] * wh2[..., 1]
    return iou - (area - union) / area.clamp(min=1e-7)


def paired_giou(a, b):
    """GIoU of xyxy boxes a and b paired elementwise ([..., 4] each, broadcastable) -> [...]:
    the diagonal of generalized_box_iou without the pairwise matrix."""
    area_a = (a[..., 2] - a[..., 0]) * (a[..., 3] - a[..., 1])
    area_b = (b[..., 2] - b[..., 0]) * (b[..., 3] - b[..., 1])
    wh = (torch.minimum(a[..., 2:], b[..., 2:]) - torch.maximum(a[..., :2], b[..., :2])).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    union = area_a + area_b - inter
    iou = inter / union.clamp(min=1e-7)
    wh2 = (torch.maximum(a[..., 2:], b[..., 2:]) - torch.minimum(a[..., :2], b[..., :2])).clamp(min=0)
    area = wh2[..., 0] * wh2[..., 1]
    return iou - (area - union) / area.clamp(min=1e-7)


def masks_to_boxes(masks):
    """bool [..., H, W] -> normalised (cx, cy, w, h) [..., 4] of each mask's pixel bounds
    (the detectron2 gt_boxes of a polygon instance); empty masks give zeros.  On the
    device, no host sync."""
    H, W = masks.shape[-2:]
    rows, cols = masks.any(-1), masks.any(-2)
    ay = torch.arange(H, device=masks.device)
    ax = torch.arange(W, device=masks.device)
    y0 = torch.where(rows, ay, H).amin(-1).float()
    y1 = torch.where(rows, ay, -1).amax(-1).float() + 1
    x0 = torch.where(cols, ax, W).amin(-1).float()
    x1 = torch.where(cols, ax, -1).amax(-1).float() + 1
    ok = rows.any(-1)
    b = torch.stack(((x0 + x1) / (2 * W), (y0 + y1) / (2 * H), (x1 - x0) / W, (y1 - y0) / H), -1)
    return torch.where(ok[..., None], b, torch.zeros_like(b))


def sine_embed_boxes(boxes, d: int = 256):
    """DINO gen_sineembed_for_position: (cx, cy, w, h) -> [..., 2d] = cat(y, x, w, h)
    embeddings of d/2 features each (temperature 10000, scale 2 pi)."""
    n = d // 2
    dim_t = torch.arange(n, dtype=torch.float32, device=boxes.device)
    dim_t = 10000 ** (2 * torch.div(dim_t, 2, rounding_mode="floor") / n)
    out = []
    for i in (1, 0, 2, 3):
        p = boxes[..., i, None].float() * (2 * math.pi) / dim_t
        out.append(torch.stack((p[..., 0::2].sin(), p[..., 1::2].cos()), -1).flatten(-2))
    return torch.cat(out, -1)


class MLP(nn.Module):
    def __init__(self, din, dh, dout, n):
        super().__init__()
        dims = [din] + [dh] * (n - 1) + [dout]
        self.layers = nn.ModuleList(SmallLinear(a, b) for a, b in zip(dims[:-1], dims[1:]))

    def forward(self, x):
        for i, l in enumerate(self.layers):
            x = l(x)
            if i < len(self.layers) - 1:
                x = F.relu(x)
        return x


class DeformCrossAttn(nn.Module):
    """MSDeformAttn of the DINO decoder: queries [B, Q, d], reference BOXES [B, Q, 4]
    (normalised cxcywh, the same for every level): loc = c + off / P * wh / 2."""

    def __init__(self, d, heads, levels, points):
        super().__init__()
        self.d, self.heads, self.levels, self.points = d, heads, levels, points
        self.sampling_offsets = SmallLinear(d, heads * levels * points * 2)
        self.attention_weights = SmallLinear(d, heads * levels * points)
        self.value_proj = TokenLinear(d, d)
        self.output_proj = SmallLinear(d, d)

    def forward(self, query, boxes, memory, shapes):
        B, Q, _ = query.shape
        S = memory.shape[1]
        H, L, P = self.heads, self.levels, self.points
        value = self.value_proj(memory).view(B, S, H, self.d // H)
        off = self.sampling_offsets(query).view(B, Q, H, L, P, 2).float()
        aw = F.softmax(self.attention_weights(query).view(B, Q, H, L * P).float(), -1).view(B, Q, H, L, P)
        bx = boxes.float()[:, :, None, None, None, :]
        loc = bx[..., :2] + off / P * bx[..., 2:] * 0.5
        out = ops.ms_deform_attn(value, shapes, loc, aw)
        return self.output_proj(out)


class DINODecoderLayer(nn.Module):
    def __init__(self, d, ffn, heads, levels, points):
        super().__init__()
        self.heads = heads
        self.q_proj, self.k_proj, self.v_proj, self.out_proj = (SmallLinear(d, d) for _ in range(4))
        self.norm2 = TokenLayerNorm(d)
        self.cross_attn = DeformCrossAttn(d, heads, levels, points)
        self.norm1 = TokenLayerNorm(d)
        self.linear1 = SmallLinear(d, ffn)
        self.linear2 = SmallLinear(ffn, d)
        self.norm3 = TokenLayerNorm(d)

    def forward(self, tgt, qpos, boxes, memory, shapes, attn_words):
        B, Q, D = tgt.shape
        H, dh = self.heads, D // self.heads
        qk = tgt + qpos
        # attn_words: the DN-group mask as bitmask words [Q, ceil(Q/32)] (True = blocked), or None
        att = self_attention_core(self.q_proj(qk), self.k_proj(qk), self.v_proj(tgt), H, dh ** -0.5, attn_words)
        _, tgt = self.norm2.add_forward(tgt, self.out_proj(att))
        ca = self.cross_attn(tgt + qpos, boxes, memory, shapes)
        _, tgt = self.norm1.add_forward(tgt, ca)
        _, tgt = self.norm3.add_forward(tgt, self.linear2(F.relu(self.linear1(tgt))))
        return tgt


class MaskDINODecoder(nn.Module):
    def __init__(self, cfg: MaskDINOConfig):
        super().__init__()
        d = cfg.hidden_dim
        self.cfg = cfg
        self.enc_output = TokenLinear(d, d)
        self.enc_output_norm = TokenLayerNorm(d)
        self.class_embed = SmallLinear(d, cfg.num_labels)
        self.label_enc = nn.Embedding(cfg.num_labels, d)
        self.mask_embed = MLP(d, d, cfg.mask_feature_size, 3)
        self.bbox_embed = MLP(d, d, 4, 3)              # shared by the layers (upstream box_embed_layerlist)
        self.ref_point_head = MLP(2 * d, d, d, 2)
        self.decoder_norm = TokenLayerNorm(d)
        self.layers = nn.ModuleList(DINODecoderLayer(d, cfg.dec_ffn, cfg.dec_heads, cfg.n_levels, cfg.n_points)
                                    for _ in range(cfg.dec_layers))
        self._prop_cache = {}

    # ------------------------------------------------------------------ pieces
    def _proposals(self, shapes, device):
        """Anchor proposals per memory token (upstream gen_encoder_output_proposals, valid
        ratios 1): centre of the cell, w = h = 0.05 * 2^level, unsigmoided; tokens whose
        proposal leaves (0.01, 0.99) are invalid (memory zeroed, proposal +inf)."""
        key = (tuple(shapes), device)
        hit = self._prop_cache.get(key)
        if hit is None:
            props = []
            for lvl, (Hl, Wl) in enumerate(shapes):
                gy, gx = torch.meshgrid(torch.arange(Hl, dtype=torch.float32, device=device),
                                        torch.arange(Wl, dtype=torch.float32, device=device), indexing="ij")
                c = torch.stack(((gx.reshape(-1) + 0.5) / Wl, (gy.reshape(-1) + 0.5) / Hl), -1)
                wh = torch.full_like(c, 0.05 * 2.0 ** lvl)
                props.append(torch.cat((c, wh), -1))
            p = torch.cat(props, 0)
            valid = ((p > 0.01) & (p < 0.99)).all(-1)
            unsig = torch.log(p / (1 - p)).masked_fill(~valid[:, None], float("inf"))
            hit = self._prop_cache[key] = (unsig, valid)
        return hit

    def heads(self, out, mf, Hm, Wm, sink):
        """forward_prediction_heads: decoder_norm -> class logits, mask embedding -> mask
        logits (csrc/mask_head.hip)."""
        x = self.decoder_norm(out)
        cls = self.class_embed(x)
        e = self.mask_embed(x).to(mf.dtype)
        return cls, ops.mask_head(e, mf, Hm, Wm, sink=sink)

    def _dn(self, tg, boxes, B, dev, dtype):
        """Denoising queries (upstream prepare_for_dn).  With K = the batch's largest
        target count, dn_num // K groups of K slots: slot k of every group is target k of
        the image, slots past an image's count are padding queries (zero label embedding,
        zero unsigmoided box, as upstream); label flips with probability noise_scale/2,
        box jitter noise_scale * (wh/2, wh), clamped to [0, 1].

        K is read ON THE DEVICE (no host sync), so the layout depends only on the true
        counts, not on the capacity the targets are padded to: an eager step (capacity =
        K) and a graph-replayed one (capacity rounded up to a multiple of 4) build the same
        groups.  The query count is fixed at dn_num (>= groups x K for every K), so one
        captured graph serves every batch; queries past groups x K are inactive: each is a
        group of its own (no other query sees it) and every loss masks it out.

        Returns (label embeddings [B, dn_num, d], unsigmoided boxes [B, dn_num, 4],
        attention mask [Qt, Qt] (True = blocked), meta)."""
        c = self.cfg
        if tg.kc == 0 or c.dn_num <= 0:
            return None
        pad = c.dn_num
        counts = tg.counts.long()
        kmax = counts.max().clamp(min=1)                                           # device scalar
        groups = torch.div(pad, kmax, rounding_mode="floor")
        i = torch.arange(pad, device=dev)
        slot = i % kmax                                                            # < K <= capacity
        grp = torch.div(i, kmax, rounding_mode="floor")
        active = (grp < groups) & (counts.max() > 0)       # [pad]; no targets: no DN (upstream scalar 0)
        valid = active[None] & (slot[None] < counts[:, None])                      # [B, pad]
        labels = torch.gather(tg.classes, 1, slot[None].expand(B, pad))
        bx = torch.gather(boxes, 1, slot[None, :, None].expand(B, pad, 4))
        if c.noise_scale > 0:
            flip = torch.rand(B, pad, device=dev) < c.noise_scale * 0.5
            labels = torch.where(flip, torch.randint_like(labels, 0, c.num_labels), labels)
            diff = torch.cat((bx[..., 2:] / 2, bx[..., 2:]), -1)
            bx = (bx + (torch.rand_like(bx) * 2 - 1) * diff * c.noise_scale).clamp(0.0, 1.0)
        emb = self.label_enc(labels).to(dtype) * valid[..., None].to(dtype)
        unsig = torch.where(valid[..., None], inverse_sigmoid(bx), torch.zeros_like(bx))
        Qt = pad + c.num_queries
        g = torch.arange(Qt, device=dev)
        # group id: DN group, a private id for an inactive DN query, -1 for matching queries
        gid = torch.full((Qt,), -1, dtype=torch.long, device=dev)
        gid[:pad] = torch.where(active, grp, pad + i)
        dn_q = g < pad
        blocked = dn_q[:, None] & dn_q[None, :] & (gid[:, None] != gid[None, :])
        blocked |= ~dn_q[:, None] & dn_q[None, :]                          # matching queries cannot see DN
        return emb, unsig.to(dtype), blocked, dict(pad=pad, groups=groups, slot=slot, active=active, valid=valid)

    # ------------------------------------------------------------------ forward
    def forward(self, ms_feats, mask_features, targets=None, boxes=None):
        """ms_feats: [(tokens [B, HW, d], (H, W))] coarse to fine; mask_features [B, C,
        Hm, Wm]; targets: a criterion.PaddedTargets (+ their boxes [B, Kc, 4]) for the
        denoising queries during training.  Returns a dict of per-step lists (classes,
        masks, boxes), the two-stage "interm" predictions and the DN metadata."""
        c = self.cfg
        B, _, Hm, Wm = mask_features.shape
        dev = mask_features.device
        mf = mask_features.to(_compute_dtype(mask_features)).permute(0, 2, 3, 1).reshape(B, Hm * Wm, -1).contiguous()
        sink = ops.GradSink() if (mf.requires_grad and torch.is_grad_enabled() and mf.is_cuda) else None
        if sink is not None:
            mf = sink.source(mf)
        shapes = [hw for _, hw in ms_feats]
        memory = torch.cat([t for t, _ in ms_feats], 1)
        dtype = memory.dtype
        # ---- two-stage query selection
        unsig, valid = self._proposals(shapes, dev)
        out_mem = self.enc_output_norm(self.enc_output(memory * valid[None, :, None].to(dtype)))
        enc_cls = self.class_embed(out_mem)                                          # [B, S, K]
        enc_box = self.bbox_embed(out_mem).float() + unsig[None]
        score = enc_cls.float().amax(-1).masked_fill(~valid[None], float("-inf"))
        idx = score.topk(c.num_queries, dim=1)[1]                                    # [B, Nq]
        ref_undetach = torch.gather(enc_box, 1, idx[..., None].expand(-1, -1, 4))
        tgt_undetach = torch.gather(out_mem, 1, idx[..., None].expand(-1, -1, out_mem.shape[-1]))
        i_cls, i_mask = self.heads(tgt_undetach, mf, Hm, Wm, sink)
        interm = dict(classes=i_cls, masks=i_mask, boxes=ref_undetach.sigmoid())
        tgt = tgt_undetach.detach()
        ref_unsig = ref_undetach.detach()
        attn_words, dn = None, None
        if c.dn and self.training and targets is not None and targets.kc > 0:
            made = self._dn(targets, boxes, B, dev, dtype)
            if made is not None:
                emb, dn_unsig, blocked, dn = made
                tgt = torch.cat((emb, tgt), 1)
                ref_unsig = torch.cat((dn_unsig.float(), ref_unsig), 1)
                attn_words = ops.pack_blocked(blocked)                               # bit set = blocked
        # ---- initial prediction + decoder layers with iterative box refinement
        cls0, mask0 = self.heads(tgt, mf, Hm, Wm, sink)
        classes, masks = [cls0], [mask0]
        ref = ref_unsig.sigmoid()
        refs, hs = [ref], []
        out = tgt
        for layer in self.layers:
            qpos = self.ref_point_head(sine_embed_boxes(ref, c.hidden_dim).to(dtype))
            out = layer(out, qpos, ref, memory, shapes, attn_words)
            new_ref = (self.bbox_embed(out).float() + inverse_sigmoid(ref)).sigmoid()
            ref = new_ref.detach()
            refs.append(new_ref)
            hs.append(self.decoder_norm(out))
        for h in hs:                                   # upstream: decoder_norm again in the heads
            cl, mk = self.heads(h, mf, Hm, Wm, sink)
            classes.append(cl)
            masks.append(mk)
        # boxes (upstream pred_box): the initial reference, then each layer's refinement of
        # the reference it started from, on the normalised layer output
        boxes_out = [refs[0]] + [(self.bbox_embed(h).float() + inverse_sigmoid(r)).sigmoid()
                                 for h, r in zip(hs, refs[:-1])]
        return dict(classes=[x.float() for x in classes], masks=[m.float() for m in masks], boxes=boxes_out,
                    interm=dict(classes=interm["classes"].float(), masks=interm["masks"].float(),
                                boxes=interm["boxes"]), dn=dn)


class MaskDINO(nn.Module):
    """Swin + MaskDINO: forward(pixel_values, targets=None, boxes=None) -> the decoder's
    output dict (see MaskDINODecoder.forward)."""

    takes_targets = True           # Trainer: forward(images, PaddedTargets, boxes)

    def __init__(self, cfg: MaskDINOConfig):
        super().__init__()
        self.cfg = cfg
        self.backbone = SwinBackbone(cfg)
        chans = [cfg.embed_dim * 2 ** i for i in range(len(cfg.depths))]
        self.pixel_decoder = PixelDecoder(cfg, chans)
        self.decoder = MaskDINODecoder(cfg)

    def forward(self, pixel_values, targets=None, boxes=None):
        feats = self.backbone(pixel_values.to(self.backbone.patch_embed.proj.weight.dtype))
        mask_features, ms = self.pixel_decoder(feats)
        return self.decoder(ms, mask_features, targets, boxes)

    @torch.no_grad()
    def init_weights(self, seed: int = 0):
        """Upstream-style init: trunc-normal Linears, Deformable-DETR MSDA init (zero
        offset weights, offset biases on a per-head ring, zero attention weights), zero
        last layer of the box head (DINO), focal-loss prior on the class bias."""
        from .model import Mask2Former
        Mask2Former.init_weights(self, seed)        # Linear / LayerNorm / Embedding / encoder MSDA / Swin
        for m in self.modules():
            if isinstance(m, DeformCrossAttn):
                m.sampling_offsets.weight.zero_()
                th = torch.arange(m.heads, dtype=torch.float32) * (2.0 * math.pi / m.heads)
                grid = torch.stack([th.cos(), th.sin()], -1)
                grid = (grid / grid.abs().max(-1, keepdim=True)[0]).view(m.heads, 1, 1, 2).repeat(1, m.levels,
                                                                                                  m.points, 1)
                for i in range(m.points):
                    grid[:, :, i, :] *= i + 1
                m.sampling_offsets.bias.copy_(grid.view(-1))
                m.attention_weights.weight.zero_()
                m.attention_weights.bias.zero_()
        last = self.decoder.bbox_embed.layers[-1]
        last.weight.zero_()
        last.bias.zero_()
        self.decoder.class_embed.bias.fill_(-math.log((1 - 0.01) / 0.01))
        return self


# ----------------------------------------------------------------------------------
# Criterion (upstream MaskDINO criterion.py + matcher.py; parity unpinned)
# ----------------------------------------------------------------------------------


def sigmoid_focal_loss(logits, targets, alpha: float = 0.25, gamma: float = 2.0):
    """Element-wise DINO focal loss (alpha-balanced, gamma-modulated sigmoid CE)."""
    p = logits.sigmoid()
    ce = F.binary_cross_entropy_with_logits(logits, targets, reduction="none")
    p_t = p * targets + (1 - p) * (1 - targets)
    loss = ce * (1 - p_t) ** gamma
    return (alpha * targets + (1 - alpha) * (1 - targets)) * loss


def _point_sample(feat, coords):
    """feat [N, 1, H, W], coords [N, P, 2] in [0, 1] -> [N, P] (HF:m2f:245-275; ops.point_sample:
    the HIP point gather on the device)."""
    return ops.point_sample(feat, coords)


def _point_sample_rows(maps, rows, coords):
    """maps [M, H, W] f32, rows [N] int64 (which map each of N point sets reads), coords
    [N, P, 2] in [0, 1] -> [N, P]: `_point_sample(maps[rows][:, None], coords)` without
    materialising maps[rows] (grid_sample's bilinear rule, align_corners=False, zeros
    outside), one HIP thread per point (csrc/mask_head.hip point_sample_rows_kernel); host
    tensors (the CPU criterion tests) take the same rule as four gathers."""
    M, H, W = maps.shape
    if not maps.is_cuda:
        flat = maps.reshape(-1)
        g = 2.0 * coords - 1.0
        ix = ((g[..., 0] + 1) * W - 1) / 2
        iy = ((g[..., 1] + 1) * H - 1) / 2
        x0, y0 = torch.floor(ix), torch.floor(iy)
        x1, y1 = x0 + 1, y0 + 1
        base = (rows * (H * W))[:, None]
        out = torch.zeros_like(ix)
        for xx, yy, wgt in ((x0, y0, (x1 - ix) * (y1 - iy)), (x1, y0, (ix - x0) * (y1 - iy)),
                            (x0, y1, (x1 - ix) * (iy - y0)), (x1, y1, (ix - x0) * (iy - y0))):
            inside = (xx >= 0) & (xx <= W - 1) & (yy >= 0) & (yy <= H - 1)
            idx = base + (yy.clamp(0, H - 1).long() * W + xx.clamp(0, W - 1).long())
            out = out + torch.where(inside, flat[idx], 0.0) * wgt
        return out
    return ops.point_sample_rows(maps, rows, coords)


class MaskDINOCriterion:
    """Hungarian matching (focal class 4 + L1 box 5 + GIoU 2 + point-sampled mask BCE 5
    + dice 5) of every decoder step and of the two-stage selection, solved on the device
    (csrc/match.hip, no host sync); losses: focal class (x4), L1 (x5) and GIoU (x2) on
    matched boxes, point-sampled BCE (x5) and dice (x5) on matched masks, the same on the
    denoising queries against the targets they were made from.  Targets are
    criterion.PaddedTargets (+ boxes from masks_to_boxes).  Normalised by the global
    (all-reduced) mean target count, as upstream."""

    def __init__(self, cfg: MaskDINOConfig, matcher: str = "device", factor_losses: bool = True):
        self.cfg = cfg
        self.matcher = matcher
        self.num_masks_total = None
        # mask losses through the mask head's factors (ops.RowPointLogitsFunction) when the
        # logits carry them; False: autograd through the full logits (A/B, tests)
        self.factor_losses = factor_losses

    def _num_boxes(self, tg):
        import torch.distributed as dist
        if self.num_masks_total is not None:
            ws = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
            return torch.clamp(self.num_masks_total / ws, min=1)
        n = tg.counts.sum().float()
        ws = 1
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(n)
            ws = dist.get_world_size()
        return torch.clamp(n / ws, min=1)

    @torch.no_grad()
    def match(self, cls, box, masks, tg, tboxes, facs=None):
        """cls [S,B,Q,K], box [S,B,Q,4], masks S x [B,Q,H,W], targets (kc >= 1) ->
        int32 [S,B,Kc]: the query matched to each target (-1 past the image's count).
        facs: per step (E [B, Qt, C], P [B, HW, C], row offset of masks[s] in E, _) when
        the masks came from the mask head: the point-sampled mask costs are then computed
        from the factors (csrc/match_factors.hip, as the Mask2Former criterion does)."""
        c = self.cfg
        S, B, Q, _ = cls.shape
        Kc = tg.kc
        dev = cls.device
        p = cls.float().sigmoid()
        a, gam = c.focal_alpha, 2.0
        neg = (1 - a) * p ** gam * (-(1 - p + 1e-8).log())
        pos = a * (1 - p) ** gam * (-(p + 1e-8).log())
        idx = tg.classes[None, :, None, :].expand(S, B, Q, Kc)
        cost_class = torch.gather(pos, 3, idx) - torch.gather(neg, 3, idx)
        tb = tboxes[None].expand(S, B, Kc, 4).float()
        cost_box = torch.cdist(box.float(), tb, p=1)
        cost_giou = -generalized_box_iou(box_cxcywh_to_xyxy(box.float()), box_cxcywh_to_xyxy(tb))
        P = c.train_num_points
        grid = (2.0 * torch.rand(B, P, 2, device=dev) - 1.0).unsqueeze(2)
        tp = F.grid_sample(tg.masks.float(), grid, align_corners=False).squeeze(3)          # [B,Kc,P]
        H, W = masks[0].shape[-2:]
        if (facs is not None and all(f is not None for f in facs) and facs[0][1].dtype == torch.bfloat16
                and facs[0][0].shape[-1] in (64, 128, 256) and 1 <= Kc <= 16 and facs[0][1].shape[1] == H * W):
            # mask costs from E_s . F(p): F sampled once at the points, no logit map read
            E = torch.stack([f[0].detach()[:, f[2]:f[2] + Q] for f in facs]).contiguous()     # [S,B,Q,C]
            fp = ops.feature_sample_hilo(facs[0][1].detach(), H, W, grid.squeeze(2))
            zp = torch.zeros(S, B, Q, 1, device=dev)
            zc = torch.zeros(B, Kc, dtype=torch.int64, device=dev)
            cmask = ops.match_cost_factors(E, fp, zp, zc, tp, c.mask_weight, 0.0, c.dice_weight)
        else:
            pp = torch.stack([F.grid_sample(m.float(), grid, align_corners=False).squeeze(3) for m in masks])
            tpt = tp.transpose(1, 2)[None]
            cm = torch.matmul(F.softplus(-pp) / P, tpt) + torch.matmul(F.softplus(pp) / P, 1 - tpt)
            sg = pp.sigmoid()
            cd = 1 - (2 * torch.matmul(sg, tpt) + 1) / (sg.sum(-1)[..., None] + tp.sum(-1)[None, :, None, :] + 1)
            cmask = c.mask_weight * cm + c.dice_weight * cd
        cost = c.class_weight * cost_class + c.box_weight * cost_box + c.giou_weight * cost_giou + cmask
        cost = torch.nan_to_num(cost.clamp(-1e10, 1e10), 0.0)
        if self.matcher == "device" and cost.is_cuda and Kc <= ops.lsa_max_targets(Q):
            return ops.linear_sum_assignment_padded(cost, tg.counts)
        import numpy as np
        from scipy.optimize import linear_sum_assignment
        host, ks = cost.cpu().numpy(), tg.counts.cpu().tolist()
        out = np.full((S, B, Kc), -1, dtype=np.int32)
        for s in range(S):
            for b in range(B):
                if ks[b]:
                    r, col = linear_sum_assignment(host[s, b, :, :ks[b]])
                    out[s, b, col] = r
        return torch.from_numpy(out).to(dev)

    def _mask_losses(self, pred, tmask, slot, keep, nb, fac=None):
        """pred [B, R, H, W]: the logits of R queries per image; tmask [B, Kc, Ht, Wt] f32
        the targets; slot [B, R] the target slot each query is paired with; keep [B, R]
        bool.  Importance-sampled point BCE and dice (HF:m2f:671-724 semantics).  The
        labels: each query's own target (row b * Kc + slot of the flattened targets)
        sampled at that query's P points (`_point_sample_rows`: fixed shapes whatever the
        pairing, work and memory independent of Kc).  fac = (E [B, Q, C], P [B, HW, C],
        rows [B, R], sink): the logits came from the mask head and the loss differentiates
        through its factors on the R selected rows (ops.RowPointLogitsFunction)."""
        c = self.cfg
        B, R = slot.shape
        Kc = tmask.shape[1]
        N = B * R
        if fac is not None:
            # pred is None: the selected rows qrows of the head's full logits `full`
            E, Pf, qrows, sink, full = fac
            Esel = torch.gather(E, 1, qrows[..., None].expand(B, R, E.shape[-1]))
            Qt, H, W = full.shape[1:]
            flat = full.detach().reshape(-1, H, W)
            frows = (torch.arange(B, device=qrows.device)[:, None] * Qt + qrows).reshape(N)
        else:
            pred = pred.reshape(N, 1, *pred.shape[-2:])
        P = c.train_num_points
        dev = Esel.device if fac is not None else pred.device
        with torch.no_grad():
            ns, nu = int(P * c.oversample_ratio), int(c.importance_sample_ratio * P)
            coords = torch.rand(N, ns, 2, device=dev)
            if fac is not None:
                unc = -torch.abs(ops.point_sample_rows(flat, frows, coords))
            else:
                unc = -torch.abs(_point_sample(pred.detach().float(), coords))
            top = ops.topk_rows(unc, nu) if unc.is_cuda else torch.topk(unc, k=nu, dim=1)[1]
            coords = torch.gather(coords, 1, top[..., None].expand(-1, -1, 2))
            if P - nu > 0:
                coords = torch.cat([coords, torch.rand(N, P - nu, 2, device=dev)], 1)
            rows = (torch.arange(B, device=dev)[:, None] * Kc + slot.clamp(0, Kc - 1)).reshape(N)
            lab = _point_sample_rows(tmask.reshape(B * Kc, *tmask.shape[-2:]), rows, coords)
        if fac is not None:
            logit = ops.row_point_logits(flat, frows, coords, Esel, Pf, sink)
        else:
            logit = _point_sample(pred.float(), coords)
        keep = keep.reshape(N)
        zero = torch.zeros((), device=dev)
        bce = torch.where(keep, F.binary_cross_entropy_with_logits(logit, lab, reduction="none").mean(1), zero)
        pr = logit.sigmoid()
        dice = torch.where(keep, 1 - (2 * (pr * lab).sum(-1) + 1) / (pr.sum(-1) + lab.sum(-1) + 1), zero)
        return bce.sum() / nb, dice.sum() / nb

    def _mask_losses_steps(self, steps, tmask, slot, keep, norm):
        """_mask_losses of S prediction sets from the mask head's factors in one pass:
        steps = [(E [B, Qt, C], P, qrows [B, R], sink, full logits [B, Qt, H, W])] (one P and
        sink for all), slot [B, R] the target slot of each selected query (the same for
        every step), keep [S, B, R] bool, norm scalar or [S] -> (bce [S], dice [S]).  The
        points are drawn per step in the per-step order (oversampled, then the uniform
        remainder), so a step sees the draws _mask_losses would give it."""
        c = self.cfg
        S = len(steps)
        B, R = slot.shape
        Kc = tmask.shape[1]
        N = B * R
        P_f, sink = steps[0][1], steps[0][3]
        dev = slot.device
        flats, frows, esel = [], [], []
        for E, _, qrows, _, full in steps:
            Qt, H, W = full.shape[1:]
            flats.append(full.detach().reshape(-1, H, W))
            frows.append((torch.arange(B, device=dev)[:, None] * Qt + qrows).reshape(N))
            esel.append(torch.gather(E, 1, qrows[..., None].expand(B, R, E.shape[-1])))
        Esel = torch.stack(esel, 1).reshape(B, S * R, -1)                      # image-major, step-major rows
        Pn = c.train_num_points
        ns, nu = int(Pn * c.oversample_ratio), int(c.importance_sample_ratio * Pn)
        with torch.no_grad():
            over, rest = [], []
            for _ in range(S):
                over.append(torch.rand(N, ns, 2, device=dev))
                if Pn - nu > 0:
                    rest.append(torch.rand(N, Pn - nu, 2, device=dev))
            coords = torch.cat(over, 0)                                        # [S*N, ns, 2]
            unc = torch.cat([-torch.abs(ops.point_sample_rows(fl, fr, co)) for fl, fr, co in zip(flats, frows, over)])
            # one radix select over all S * N rows (torch.topk here sorts per step -- one call
            # over all rows is not capturable in a HIP graph -- ~6 ms of the C4 step)
            top = ops.topk_rows(unc, nu)
            coords = torch.gather(coords, 1, top[..., None].expand(-1, -1, 2))
            if rest:
                coords = torch.cat([coords, torch.cat(rest, 0)], 1)
            rows = (torch.arange(B, device=dev)[:, None] * Kc + slot.clamp(0, Kc - 1)).reshape(1, N).expand(S, N)
            lab = _point_sample_rows(tmask.reshape(B * Kc, *tmask.shape[-2:]), rows.reshape(S * N), coords)
        logit = ops.step_row_point_logits(flats, torch.stack(frows), coords, Esel, P_f, sink)
        keep = keep.reshape(S * N)
        zero = torch.zeros((), device=dev)
        bce = torch.where(keep, F.binary_cross_entropy_with_logits(logit, lab, reduction="none").mean(1), zero)
        pr = logit.sigmoid()
        dice = torch.where(keep, 1 - (2 * (pr * lab).sum(-1) + 1) / (pr.sum(-1) + lab.sum(-1) + 1), zero)
        return bce.view(S, N).sum(1) / norm, dice.view(S, N).sum(1) / norm

    def _pair_losses(self, cls, box, mask, qsel, valid, tg, tmf, tboxes, nb, fac=None):
        """Losses of one prediction set: cls [B,Q,K], box [B,Q,4], mask [B,Q,H,W]; qsel
        [B,Kc] the query paired with each target slot, valid [B,Kc]; tmf the target masks
        in f32; fac: (E, P, query offset of mask's rows in E, sink) when mask came from the
        mask head (see _mask_losses)."""
        c = self.cfg
        B, Q, K = cls.shape
        Kc = tg.kc
        onehot = torch.zeros(B, Q + 1, K, device=cls.device, dtype=cls.dtype)
        qi = torch.where(valid, qsel, torch.full_like(qsel, Q))
        onehot.scatter_(1, qi[..., None].expand(B, Kc, K),
                        F.one_hot(tg.classes, K).to(cls.dtype) * valid[..., None].to(cls.dtype))
        l_cls = sigmoid_focal_loss(cls, onehot[:, :Q], c.focal_alpha).sum() / nb
        bidx = torch.arange(B, device=cls.device)[:, None].expand(B, Kc)
        qs = qsel.clamp(0, Q - 1)
        pb = box[bidx, qs].float()                                                    # [B,Kc,4]
        tb = tboxes.float()
        v = valid.float()
        l_l1 = ((pb - tb).abs().sum(-1) * v).sum() / nb
        giou = torch.diagonal(generalized_box_iou(box_cxcywh_to_xyxy(pb), box_cxcywh_to_xyxy(tb)), dim1=-2, dim2=-1)
        l_giou = ((1 - giou) * v).sum() / nb
        slots = torch.arange(Kc, device=cls.device)[None].expand(B, Kc)
        if fac is not None:     # the selected rows are read from the full logits
            pm, mfac = None, (fac[0], fac[1], qs + fac[2], fac[3], fac[4])
        else:
            pm, mfac = mask[bidx, qs], None                                           # [B,Kc,H,W]
        l_bce, l_dice = self._mask_losses(pm, tmf, slots, valid, nb, mfac)
        return dict(loss_ce=c.class_weight * l_cls, loss_bbox=c.box_weight * l_l1, loss_giou=c.giou_weight * l_giou,
                    loss_mask=c.mask_weight * l_bce, loss_dice=c.dice_weight * l_dice)

    def _cls_box_losses(self, cls, box, qsel, valid, tcls, tboxes, norm):
        """Focal class, L1 and GIoU losses of S prediction sets at once (one launch per op
        for all decoder steps instead of one per step): cls [S,B,Q,K], box [S,B,Q,4]; qsel
        [S,B,R] the query paired with each of R targets (tcls [B,R] classes, tboxes [B,R,4]),
        valid [S,B,R]; norm: scalar or [S].  -> (l_cls, l_l1, l_giou) each [S] (unweighted)."""
        c = self.cfg
        S, B, Q, K = cls.shape
        R = qsel.shape[-1]
        onehot = torch.zeros(S, B, Q + 1, K, device=cls.device, dtype=cls.dtype)
        qi = torch.where(valid, qsel, torch.full_like(qsel, Q))
        onehot.scatter_(2, qi[..., None].expand(S, B, R, K),
                        F.one_hot(tcls, K).to(cls.dtype)[None].expand(S, B, R, K) * valid[..., None].to(cls.dtype))
        l_cls = sigmoid_focal_loss(cls, onehot[:, :, :Q], c.focal_alpha).sum((1, 2, 3)) / norm
        qs = qsel.clamp(0, Q - 1)
        pb = torch.gather(box, 2, qs[..., None].expand(S, B, R, 4)).float()
        tb = tboxes.float()[None]
        v = valid.float()
        l_l1 = ((pb - tb).abs().sum(-1) * v).sum((1, 2)) / norm
        giou = paired_giou(box_cxcywh_to_xyxy(pb), box_cxcywh_to_xyxy(tb))
        l_giou = ((1 - giou) * v).sum((1, 2)) / norm
        return l_cls, l_l1, l_giou

    def _dn_losses(self, cls, box, mask, dn, tg, tmf, tboxes, nb, fac=None):
        """Denoising queries against the targets they were made from: DN query i <->
        target slot dn["slot"][i] (valid where its group is active and the image has that
        target); normalised by the target count x the number of groups (upstream
        num_boxes * scalar).  The class loss covers the active DN queries (upstream: the
        first groups x K queries, padding slots as negatives)."""
        c = self.cfg
        pad, slot, valid, active = dn["pad"], dn["slot"], dn["valid"], dn["active"]
        B, _, K = cls.shape
        nbg = nb * dn["groups"].clamp(min=1).float()
        sl = slot[None].expand(B, pad)
        tcls = torch.gather(tg.classes, 1, sl)
        onehot = F.one_hot(tcls, K).to(cls.dtype) * valid[..., None].to(cls.dtype)
        focal = sigmoid_focal_loss(cls[:, :pad], onehot, c.focal_alpha)
        l_cls = (focal * active[None, :, None].to(focal.dtype)).sum() / nbg
        pb, v = box[:, :pad].float(), valid.float()
        tb = torch.gather(tboxes.float(), 1, sl[..., None].expand(B, pad, 4))
        l_l1 = ((pb - tb).abs().sum(-1) * v).sum() / nbg
        giou = torch.diagonal(generalized_box_iou(box_cxcywh_to_xyxy(pb), box_cxcywh_to_xyxy(tb)), dim1=-2, dim2=-1)
        l_giou = ((1 - giou) * v).sum() / nbg
        if fac is not None:
            rows = torch.arange(pad, device=cls.device)[None].expand(B, pad)
            l_bce, l_dice = self._mask_losses(None, tmf, sl, valid, nbg, (fac[0], fac[1], rows, fac[3], fac[4]))
        else:
            l_bce, l_dice = self._mask_losses(mask[:, :pad], tmf, sl, valid, nbg)
        return dict(loss_ce=c.class_weight * l_cls, loss_bbox=c.box_weight * l_l1, loss_giou=c.giou_weight * l_giou,
                    loss_mask=c.mask_weight * l_bce, loss_dice=c.dice_weight * l_dice)

    def __call__(self, out, targets, boxes):
        """out: MaskDINO.forward output; targets: PaddedTargets; boxes [B, Kc, 4] ->
        (total loss, dict of weighted components: final step un-suffixed, aux steps
        `_{i}`, two-stage `_interm`, denoising `_dn` / `_dn_{i}`)."""
        tg = targets
        dn = out["dn"]
        pad = dn["pad"] if dn else 0
        S = len(out["classes"])
        cls_m = torch.stack([x[:, pad:] for x in out["classes"]] + [out["interm"]["classes"]])
        box_m = torch.stack([x[:, pad:] for x in out["boxes"]] + [out["interm"]["boxes"]])
        masks_m = [x[:, pad:] for x in out["masks"]] + [out["interm"]["masks"]]
        nb = self._num_boxes(tg)
        losses = {}
        names = [("" if s == S - 1 else f"_{s}") for s in range(S)] + ["_interm"]
        if tg.kc == 0:
            zero = sum(x.sum() for x in out["classes"]) * 0.0
            total = zero
            for s, nm in enumerate(names):
                B, Q, K = cls_m[s].shape
                l = self.cfg.class_weight * sigmoid_focal_loss(cls_m[s], torch.zeros_like(cls_m[s])).sum() / nb
                losses[f"loss_ce{nm}"] = l
                total = total + l
            return total, losses
        # the mask head's factors of every step (E, P), when the logits came from it with one
        # shared pixel embedding: the matcher's mask costs and the mask losses then use the
        # factors (the losses differentiate through the selected rows only; P goes through
        # one GradSink so the calls sum dP in place)
        srcs = [getattr(m, "_vs_src", None) for m in out["masks"]] + [getattr(out["interm"]["masks"], "_vs_src", None)]
        facs = [None] * len(srcs)
        if (self.factor_losses and all(sr is not None for sr in srcs) and all(sr[1] is srcs[0][1] for sr in srcs)
                and srcs[0][1].is_cuda):
            sink = ops.GradSink() if torch.is_grad_enabled() else None
            P = sink.source(srcs[0][1]) if sink is not None else srcs[0][1]
            fulls = out["masks"] + [out["interm"]["masks"]]
            facs = [(sr[0], P, pad if i < S else 0, sink, fulls[i]) for i, sr in enumerate(srcs)]
        assign = self.match(cls_m.detach(), box_m.detach(), [m.detach() for m in masks_m], tg, boxes,
                            facs if facs[0] is not None else None)
        valid = tg.valid()
        tmf = tg.masks.float()                         # the targets as f32 once per step
        c = self.cfg
        Kc = tg.kc
        qsel = assign.long()
        vs = valid[None] & (assign >= 0)                                               # [S+1,B,Kc]
        l_cls, l_l1, l_giou = self._cls_box_losses(cls_m, box_m, qsel, vs, tg.classes, boxes, nb)
        B = cls_m.shape[1]
        slots = torch.arange(Kc, device=cls_m.device)[None].expand(B, Kc)
        if facs[0] is not None:         # the selected rows of every step, read from the full logits
            steps = [(f[0], f[1], qsel[s].clamp(0, masks_m[s].shape[1] - 1) + f[2], f[3], f[4])
                     for s, f in enumerate(facs)]
            m_bce, m_dice = self._mask_losses_steps(steps, tmf, slots, vs, nb)
        for s, nm in enumerate(names):
            if facs[0] is not None:
                l_bce, l_dice = m_bce[s], m_dice[s]
            else:
                bidx = torch.arange(B, device=cls_m.device)[:, None].expand(B, Kc)
                pm = masks_m[s][bidx, qsel[s].clamp(0, masks_m[s].shape[1] - 1)]
                l_bce, l_dice = self._mask_losses(pm, tmf, slots, vs[s], nb)
            losses.update({"loss_ce" + nm: c.class_weight * l_cls[s], "loss_bbox" + nm: c.box_weight * l_l1[s],
                           "loss_giou" + nm: c.giou_weight * l_giou[s], "loss_mask" + nm: c.mask_weight * l_bce,
                           "loss_dice" + nm: c.dice_weight * l_dice})
        if dn:
            pad, slot, dvalid, active = dn["pad"], dn["slot"], dn["valid"], dn["active"]
            nbg = nb * dn["groups"].clamp(min=1).float()
            sl = slot[None].expand(B, pad)
            tcls = torch.gather(tg.classes, 1, sl)
            K = cls_m.shape[-1]
            cls_d = torch.stack([x[:, :pad] for x in out["classes"]])                   # [S,B,pad,K]
            box_d = torch.stack([x[:, :pad] for x in out["boxes"]]).float()
            # class loss over the active DN queries (padding slots as negatives), L1 / GIoU
            # on the valid ones: DN query i <-> target slot slot[i]
            onehot = F.one_hot(tcls, K).to(cls_d.dtype) * dvalid[..., None].to(cls_d.dtype)
            focal = sigmoid_focal_loss(cls_d, onehot[None].expand_as(cls_d), c.focal_alpha)
            d_cls = (focal * active[None, None, :, None].to(focal.dtype)).sum((1, 2, 3)) / nbg
            tb = torch.gather(boxes.float(), 1, sl[..., None].expand(B, pad, 4))[None]
            v = dvalid.float()[None]
            d_l1 = ((box_d - tb).abs().sum(-1) * v).sum((1, 2)) / nbg
            d_giou = ((1 - paired_giou(box_cxcywh_to_xyxy(box_d), box_cxcywh_to_xyxy(tb))) * v).sum((1, 2)) / nbg
            rows = torch.arange(pad, device=cls_m.device)[None].expand(B, pad)
            if facs[0] is not None:
                steps = [(facs[s][0], facs[s][1], rows, facs[s][3], facs[s][4]) for s in range(S)]
                d_bce, d_dice = self._mask_losses_steps(steps, tmf, sl, dvalid[None].expand(S, B, pad), nbg)
            for s in range(S):
                if facs[0] is not None:
                    l_bce, l_dice = d_bce[s], d_dice[s]
                else:
                    l_bce, l_dice = self._mask_losses(out["masks"][s][:, :pad], tmf, sl, dvalid, nbg)
                nm = "_dn" if s == S - 1 else f"_dn_{s}"
                losses.update({"loss_ce" + nm: c.class_weight * d_cls[s], "loss_bbox" + nm: c.box_weight * d_l1[s],
                               "loss_giou" + nm: c.giou_weight * d_giou[s], "loss_mask" + nm: c.mask_weight * l_bce,
                               "loss_dice" + nm: c.dice_weight * l_dice})
        total = sum(losses.values())
        return total, losses
