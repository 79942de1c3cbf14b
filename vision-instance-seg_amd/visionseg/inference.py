"""Inference seam for labeling_server/ai_segmentation.py (`AISegmentationModel`).

The reference's predictor calls `mmdet.apis.init_detector(config, checkpoint, device)`
and `inference_detector(model, image)` and reads `result.pred_instances.{scores,
masks, labels}` (labeling_server/ai_segmentation.py:41-50, 70-97).  This module
provides the same two functions and result shape on top of the MI355X model, so the
caller swaps one import and keeps its own top-score selection,
thresholding and polygon extraction unchanged.

Post-processing follows Mask2Former's instance inference (upstream `instance_inference`;
in-container oracle HF:m2f-proc:627-746): per image, class scores softmax[:, :-1],
top-k over queries x classes, binary mask = mask logit > 0 at image resolution, final
score = class score x mean foreground probability inside the binary mask.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

from .data import PIXEL_MEAN, PIXEL_STD
from .model import M2FConfig, Mask2Former


@dataclass
class InstanceData:
    """The subset of mmengine's InstanceData the caller reads."""
    scores: torch.Tensor     # [N] float
    masks: torch.Tensor      # [N, H, W] bool (original image size)
    labels: torch.Tensor     # [N] int64

    def __len__(self):
        return int(self.scores.shape[0])


@dataclass
class DetResult:
    pred_instances: InstanceData


@torch.no_grad()
def instance_inference(mask_logits, class_logits, out_hw, valid_hw=None, pad_hw=None, top_k: int | None = None,
                       sigmoid_classes: bool = False):
    """mask_logits [Q,h,w], class_logits [Q,K+1] -> (scores [k], labels [k], masks bool [k,H,W]).

    Scores and binary masks as HF:m2f-proc:695-709 (softmax over classes without the
    no-object column, top-k over queries x classes, mask = logit > 0, score x mean
    foreground probability inside the mask); pinned by tests/golden/postproc.npz.
    Resizing as upstream sem_seg_postprocess (detectron2): with `pad_hw` / `valid_hw`
    the logits are first upsampled to the padded input size, cropped to the valid
    (un-padded) region, then resized to `out_hw` -- bilinear, align_corners=False.
    sigmoid_classes: MaskDINO's scoring (focal-loss classes, no no-object column: class
    scores = sigmoid(logits) over all K columns; upstream MaskDINO instance_inference, not
    in the container -- parity unpinned), the rest as above."""
    Q, K1 = class_logits.shape
    if sigmoid_classes:
        K = K1
        scores = class_logits.float().sigmoid()
    else:
        K = K1 - 1
        scores = F.softmax(class_logits.float(), -1)[:, :-1]
    labels = torch.arange(K, device=scores.device).unsqueeze(0).repeat(Q, 1).flatten(0, 1)
    k = top_k or Q
    sc, idx = scores.flatten(0, 1).topk(min(k, Q * K), sorted=False)
    lab = labels[idx]
    qi = torch.div(idx, K, rounding_mode="floor")
    m = mask_logits[qi].float()[None]
    if pad_hw is not None:
        m = F.interpolate(m, size=tuple(pad_hw), mode="bilinear", align_corners=False)
    if valid_hw is not None:
        m = m[..., : valid_hw[0], : valid_hw[1]]
    if tuple(m.shape[-2:]) != tuple(out_hw):
        m = F.interpolate(m, size=tuple(out_hw), mode="bilinear", align_corners=False)
    m = m[0]
    binm = m > 0
    prob = m.sigmoid()
    mscore = (prob * binm).flatten(1).sum(1) / (binm.flatten(1).sum(1) + 1e-6)
    return sc * mscore, lab, binm


class Predictor:
    """Swin + Mask2Former (or MaskDINO) predictor on the MI355X kernels, eval mode.

    On a HIP device with `amp` the model runs the training step's production path: bf16
    parameters and activations (the fused kernels need matching dtypes; autocast would
    leave them), and each padded input shape is captured once as a HIP graph and
    replayed (`graphs`; the eager forward is ~1 000 host launches).  A small LRU keeps
    the graphs of the last `max_graphs` shapes (the preprocessing pads to multiples of
    32, so a labelling session sees a handful of shapes).  Without a device, or with
    graphs off, the forward runs eagerly (f32 autocast-free on CPU)."""

    def __init__(self, model: Mask2Former, device="cuda:0", min_size: int = 640, max_size: int = 800,
                 amp: bool = True, top_k: int = 100, graphs: bool = True, max_graphs: int = 4):
        self.device = torch.device(device)
        self.bf16 = bool(amp) and self.device.type == "cuda"
        if self.device.type == "cuda":
            # MIOpen Find (as the Trainer): without it MIOpen's immediate mode ran a fallback
            # solver on the FIRST call of a convolution shape and another afterwards, so the
            # first forward of a shape differed from every later one -- and from its graph
            # capture (tools/det_debug.py: pixel_decoder.input_proj.0.conv)
            torch.backends.cudnn.benchmark = True
        if self.bf16 and next(model.parameters()).dtype != torch.bfloat16:
            # a bf16 copy: the caller's model (e.g. an f32 Trainer's, whose parameters are
            # views of its flat buffers) is left as it is
            import copy
            model = copy.deepcopy(model).to(torch.bfloat16)
        self.model = model.to(self.device).eval()
        self.min_size, self.max_size, self.amp, self.top_k = min_size, max_size, amp, top_k
        from .train import graph_capture_safe
        self.graphs = bool(graphs) and self.bf16 and graph_capture_safe()
        self.max_graphs = int(max_graphs)
        self._graphs = {}                     # padded input shape -> (graph, static input, static outputs)

    def _forward(self, x):
        if not self.graphs:
            return self.model(x)
        key = tuple(x.shape)
        hit = self._graphs.pop(key, None)
        if hit is None:
            self.model(x)                     # lazy library state before the capture
            torch.cuda.synchronize(self.device)
            while len(self._graphs) >= self.max_graphs:      # oldest shape out
                old = self._graphs.pop(next(iter(self._graphs)))
                old[0].reset()
            g = torch.cuda.CUDAGraph()
            static = x.clone()
            with torch.cuda.graph(g):
                out = self.model(static)
            from .model import cached_constants
            hit = (g, static, out, cached_constants())   # constants the graph reads stay alive
        self._graphs[key] = hit               # most recently used last
        g, static, out = hit[:3]
        static.copy_(x)
        g.replay()
        return out

    def _preprocess(self, image_bgr: np.ndarray):
        h, w = image_bgr.shape[:2]
        s = self.min_size / min(h, w)
        if max(h, w) * s > self.max_size:
            s = self.max_size / max(h, w)
        nh, nw = int(round(h * s)), int(round(w * s))
        rgb = torch.from_numpy(np.ascontiguousarray(image_bgr[:, :, ::-1])).to(self.device)
        x = rgb.permute(2, 0, 1).float()[None]
        x = F.interpolate(x, size=(nh, nw), mode="bilinear", align_corners=False)
        x = (x - torch.tensor(PIXEL_MEAN, device=self.device).view(1, 3, 1, 1)) / \
            torch.tensor(PIXEL_STD, device=self.device).view(1, 3, 1, 1)
        ph, pw = (nh + 31) // 32 * 32, (nw + 31) // 32 * 32
        x = F.pad(x, (0, pw - nw, 0, ph - nh))
        return x, (nh, nw), (h, w)

    @torch.no_grad()
    def __call__(self, image_bgr: np.ndarray) -> DetResult:
        x, valid, orig = self._preprocess(image_bgr)
        out = self._forward(x.to(torch.bfloat16) if self.bf16 else x)
        if isinstance(out, dict):            # MaskDINO: per-step lists in a dict, sigmoid class scores
            m, c, sig = out["masks"][-1][0], out["classes"][-1][0], True
        else:
            m, c, sig = out[0][-1][0], out[1][-1][0], False
        # stride-4 logits -> padded input size -> crop the valid region -> original size
        scores, labels, binm = instance_inference(m, c, orig, valid_hw=valid, pad_hw=tuple(x.shape[-2:]),
                                                  top_k=self.top_k, sigmoid_classes=sig)
        return DetResult(InstanceData(scores=scores, masks=binm, labels=labels))


def load_checkpoint(path: str, device="cpu") -> dict:
    """Trainer.save() checkpoints ({'model': sd, ...}) or bare state dicts, in the build's
    or the HF layout (converted).  Safe loader only (weights_only=True)."""
    from .convert import from_hf_state_dict
    sd = torch.load(path, map_location=device, weights_only=True)
    if isinstance(sd, dict) and "model" in sd and isinstance(sd["model"], dict):
        sd = sd["model"]
    if any(k.startswith("model.pixel_level_module.") for k in sd):
        sd = from_hf_state_dict(sd)
    return sd


def backbone_from_state_dict(sd: dict) -> dict:
    """Swin backbone hyper-parameters (embed_dim, depths, num_heads, window_size) read off a
    checkpoint's backbone tensors: patch-embedding width, blocks per stage, and the
    relative-position tables [(2ws-1)^2, heads] of each stage."""
    import math
    import re
    embed = int(sd["backbone.patch_embed.proj.weight"].shape[0])
    blocks, heads, ws = {}, {}, None
    for k, v in sd.items():
        mt = re.match(r"backbone\.stages\.(\d+)\.blocks\.(\d+)\.attn\.rel_table$", k)
        if mt:
            i, j = int(mt.group(1)), int(mt.group(2))
            blocks[i] = max(blocks.get(i, 0), j + 1)
            heads[i] = int(v.shape[1])
            ws = (int(round(math.sqrt(v.shape[0]))) + 1) // 2
    n = len(blocks)
    if not n or sorted(blocks) != list(range(n)):
        raise ValueError("the checkpoint's backbone stages could not be read")
    return dict(embed_dim=embed, depths=tuple(blocks[i] for i in range(n)),
                num_heads=tuple(heads[i] for i in range(n)), window_size=ws)


def init_detector(config, checkpoint: str | None = None, device: str = "cuda:0") -> Predictor:
    """mmdet.apis.init_detector-compatible entry (ai_segmentation.py:41-50).
    `config`: an M2FConfig / MaskDINOConfig, a preset name ("swin_t", "swin_b", ...;
    "maskdino_swin_t" ... for MaskDINO), or a JSON file (a config dict, or {"preset":
    name}).  A MaskDINO checkpoint (train_maskdino's) is recognised by its keys; its
    backbone comes from the config when one is given, else from the checkpoint's own
    backbone tensors (an explicit error when neither can be read)."""
    from .maskdino import MaskDINO, MaskDINOConfig
    sd = load_checkpoint(checkpoint) if checkpoint else None
    name = config if isinstance(config, str) and not os.path.exists(config) else None
    given = None                                    # a config dict from the argument / JSON file
    if isinstance(config, M2FConfig):
        given = config.to_dict()
    elif isinstance(config, str) and os.path.exists(config):
        with open(config) as f:
            given = json.load(f)
        if set(given) == {"preset"}:
            name, given = given["preset"], None
    maskdino = isinstance(config, MaskDINOConfig) or bool(name and name.startswith("maskdino")) or bool(
        sd is not None and any(k.startswith("decoder.enc_output.") for k in sd))
    if maskdino:
        if given is not None:
            cfg = MaskDINOConfig.from_dict(given)
        elif name:
            cfg = MaskDINOConfig.preset(name.replace("maskdino_", "") or "swin_t")
        elif sd is not None:
            cfg = MaskDINOConfig.from_dict(backbone_from_state_dict(sd))
        else:
            cfg = MaskDINOConfig.preset("swin_t")
        if sd is not None and "decoder.class_embed.weight" in sd:
            cfg.num_labels = int(sd["decoder.class_embed.weight"].shape[0])
        model = MaskDINO(cfg)
    else:
        if given is not None:
            cfg = M2FConfig.from_dict(given)
        else:
            cfg = M2FConfig.preset(name or "swin_t")
        model = Mask2Former(cfg)
    if sd is not None:
        model.load_state_dict(sd)
    else:
        model.init_weights()
    return Predictor(model, device=device)


def inference_detector(model: Predictor, image: np.ndarray) -> DetResult:
    """mmdet.apis.inference_detector-compatible entry (ai_segmentation.py:74-77)."""
    return model(image)
