"""State-dict conversion between the HF/upstream Mask2Former layout and this build's.

Users coming from `Mask2FormerForUniversalSegmentation` (HF:m2f:2278) checkpoints, or
from the upstream Mask2Former/detectron2 module tree it mirrors, load them with
`from_hf_state_dict`.  The build's layout differs in three places, all for the
kernels' sake:

* Swin attention q/k/v Linears are fused into one `qkv` Linear (rows q;k;v), so the
  window-attention kernel reads one [tokens, 3C] projection (HF:swin:411-414).
* Module paths are flattened (`backbone.stages.{s}.blocks.{b}...`).
* The pixel decoder's FPN adapter/layer (`adapter_1`/`layer_1`, HF:m2f:1294-1297)
  become `lateral`/`output`.

Pure tensor-dict manipulation: no device work, importable without a GPU.
"""
from __future__ import annotations

import re

import torch

_HF_BB = "model.pixel_level_module.encoder."
_HF_PD = "model.pixel_level_module.decoder."
_HF_TM = "model.transformer_module."


def from_hf_state_dict(sd: dict) -> dict:
    """HF Mask2FormerForUniversalSegmentation state dict -> build layout."""
    out = {}
    qkv = {}
    for k, v in sd.items():
        if k.startswith("criterion.") or k.endswith("relative_position_index"):
            continue
        if k.startswith(_HF_BB + "swin.layernorm."):
            continue  # SwinModel's final norm is unused by the backbone (HF:swin:1131-1138)
        m = re.match(re.escape(_HF_BB) + r"swin\.embeddings\.patch_embeddings\.projection\.(weight|bias)", k)
        if m:
            out[f"backbone.patch_embed.proj.{m[1]}"] = v
            continue
        m = re.match(re.escape(_HF_BB) + r"swin\.embeddings\.norm\.(weight|bias)", k)
        if m:
            out[f"backbone.patch_embed.norm.{m[1]}"] = v
            continue
        m = re.match(re.escape(_HF_BB) + r"swin\.encoder\.layers\.(\d+)\.blocks\.(\d+)\.(.*)", k)
        if m:
            s, b, rest = m[1], m[2], m[3]
            pre = f"backbone.stages.{s}.blocks.{b}."
            mm = re.match(r"attention\.(q|k|v)_proj\.(weight|bias)", rest)
            if mm:
                qkv.setdefault((pre, mm[2]), {})[mm[1]] = v
                continue
            rest = (rest.replace("layernorm_before", "norm1").replace("layernorm_after", "norm2")
                    .replace("attention.o_proj", "attn.proj")
                    .replace("attention.relative_position_bias.relative_position_bias_table", "attn.rel_table"))
            out[pre + rest] = v
            continue
        m = re.match(re.escape(_HF_BB) + r"swin\.encoder\.layers\.(\d+)\.downsample\.(norm|reduction)\.(weight|bias)", k)
        if m:
            out[f"backbone.stages.{m[1]}.merge.{m[2]}.{m[3]}"] = v
            continue
        m = re.match(re.escape(_HF_BB) + r"hidden_states_norms\.stage(\d+)\.(weight|bias)", k)
        if m:
            out[f"backbone.out_norms.{int(m[1]) - 1}.{m[2]}"] = v
            continue
        if k.startswith(_HF_PD):
            r = k[len(_HF_PD):]
            r = re.sub(r"^input_projections\.(\d+)\.0\.", r"input_proj.\1.conv.", r)
            r = re.sub(r"^input_projections\.(\d+)\.1\.", r"input_proj.\1.gn.", r)
            r = re.sub(r"^adapter_1\.0\.", "lateral.conv.", r)
            r = re.sub(r"^adapter_1\.1\.", "lateral.gn.", r)
            r = re.sub(r"^layer_1\.0\.", "output.conv.", r)
            r = re.sub(r"^layer_1\.1\.", "output.gn.", r)
            r = re.sub(r"^mask_projection\.", "mask_proj.", r)
            r = re.sub(r"^encoder\.layers\.(\d+)\.self_attn\.", r"encoder.\1.attn.", r)
            r = re.sub(r"^encoder\.layers\.(\d+)\.self_attn_layer_norm\.", r"encoder.\1.norm1.", r)
            r = re.sub(r"^encoder\.layers\.(\d+)\.final_layer_norm\.", r"encoder.\1.norm2.", r)
            r = re.sub(r"^encoder\.layers\.(\d+)\.(fc\d)\.", r"encoder.\1.\2.", r)
            out["pixel_decoder." + r] = v
            continue
        if k.startswith(_HF_TM):
            r = k[len(_HF_TM):]
            r = r.replace("queries_embedder", "query_embed").replace("queries_features", "query_feat")
            r = re.sub(r"^decoder\.layers\.", "layers.", r)
            r = re.sub(r"^decoder\.layernorm\.", "norm.", r)
            r = re.sub(r"^decoder\.mask_predictor\.mask_embedder\.(\d)\.0\.", r"mask_embed.\1.", r)
            r = r.replace("cross_attn_layer_norm", "norm_cross").replace("self_attn_layer_norm", "norm_self")
            r = r.replace("final_layer_norm", "norm_ffn")
            out["decoder." + r] = v
            continue
        if k.startswith("class_predictor."):
            out["class_head." + k.split(".", 1)[1]] = v
            continue
        raise KeyError(f"unmapped HF key {k}")
    for (pre, kind), d in qkv.items():
        out[pre + f"attn.qkv.{kind}"] = torch.cat([d["q"], d["k"], d["v"]], 0)
    return out


def to_hf_state_dict(sd: dict, num_labels: int = 1, no_object_weight: float = 0.1) -> dict:
    """Inverse of `from_hf_state_dict` (build layout -> HF layout)."""
    out = {}
    for k, v in sd.items():
        m = re.match(r"backbone\.patch_embed\.proj\.(weight|bias)", k)
        if m:
            out[_HF_BB + f"swin.embeddings.patch_embeddings.projection.{m[1]}"] = v
            continue
        m = re.match(r"backbone\.patch_embed\.norm\.(weight|bias)", k)
        if m:
            out[_HF_BB + f"swin.embeddings.norm.{m[1]}"] = v
            continue
        m = re.match(r"backbone\.stages\.(\d+)\.blocks\.(\d+)\.(.*)", k)
        if m:
            pre = _HF_BB + f"swin.encoder.layers.{m[1]}.blocks.{m[2]}."
            rest = m[3]
            mm = re.match(r"attn\.qkv\.(weight|bias)", rest)
            if mm:
                q, kk, vv = v.chunk(3, 0)
                for n, t in (("q", q), ("k", kk), ("v", vv)):
                    out[pre + f"attention.{n}_proj.{mm[1]}"] = t.contiguous()
                continue
            rest = (rest.replace("norm1", "layernorm_before").replace("norm2", "layernorm_after")
                    .replace("attn.proj", "attention.o_proj")
                    .replace("attn.rel_table", "attention.relative_position_bias.relative_position_bias_table"))
            out[pre + rest] = v
            continue
        m = re.match(r"backbone\.stages\.(\d+)\.merge\.(norm|reduction)\.(weight|bias)", k)
        if m:
            out[_HF_BB + f"swin.encoder.layers.{m[1]}.downsample.{m[2]}.{m[3]}"] = v
            continue
        m = re.match(r"backbone\.out_norms\.(\d+)\.(weight|bias)", k)
        if m:
            out[_HF_BB + f"hidden_states_norms.stage{int(m[1]) + 1}.{m[2]}"] = v
            continue
        if k.startswith("pixel_decoder."):
            r = k[len("pixel_decoder."):]
            r = re.sub(r"^input_proj\.(\d+)\.conv\.", r"input_projections.\1.0.", r)
            r = re.sub(r"^input_proj\.(\d+)\.gn\.", r"input_projections.\1.1.", r)
            r = re.sub(r"^lateral\.conv\.", "adapter_1.0.", r)
            r = re.sub(r"^lateral\.gn\.", "adapter_1.1.", r)
            r = re.sub(r"^output\.conv\.", "layer_1.0.", r)
            r = re.sub(r"^output\.gn\.", "layer_1.1.", r)
            r = re.sub(r"^mask_proj\.", "mask_projection.", r)
            r = re.sub(r"^encoder\.(\d+)\.attn\.", r"encoder.layers.\1.self_attn.", r)
            r = re.sub(r"^encoder\.(\d+)\.norm1\.", r"encoder.layers.\1.self_attn_layer_norm.", r)
            r = re.sub(r"^encoder\.(\d+)\.norm2\.", r"encoder.layers.\1.final_layer_norm.", r)
            r = re.sub(r"^encoder\.(\d+)\.(fc\d)\.", r"encoder.layers.\1.\2.", r)
            out[_HF_PD + r] = v
            continue
        if k.startswith("decoder."):
            r = k[len("decoder."):]
            r = r.replace("query_embed", "queries_embedder").replace("query_feat", "queries_features")
            r = re.sub(r"^layers\.", "decoder.layers.", r)
            r = re.sub(r"^norm\.", "decoder.layernorm.", r)
            r = re.sub(r"^mask_embed\.(\d)\.", r"decoder.mask_predictor.mask_embedder.\1.0.", r)
            r = r.replace("norm_cross", "cross_attn_layer_norm").replace("norm_self", "self_attn_layer_norm")
            r = r.replace("norm_ffn", "final_layer_norm")
            out[_HF_TM + r] = v
            continue
        if k.startswith("class_head."):
            out["class_predictor." + k.split(".", 1)[1]] = v
            continue
        raise KeyError(f"unmapped build key {k}")
    ew = torch.ones(num_labels + 1)
    ew[-1] = no_object_weight
    out["criterion.empty_weight"] = ew
    return out
