"""Swin + Mask2Former on the MI355X kernels.

Same module tree and parameter names as the oracle restatement (oracle/ref_model.py)
so one state dict drives both; `visionseg.convert.from_hf_state_dict` loads HF /
upstream-layout checkpoints.  The hot path runs on the hand-written HIP kernels:

  Swin block      LN -> window_partition (pad+roll+partition, HIP) -> fused qkv Linear
                  -> window_attention (rel-bias + shift mask in-kernel, HIP) -> proj
                  -> window_reverse (HIP) -> residual -> MLP            (HF:swin:508-574)
  pixel decoder   6 x MSDeformAttn encoder layers, sampling on the HIP gather kernel
                  (HF:m2f:919-1103); FPN tail on MIOpen convs (HF:m2f:1394-1419)
  decoder         9 x [masked cross-attn (HIP) -> self-attn -> FFN]; every mask
                  prediction = query MLP -> mask_head MFMA kernel -> attn_bitmask kernel
                  (HF:m2f:1801-1960, 2018-2056)

Plain Linear / LayerNorm / conv / GroupNorm stay on hipBLASLt / MIOpen through torch.
Under torch.autocast(bfloat16) the kernels run their bf16 path (f32 accumulate); in
fp32 they run the exact-f32 path used by the parity tests.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, asdict

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from . import linear as linear_mod
from .linear import (SmallLinear, TokenLayerNorm, TokenLinear, fp8_operand_ok, in_projection, linear_fp8_tokens,
                     linear_gelu_tokens,
                     linear_relu_tokens, mlp_fp8, linear_tokens, plane_projection, token_plane_projection, self_attn_in_proj, small_linear, value_query_projection,
                     reattach_level_embed)


@dataclass
class M2FConfig:
    embed_dim: int = 96
    depths: tuple = (2, 2, 6, 2)
    num_heads: tuple = (3, 6, 12, 24)
    window_size: int = 7
    mlp_ratio: float = 4.0
    feature_size: int = 256
    mask_feature_size: int = 256
    hidden_dim: int = 256
    enc_ffn: int = 1024
    dec_ffn: int = 2048
    dec_heads: int = 8
    enc_layers: int = 6
    dec_layers: int = 10
    num_queries: int = 100
    num_labels: int = 1
    n_points: int = 4
    n_levels: int = 3
    no_object_weight: float = 0.1
    class_weight: float = 2.0
    mask_weight: float = 5.0
    dice_weight: float = 5.0
    train_num_points: int = 12544
    oversample_ratio: float = 3.0
    importance_sample_ratio: float = 0.75
    # BASELINE config C5: the Swin window-attention core on fp8 (e4m3) MFMA
    # (vs_window_attn_forward_fp8; bf16 activations, window^2 <= 160)
    attn_fp8: bool = False
    # BASELINE config C5: the Swin block's K-deep Linears (qkv, proj, fc1, fc2 with K % 128 == 0
    # and K >= linear.FP8_MIN_K) on the block-scaled MX fp8 MFMA (vs_token_gemm; straight-through
    # backward in bf16)
    linear_fp8: bool = False

    @staticmethod
    def preset(name: str, **kw) -> "M2FConfig":
        """Backbone presets of BASELINE.json's configs (upstream Mask2Former Swin configs)."""
        p = {
            "swin_t": dict(embed_dim=96, depths=(2, 2, 6, 2), num_heads=(3, 6, 12, 24), window_size=7),
            "swin_s": dict(embed_dim=96, depths=(2, 2, 18, 2), num_heads=(3, 6, 12, 24), window_size=7),
            "swin_b": dict(embed_dim=128, depths=(2, 2, 18, 2), num_heads=(4, 8, 16, 32), window_size=12),
            "swin_l": dict(embed_dim=192, depths=(2, 2, 18, 2), num_heads=(6, 12, 24, 48), window_size=12),
        }[name]
        p.update(kw)
        return M2FConfig(**p)

    @staticmethod
    def from_dict(d):
        d = dict(d)
        for k in ("depths", "num_heads"):
            if k in d:
                d[k] = tuple(d[k])
        return M2FConfig(**{k: v for k, v in d.items() if k in M2FConfig.__dataclass_fields__})

    def to_dict(self):
        d = asdict(self)
        d["depths"] = list(self.depths)
        d["num_heads"] = list(self.num_heads)
        return d


def _padded(n, ws):
    return n + (ws - n % ws) % ws


def _compute_dtype(t):
    return torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled() else t.dtype


# ----------------------------------------------------------------------------------
# Swin backbone
# ----------------------------------------------------------------------------------


class WindowAttention(nn.Module):
    def __init__(self, dim, heads, ws):
        super().__init__()
        if dim != heads * 32:
            raise ValueError("the window-attention kernel needs head_dim == 32")
        self.heads, self.ws = heads, ws
        self.qkv = TokenLinear(dim, 3 * dim)
        self.proj = TokenLinear(dim, dim)
        self.rel_table = nn.Parameter(torch.zeros((2 * ws - 1) ** 2, heads))


class Mlp(nn.Module):
    """fc1 -> GELU (exact erf) -> fc2 (HF:swin:511-536): fc1's GELU in the token GEMM's
    epilogue (linear.linear_gelu_tokens); fp8 (config C5): the K-deep products on the MX
    MFMA (linear.linear_fp8_tokens)."""

    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = TokenLinear(dim, hidden)
        self.fc2 = TokenLinear(hidden, dim)
        self.fp8 = False

    def forward(self, x, xq=None):
        if self.fp8:
            return mlp_fp8(x, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias, xq)
        # the GELU output feeds fc2 only: its backward rides in fc2's dX GEMM (ops.GeluBackwardSink)
        gs = ops.GeluBackwardSink()
        h = linear_gelu_tokens(x, self.fc1.weight, self.fc1.bias, gelu_sink=gs)
        return linear_tokens(h, self.fc2.weight, self.fc2.bias, gelu_sink=gs)


class SwinBlock(nn.Module):
    def __init__(self, dim, heads, ws, shift, mlp_ratio):
        super().__init__()
        self.ws, self.shift = ws, shift
        self.attn_fp8 = False                  # set by SwinBackbone from M2FConfig.attn_fp8
        self.linear_fp8 = False                # set by SwinBackbone from M2FConfig.linear_fp8
        self.norm1 = TokenLayerNorm(dim)
        self.attn = WindowAttention(dim, heads, ws)
        self.norm2 = TokenLayerNorm(dim)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))

    def forward(self, x, H, W, res=None, table32=None):
        """x: residual stream; res: the previous block's pending MLP branch (added to x
        inside this block's first LayerNorm); table32: the relative-position table already in
        f32 (SwinBackbone casts all blocks' at once).  Returns (stream, pending MLP branch):
        the caller adds the branch in the next norm (ops.add_layer_norm)."""
        B, L, C = x.shape
        ws, shift = self.ws, self.shift
        # the window partition folded into the norm's stores (ops.WindowRows): h comes out
        # in the window layout [B*nW*ws^2, C], padding rows zero
        wr = ops.window_rows(B, H, W, ws, shift, x.device)
        # MX backend: the Linears over C features take the MX fp8 path and the norms write
        # their MX operand copies; the rowwise backend (linear.FP8_GEMM "rows") quantises in
        # linear_fp8_tokens / the MLP's fused GELU pass instead
        q8 = self.linear_fp8 and fp8_operand_ok(C) and linear_mod.FP8_GEMM == "mx"
        # rowwise backend: the norms write the row-scaled e4m3 copy of their output where the
        # consuming Linear (qkv: C -> 3C, fc1: C -> 4C) takes the fp8 GEMM
        Mw = wr.total if wr is not None else B * L
        r_qkv = self.linear_fp8 and linear_mod.FP8_GEMM == "rows" and linear_mod.fp8_rows_ok(Mw, 3 * C, C)
        r_fc1 = (self.linear_fp8 and linear_mod.FP8_GEMM == "rows"
                 and linear_mod.fp8_rows_ok(B * L, self.mlp.fc1.weight.shape[0], C))
        if r_qkv:
            if res is None:
                h, hq = self.norm1.forward_windows(x, wr, quant="rows")
            else:
                x, h, hq = self.norm1.add_forward_windows(x, res, wr, quant="rows")
            qkv = linear_fp8_tokens(h.view(-1, ws * ws, C), self.attn.qkv.weight, self.attn.qkv.bias, hq)
        elif q8:
            # the norms also write their output as the fp8 GEMM operand (no quantisation pass)
            if res is None:
                h, hq = self.norm1.forward_windows(x, wr, quant=True)
            else:
                x, h, hq = self.norm1.add_forward_windows(x, res, wr, quant=True)
            qkv = linear_fp8_tokens(h.view(-1, ws * ws, C), self.attn.qkv.weight, self.attn.qkv.bias, hq)
        elif res is None:
            h = self.norm1.forward_windows(x, wr)
        else:
            x, h = self.norm1.add_forward_windows(x, res, wr)
        if not (q8 or r_qkv):
            qkv = (linear_fp8_tokens(h.view(-1, ws * ws, C), self.attn.qkv.weight, self.attn.qkv.bias)
                   if self.linear_fp8 else self.attn.qkv(h.view(-1, ws * ws, C)))
        # output in the image layout (window reverse folded into the kernel); the per-token
        # proj commutes with the crop
        o = ops.window_attention_image(qkv, self.attn.rel_table, self.attn.heads, ws, shift, B, H, W,
                                       fp8=self.attn_fp8 and qkv.dtype == torch.bfloat16, table32=table32)
        # proj (C -> C): the MX backend only; on the rowwise backend its input would need a
        # quantisation pass of its own, which costs what the fp8 GEMM saves (Swin-L stage 3:
        # 0.0355 vs 0.0432 ms, tools/r5/scaled_mm_probe.py)
        if self.linear_fp8 and linear_mod.FP8_GEMM == "mx":
            o = linear_fp8_tokens(o.view(B, H * W, C), self.attn.proj.weight, self.attn.proj.bias)
        else:
            o = self.attn.proj(o.view(B, H * W, C))
        if q8 or r_fc1:
            x, h2, h2q = self.norm2.add_forward(x, o, quant="rows" if r_fc1 else True)
            return x, self.mlp(h2, h2q)
        x, h2 = self.norm2.add_forward(x, o)
        return x, self.mlp(h2)


class PatchMerging(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.norm = TokenLayerNorm(4 * dim)
        self.reduction = TokenLinear(4 * dim, 2 * dim, bias=False)

    def forward(self, x, H, W):
        B, L, C = x.shape
        x = x.view(B, H, W, C)
        if H % 2 == 1 or W % 2 == 1:
            x = F.pad(x, (0, 0, 0, W % 2, 0, H % 2))
        # HF's cat of the 4 strided quarters (x0 = [0::2, 0::2], x1 = [1::2, 0::2],
        # x2 = [0::2, 1::2], x3 = [1::2, 1::2]; HF:swin PatchMerging) as one space-to-depth
        # permute: channel block j = 2 c + r.  Its backward is one copy, where the cat's was
        # 4 zero-filled slice gradients and 3 full-size adds.
        Hp, Wp = x.shape[1] // 2, x.shape[2] // 2
        x = x.view(B, Hp, 2, Wp, 2, C).permute(0, 1, 3, 4, 2, 5).reshape(B, Hp * Wp, 4 * C)
        return self.reduction(self.norm(x))


class Stage(nn.Module):
    def __init__(self, dim, depth, heads, ws, mlp_ratio, downsample):
        super().__init__()
        self.blocks = nn.ModuleList(
            [SwinBlock(dim, heads, ws, 0 if i % 2 == 0 else ws // 2, mlp_ratio) for i in range(depth)])
        self.merge = PatchMerging(dim) if downsample else None


class PatchEmbed(nn.Module):
    """Swin patch embedding (HF:swin:231-260): Conv2d(3, dim, 4, stride 4), then LayerNorm.
    The stride equals the kernel, so the conv is one GEMM over non-overlapping 4x4 patches:
    the image is cut into [B * H/4 * W/4, 3 * 4 * 4] patch rows (one permute copy of the
    input, which needs no gradient) and projected by the conv weight viewed [dim, 48] in its
    own (c, kh, kw) order -- token-major output for the LayerNorm, the split-K weight
    gradient of TokenLinear.  MIOpen ran this conv's forward at ~26 TF/s and its weight
    gradient at ~12 TF/s (C5: 0.42 + 0.90 ms per step, tools/gemm_census.py).  Training
    path only: under no_grad the library GEMM's choice differed between eager and
    graph-captured runs (tests/test_gpu_model.py::test_predictor_graph_replay_matches_eager)."""

    def __init__(self, dim):
        super().__init__()
        self.proj = nn.Conv2d(3, dim, kernel_size=4, stride=4)
        self.norm = TokenLayerNorm(dim)

    def tokens(self, px):
        """px [B, 3, H, W] (H, W multiples of 4) -> ([B, H/4 * W/4, dim], H/4, W/4)."""
        B, Ci, H, W = px.shape
        h, w = H // 4, W // 4
        if not (px.is_cuda and torch.is_grad_enabled()):   # inference keeps the conv: its graph
            x = self.proj(px)                              # replay is bit-identical to eager
            return x.flatten(2).transpose(1, 2), h, w
        # reshape, not view: a channels_last (or otherwise strided) batch is copied here
        patches = px.reshape(B, Ci, h, 4, w, 4).permute(0, 2, 4, 1, 3, 5).reshape(B * h * w, Ci * 16)
        wt = self.proj.weight
        y = linear_tokens(patches, wt.view(wt.shape[0], -1), self.proj.bias)
        return y.view(B, h * w, -1), h, w


class SwinBackbone(nn.Module):
    """Returns per-stage NCHW feature maps (pre-downsample, out-norm applied)."""

    def __init__(self, cfg: M2FConfig):
        super().__init__()
        C = cfg.embed_dim
        n = len(cfg.depths)
        self.patch_embed = PatchEmbed(C)
        self.stages = nn.ModuleList([
            Stage(C * 2 ** i, cfg.depths[i], cfg.num_heads[i], cfg.window_size, cfg.mlp_ratio, i < n - 1)
            for i in range(n)])
        self.out_norms = nn.ModuleList([TokenLayerNorm(C * 2 ** i) for i in range(n)])
        for st in self.stages:
            for blk in st.blocks:
                blk.attn_fp8 = bool(cfg.attn_fp8)
                blk.linear_fp8 = blk.mlp.fp8 = bool(cfg.linear_fp8)

    def forward(self, px):
        H, W = px.shape[-2:]
        if W % 4:
            px = F.pad(px, (0, 4 - W % 4))
        if H % 4:
            px = F.pad(px, (0, 0, 0, 4 - H % 4))
        x, H, W = self.patch_embed.tokens(px)
        B = x.shape[0]
        x = self.patch_embed.norm(x)
        feats = []
        # the attention kernels read the relative-position tables in f32: every block's as one
        # cast (cat + cast: 2 launches where each block's own cast was one launch per block);
        # the tables' gradients still reach the bf16 parameters (ops.window_attention_image)
        blocks = [blk for st in self.stages for blk in st.blocks]
        t32 = None
        if px.is_cuda and blocks and blocks[0].attn.rel_table.dtype != torch.float32:
            flat = torch.cat([blk.attn.rel_table.detach().reshape(-1) for blk in blocks]).float()
            t32, o = {}, 0
            for blk in blocks:
                n = blk.attn.rel_table.numel()
                t32[id(blk)] = flat[o:o + n].view(blk.attn.rel_table.shape)
                o += n
        for i, st in enumerate(self.stages):
            res = None
            for blk in st.blocks:
                x, res = blk(x, H, W, res, t32[id(blk)] if t32 is not None else None)
            x, f = self.out_norms[i].add_forward(x, res)     # stream + last MLP branch, stage norm
            feats.append(f.view(B, H, W, -1).permute(0, 3, 1, 2))     # NCHW view, channels-last memory
            if st.merge is not None:
                x = st.merge(x, H, W)
                H, W = (H + 1) // 2, (W + 1) // 2
        return feats


# ----------------------------------------------------------------------------------
# Pixel decoder
# ----------------------------------------------------------------------------------


def sine_pos_embed(B, H, W, num_feats, device, dtype=torch.float32, temperature=10000, scale=2 * math.pi):
    """Normalised sine embedding (HF:m2f:864-904), [B, 2*num_feats, H, W]."""
    y = torch.arange(1, H + 1, dtype=dtype, device=device)[None, :, None].expand(B, H, W)
    x = torch.arange(1, W + 1, dtype=dtype, device=device)[None, None, :].expand(B, H, W)
    eps = 1e-6
    y = y / (y[:, -1:, :] + eps) * scale
    x = x / (x[:, :, -1:] + eps) * scale
    dim_t = torch.arange(num_feats, dtype=torch.int64, device=device).to(dtype)
    dim_t = temperature ** (2 * torch.div(dim_t, 2, rounding_mode="floor") / num_feats)
    px = x[:, :, :, None] / dim_t
    py = y[:, :, :, None] / dim_t
    px = torch.stack((px[:, :, :, 0::2].sin(), px[:, :, :, 1::2].cos()), dim=4).flatten(3)
    py = torch.stack((py[:, :, :, 0::2].sin(), py[:, :, :, 1::2].cos()), dim=4).flatten(3)
    return torch.cat((py, px), dim=3).permute(0, 3, 1, 2)


_SINE_CACHE: dict = {}


def sine_pos_tokens(B, H, W, num_feats, device, dtype):
    """sine_pos_embed in the token-major layout [B, H*W, 2*num_feats] and `dtype`, made
    once per (shape, device, dtype): it depends on nothing else, so the training step does
    not recompute it (~15 kernels and 67 MB f32 intermediates per 128x128 level).  Never
    cached while a HIP graph is being captured (the entry would live in the graph's pool);
    the trainer's eager warm-up steps fill the cache first.  An LRU of 32 entries (a full
    clear could drop an entry between a warm-up and the capture that reads it)."""
    key = (B, H, W, num_feats, str(device), dtype)
    t = _SINE_CACHE.get(key)
    if t is None:
        with torch.no_grad():
            t = sine_pos_embed(B, H, W, num_feats, device).to(dtype).flatten(2).transpose(1, 2).contiguous()
        capturing = t.is_cuda and torch.cuda.is_current_stream_capturing()
        if not capturing:
            _SINE_CACHE[key] = t
            while len(_SINE_CACHE) > 32:               # LRU: the warm-up's entries stay
                _SINE_CACHE.pop(next(iter(_SINE_CACHE)))
    else:
        _SINE_CACHE[key] = _SINE_CACHE.pop(key)        # most recently used last
    return t


def cached_constants():
    """The tensors held by the process-wide constant caches right now.  A HIP graph reads
    them by address: whoever captures a graph keeps this list with it, so evicting an
    entry (the cache is cleared at 32 shapes) cannot free memory a live graph still
    replays from -- that freed block, reused, made graph replays differ from eager runs
    (tests/test_gpu_model.py::test_predictor_graph_replay_matches_eager after a suite's
    worth of shapes)."""
    return list(_SINE_CACHE.values()) + ops.window_rows_constants()


def reference_points(shapes, B, device, dtype=torch.float32):
    """HF:m2f:1127-1156 with valid ratios 1 -> [B, S, L, 2]."""
    refs = []
    for (Hl, Wl) in shapes:
        ry, rx = torch.meshgrid(torch.linspace(0.5, Hl - 0.5, Hl, dtype=dtype, device=device),
                                torch.linspace(0.5, Wl - 0.5, Wl, dtype=dtype, device=device), indexing="ij")
        refs.append(torch.stack((rx.reshape(-1)[None] / Wl, ry.reshape(-1)[None] / Hl), -1))
    r = torch.cat(refs, 1)
    return r[:, :, None].expand(B, -1, len(shapes), -1)


_MSDA_PREP = os.environ.get("VS_MSDA_PREP", "1") == "1"          # A/B switch: fused prologue


class MSDeformAttn(nn.Module):
    def __init__(self, d, heads, levels, points):
        super().__init__()
        self.d, self.heads, self.levels, self.points = d, heads, levels, points
        self.sampling_offsets = TokenLinear(d, heads * levels * points * 2)
        self.attention_weights = TokenLinear(d, heads * levels * points)
        self.value_proj = TokenLinear(d, d)
        self.output_proj = TokenLinear(d, d)

    def forward(self, h, pos, ref, shapes, norm, level=None, sink=None):
        """level: (level_embed, level sizes) when pos holds detached level-embedding rows
        (PixelDecoder); sink: ops.ResidualSink of the post-norm residual around this op."""
        B, S, _ = h.shape
        lvl_embed, lvl_sizes = level if level is not None else (None, None)
        if _MSDA_PREP:                       # one HIP kernel each way (csrc/msda_prep.hip)
            # both projections of q = h + pos as one GEMM (q read once, one dX GEMM, no add
            # of their input gradients), the value projection of h beside it (its dX lands
            # in the same GEMM epilogue); the prologue reads the packed projection's two
            # column ranges and its backward writes one packed gradient
            so, at = self.sampling_offsets, self.attention_weights
            value, proj = value_query_projection(h, pos, self.value_proj.weight, self.value_proj.bias,
                                                 torch.cat((so.weight, at.weight)), torch.cat((so.bias, at.bias)),
                                                 lvl_embed, lvl_sizes, sink)
            value = value.view(B, S, self.heads, self.d // self.heads)
            loc, aw = ops.msda_prep(proj, None, ref, shapes, self.heads, self.points)
        else:
            q = h + reattach_level_embed(pos, lvl_embed, lvl_sizes)
            value = self.value_proj(h).view(B, S, self.heads, self.d // self.heads)
            off = self.sampling_offsets(q).view(B, S, self.heads, self.levels, self.points, 2)
            aw = self.attention_weights(q).view(B, S, self.heads, self.levels * self.points)
            aw = F.softmax(aw.float(), -1).view(B, S, self.heads, self.levels, self.points)
            loc = ref[:, :, None, :, None, :] + off.float() / norm           # HF:m2f:994-1002
        out = ops.ms_deform_attn(value, shapes, loc, aw)
        return self.output_proj(out)


class EncoderLayer(nn.Module):
    def __init__(self, d, ffn, heads, levels, points):
        super().__init__()
        self.attn = MSDeformAttn(d, heads, levels, points)
        self.norm1 = TokenLayerNorm(d)
        self.fc1 = TokenLinear(d, ffn)
        self.fc2 = TokenLinear(ffn, d)
        self.norm2 = TokenLayerNorm(d)

    def forward(self, h, pos, ref, shapes, norm, level=None):
        # post-norm, residual add fused into the norm; each residual gradient is added by
        # the dX GEMM of the branch's first op (ops.ResidualSink), not by autograd
        s1, s2 = ops.ResidualSink(), ops.ResidualSink()
        _, h = self.norm1.add_forward(h, self.attn(h, pos, ref, shapes, norm, level, s1), s1)
        # bias + ReLU in the GEMM; the ReLU's backward in fc2's dX epilogue (ops.ActBackwardSink)
        rs = ops.ActBackwardSink("relu")
        f = linear_relu_tokens(h, self.fc1.weight, self.fc1.bias, s2, act_sink=rs)
        _, h = self.norm2.add_forward(h, linear_tokens(f, self.fc2.weight, self.fc2.bias, gelu_sink=rs), s2)
        return h


_TORCH_GN = os.environ.get("VS_TORCH_GROUPNORM", "0") == "1"     # A/B switch
_PIXDEC_NCHW = os.environ.get("VS_PIXDEC_NCHW", "1") == "1"    # A/B switch: NCHW 1/4-res blocks
# the bf16 1/4-res tail channels-last with the hand-written 3x3 conv (PixelDecoder._tail_nhwc)
_PIXDEC_NHWC = os.environ.get("VS_PIXDEC_NHWC", "1") == "1"


class ConvGN(nn.Module):
    """Conv2d + GroupNorm(32) (+ ReLU when relu=True), the norm on the HIP kernels
    (csrc/groupnorm.hip, ReLU fused) for device tensors of matching dtype, torch's
    otherwise.  nchw=False: the conv sees channels-last activations (Swin features) and
    the output stays channels-last (the encoder flattens it token-major for free).
    nchw=True: the 1/4-resolution blocks run NCHW end to end (MIOpen's NCHW 3x3 conv
    kernels are the fast ones there; the NCHW GroupNorm needs no layout copy)."""

    def __init__(self, cin, cout, k, bias, relu=False, nchw=False, stride=1):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, kernel_size=k, padding=k // 2, bias=bias, stride=stride)
        self.gn = nn.GroupNorm(32, cout)
        self.relu = relu
        self.nchw = nchw

    def forward(self, x):
        gn = self.gn
        hip = (x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and gn.weight.dtype == x.dtype
               and not torch.is_autocast_enabled() and not _TORCH_GN)
        conv = self.conv
        if hip and self.nchw and _PIXDEC_NCHW:
            y = self.conv(x.contiguous())
            if y.is_contiguous():
                return ops.group_norm_nchw(y, gn.weight, gn.bias, gn.num_groups, gn.eps, self.relu)
        elif (hip and conv.kernel_size == (1, 1) and conv.stride == (1, 1) and x.dim() == 4
              and x.dtype == torch.bfloat16 == conv.weight.dtype and torch.is_grad_enabled()
              and x.is_contiguous(memory_format=torch.channels_last)):
            # the input projections' 1x1 convs on the channels-last Swin features as token
            # Linears: the bias in the GEMM epilogue and its gradient in the split-K weight
            # gradient (MIOpen's conv + an ATen bias add forward, an ATen sum backward: 6 launches
            # per step).  Training only, like PatchEmbed (the inference graphs keep the conv)
            B, Ci, H, W = x.shape
            Co = conv.weight.shape[0]
            y = linear_tokens(x.permute(0, 2, 3, 1).reshape(B * H * W, Ci), conv.weight.view(Co, Ci), conv.bias)
            y = y.view(B, H, W, Co).permute(0, 3, 1, 2)       # NCHW view, channels-last memory
        else:
            y = self.conv(x)
        if hip and y.shape[1] == 8 * gn.num_groups and y.is_contiguous(memory_format=torch.channels_last):
            out = ops.group_norm_nhwc(y, gn.weight, gn.bias, gn.num_groups, gn.eps, self.relu)
            return out if _PIXDEC_NCHW else out.contiguous()
        y = gn(y)
        return F.relu(y) if self.relu else y


class PixelDecoder(nn.Module):
    """Multi-scale deformable-attention pixel decoder: Mask2Former's (3 levels: res5, res4,
    res3; HF:m2f:1236-1419) or MaskDINO's "4s" encoder (n_levels = 4: an extra 1/64
    level from a stride-2 3x3 conv + GroupNorm of res5 in front; upstream MaskDINOEncoder,
    not in the container).  Levels run coarse to fine."""

    def __init__(self, cfg: M2FConfig, channels):
        super().__init__()
        Fd = cfg.feature_size
        self.cfg = cfg
        self.n_levels = int(getattr(cfg, "n_levels", 3))
        if self.n_levels not in (3, 4):
            raise ValueError("the pixel decoder takes 3 or 4 levels")
        self.input_proj = nn.ModuleList([ConvGN(c, Fd, 1, True) for c in channels[::-1][:3]])
        self.extra = ConvGN(channels[-1], Fd, 3, True, stride=2) if self.n_levels == 4 else None
        self.level_embed = nn.Parameter(torch.zeros(self.n_levels, Fd))
        self.encoder = nn.ModuleList([EncoderLayer(Fd, cfg.enc_ffn, cfg.dec_heads, self.n_levels, cfg.n_points)
                                      for _ in range(cfg.enc_layers)])
        self.lateral = ConvGN(channels[0], Fd, 1, False, nchw=True)
        self.output = ConvGN(Fd, Fd, 3, False, relu=True, nchw=True)
        self.mask_proj = nn.Conv2d(Fd, cfg.mask_feature_size, kernel_size=1)
        self._norm_cache = {}
        self._ref_cache = {}
        self._pos_cache = {}

    def forward(self, feats):
        Fd = self.cfg.feature_size
        dev = feats[0].device
        embeds = []
        if self.extra is not None:
            embeds.append(self.extra(feats[-1]))
        for lvl, x in enumerate(feats[::-1][:3]):
            embeds.append(self.input_proj[lvl](x))
        pos = [sine_pos_tokens(e.shape[0], e.shape[2], e.shape[3], Fd // 2, dev, e.dtype) for e in embeds]
        shapes = [(int(e.shape[2]), int(e.shape[3])) for e in embeds]
        B = embeds[0].shape[0]
        h = torch.cat([e.flatten(2).transpose(1, 2) for e in embeds], 1)
        # position term with detached level-embedding rows: the layers route the level
        # embedding's gradient themselves (per-level column sums, linear.value_query_projection)
        lvl = self.level_embed.detach()
        sizes = [Hl * Wl for (Hl, Wl) in shapes]
        pkey = (tuple(shapes), B, str(dev), pos[0].dtype)
        sine = self._pos_cache.get(pkey)
        if sine is None:      # the levels' sine embeddings concatenated: constant per shape set
            sine = torch.cat(pos, 1)
            if not (sine.is_cuda and torch.cuda.is_current_stream_capturing()):
                self._pos_cache[pkey] = sine
        # + the level-embedding rows: one broadcast add (was an add per level and a cat)
        rows = torch.cat([lvl[i].to(sine.dtype).expand(n, Fd) for i, n in enumerate(sizes)], 0)
        p = sine + rows
        level = (self.level_embed, sizes)
        ref = self._ref_cache.get((tuple(shapes), B, str(dev)))
        if ref is None:       # constant per shape set, like the sine embedding (sine_pos_tokens)
            ref = reference_points(shapes, B, dev)
            if not (ref.is_cuda and torch.cuda.is_current_stream_capturing()):
                self._ref_cache[(tuple(shapes), B, str(dev))] = ref
        key = (tuple(shapes), dev)
        norm = self._norm_cache.get(key)
        if norm is None:      # made once per shape set: no host->device copy inside a graph capture
            norm = torch.tensor([[w, hh] for hh, w in shapes], device=dev, dtype=torch.float32)[None, None, None, :, None, :]
            self._norm_cache[key] = norm
        for layer in self.encoder:
            h = layer(h, p, ref, shapes, norm, level)
        # encoder levels, token-major [B, H_l*W_l, C] (split: one concatenating backward
        # instead of a zero-filled full-size gradient per slice)
        toks = torch.split(h, [Hl * Wl for (Hl, Wl) in shapes], dim=1)
        outs = [(t, hw) for t, hw in zip(toks, shapes)]
        f0 = feats[0]
        lat = self.lateral
        Hs, Ws = shapes[-1]
        if self._nhwc_tail(f0):
            return self._tail_nhwc(f0, toks[-1], Hs, Ws), outs
        if (f0.is_cuda and _PIXDEC_NCHW and not torch.is_autocast_enabled() and lat.conv.kernel_size == (1, 1)
                and f0.is_contiguous(memory_format=torch.channels_last) and f0.dtype == lat.conv.weight.dtype
                and f0.dtype in (torch.float32, torch.bfloat16) and lat.gn.weight.dtype == f0.dtype and not _TORCH_GN):
            # the 1x1 lateral conv straight from the channels-last (token-major) feature to
            # NCHW planes: no NCHW copy of the feature (linear.token_plane_projection)
            B0, C0, H0, W0 = f0.shape
            cur = token_plane_projection(f0.permute(0, 2, 3, 1).reshape(B0, H0 * W0, C0), lat.conv.weight,
                                         lat.conv.bias, H0, W0)
            cur = ops.group_norm_nchw(cur, lat.gn.weight, lat.gn.bias, lat.gn.num_groups, lat.gn.eps, lat.relu)
        else:
            cur = self.lateral(f0)
        if (cur.is_cuda and _PIXDEC_NCHW and cur.shape[1] % 32 == 0 and cur.shape[2] <= 2 * Hs
                and cur.shape[3] <= 2 * Ws and not torch.is_autocast_enabled()):
            y = ops.upsample_add(cur, toks[-1], Hs, Ws)                  # csrc/upsample.hip
        else:
            lvl = toks[-1].transpose(1, 2).reshape(B, -1, Hs, Ws)
            y = cur + F.interpolate(lvl.to(cur.dtype), size=cur.shape[-2:], mode="bilinear", align_corners=False)
        y = self.output(y)
        if y.is_cuda and _PIXDEC_NCHW:
            # token-major mask features straight from the NCHW planes (channels-last view)
            return plane_projection(y, self.mask_proj.weight, self.mask_proj.bias), outs
        return self.mask_proj(y), outs

    def _nhwc_tail(self, f0) -> bool:
        lat, out = self.lateral, self.output
        return (f0.is_cuda and _PIXDEC_NHWC and not torch.is_autocast_enabled() and not _TORCH_GN
                and f0.dtype == torch.bfloat16 and f0.is_contiguous(memory_format=torch.channels_last)
                and lat.conv.kernel_size == (1, 1) and lat.conv.weight.dtype == f0.dtype
                and out.conv.kernel_size == (3, 3) and out.conv.stride == (1, 1) and out.conv.padding == (1, 1)
                and lat.gn.weight.dtype == f0.dtype and out.gn.weight.dtype == f0.dtype
                and self.mask_proj.weight.dtype == f0.dtype
                and out.conv.out_channels == 8 * out.gn.num_groups == 8 * lat.gn.num_groups
                and out.conv.in_channels % 128 == 0 and out.conv.out_channels % 128 == 0
                and out.conv.dilation == (1, 1) and out.conv.groups == 1)

    def _tail_nhwc(self, f0, top, Hs, Ws):
        """The 1/4-resolution FPN tail (HF:m2f:1394-1419) channels-last end to end: the 1x1
        lateral conv as a token GEMM on the channels-last Swin feature, GroupNorm NHWC, the
        upsample + add of the finest encoder level (upsample.hip NHWC), the 3x3 output conv
        (conv3x3.hip) + GroupNorm + ReLU, and the 1x1 mask projection as a token GEMM whose
        output is the token-major mask-feature map the mask head reads.  No NCHW <-> NHWC
        transposes anywhere (MIOpen's conv needed 8-9 per step)."""
        lat, out, mp = self.lateral, self.output, self.mask_proj
        B0, C0, H0, W0 = f0.shape
        Fd = lat.conv.out_channels
        t0 = f0.permute(0, 2, 3, 1).reshape(B0, H0 * W0, C0)
        cur = linear_tokens(t0, lat.conv.weight.view(Fd, C0), lat.conv.bias)
        cur = ops.group_norm_nhwc(cur.view(B0, H0, W0, Fd).permute(0, 3, 1, 2), lat.gn.weight, lat.gn.bias,
                                  lat.gn.num_groups, lat.gn.eps, lat.relu)
        y = ops.upsample_add_nhwc(cur, top, Hs, Ws)
        y = ops.conv3x3_nhwc(y, out.conv.weight, out.conv.bias)
        y = ops.group_norm_nhwc(y, out.gn.weight, out.gn.bias, out.gn.num_groups, out.gn.eps, out.relu)
        Cm = mp.out_channels
        m = linear_tokens(y.permute(0, 2, 3, 1).reshape(B0, H0 * W0, Fd), mp.weight.view(Cm, Fd), mp.bias)
        return m.view(B0, H0, W0, Cm).permute(0, 3, 1, 2)


# ----------------------------------------------------------------------------------
# Masked-attention decoder
# ----------------------------------------------------------------------------------


def self_attention_core(q, k, v, heads, scale, words=None):
    """softmax(q k^T * scale [+ blocked keys]) v over [B, Q, heads*d] token rows -> [B, Q, heads*d]:
    the hand-written kernels (ops.self_attention: csrc/self_attn.hip for bf16, the scalar
    masked-attention kernels for f32) on the device; the plain composition on the CPU."""
    if q.is_cuda and q.shape[-1] == 32 * heads:
        return ops.self_attention(q, k, v, heads, scale, words=words)
    B, Q, D = q.shape
    S = k.shape[1]
    d = D // heads
    s = torch.einsum("bqhd,bkhd->bhqk", q.view(B, Q, heads, d).float(), k.view(B, S, heads, d).float()) * scale
    if words is not None:
        blocked = ops.unpack_bitmask(words, S)
        s = s.masked_fill((blocked if blocked.dim() == 3 else blocked[None])[:, None], float("-inf"))
    att = torch.einsum("bhqk,bkhd->bqhd", s.softmax(-1), v.view(B, S, heads, d).float())
    return att.reshape(B, Q, D).to(q.dtype)


class CrossAttn(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d, d))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * d))
        self.out_proj = SmallLinear(d, d)


class SelfAttn(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.q_proj = SmallLinear(d, d)
        self.k_proj = SmallLinear(d, d)
        self.v_proj = SmallLinear(d, d)
        self.out_proj = SmallLinear(d, d)


class DecoderLayer(nn.Module):
    def __init__(self, d, ffn, heads):
        super().__init__()
        self.heads = heads
        self.cross_attn = CrossAttn(d)
        self.norm_cross = TokenLayerNorm(d)
        self.self_attn = SelfAttn(d)
        self.norm_self = TokenLayerNorm(d)
        self.fc1 = SmallLinear(d, ffn)
        self.fc2 = SmallLinear(ffn, d)
        self.norm_ffn = TokenLayerNorm(d)

    def forward(self, h, qpos, mem, mem_pos, words, psink=None, msink=None):
        """mem: level memory [B, hw, D] (contiguous), mem_pos = mem + its position embedding.
        psink: ops.GradSink of qpos (the layers' query-position gradients summed in one
        buffer by the projection kernels).  Each post-norm block hands its residual-path
        gradient to the projection that consumes its input (ops.ResidualSink): no
        gradient adds between the blocks."""
        B, Q, D = h.shape
        H, d = self.heads, D // self.heads
        s1, s2, s3 = ops.ResidualSink(), ops.ResidualSink(), ops.ResidualSink()
        q, k, v = in_projection(h, mem_pos, mem, self.cross_attn.in_proj_weight, self.cross_attn.in_proj_bias,
                                q_pos=qpos, sink=s1, psink=psink, kv_sink=msink)  # query = h + qpos
        o = ops.masked_attention(q, k, v, words, H, d ** -0.5)
        _, h = self.norm_cross.add_forward(h, self.cross_attn.out_proj(o), sink=s1)   # post-norm, fused add
        sa = self.self_attn
        q_, k_, v_ = self_attn_in_proj(h, qpos, sa.q_proj, sa.k_proj, sa.v_proj, sink=s2, psink=psink)
        att = self_attention_core(q_, k_, v_, H, d ** -0.5)          # HF:m2f:1659-1664
        _, h = self.norm_self.add_forward(h, sa.out_proj(att), sink=s2)
        f = small_linear(h, self.fc1.weight, self.fc1.bias, relu=True, sink=s3)
        _, h = self.norm_ffn.add_forward(h, self.fc2(f), sink=s3)
        return h


class Decoder(nn.Module):
    def __init__(self, cfg: M2FConfig):
        super().__init__()
        d = cfg.hidden_dim
        self.cfg = cfg
        self.query_feat = nn.Embedding(cfg.num_queries, d)
        self.query_embed = nn.Embedding(cfg.num_queries, d)
        self.level_embed = nn.Embedding(3, d)
        self.layers = nn.ModuleList([DecoderLayer(d, cfg.dec_ffn, cfg.dec_heads) for _ in range(cfg.dec_layers - 1)])
        self.norm = TokenLayerNorm(d)
        self.mask_embed = nn.ModuleList([SmallLinear(d, d), SmallLinear(d, d), SmallLinear(d, cfg.mask_feature_size)])
        # Parity-test hook ("teacher forcing"): a list of bool [B,Q,h*w] blocked masks, one per
        # decoder layer, used instead of the masks this decoder derives itself.  Lets a test
        # separate threshold-decision flips (sigmoid(x) < 0.5 at |x| ~ rounding) from arithmetic.
        self.mask_override = None
        self.record = False
        self.batched_heads = True
        # training (batched heads, bf16): the steps' mask logits stay factored
        # (ops.FactoredLogits); the attention masks come from E . resize(F) at the level's
        # size and the matcher from E . F(points) (csrc/match_factors.hip).  VS_FACTORED_MASKS=0
        # keeps the full-resolution logits (A/B)
        self.factored_masks = os.environ.get("VS_FACTORED_MASKS", "1") != "0"
        # ... but only for a consumer that reads FactoredLogits (the visionseg SetCriterion,
        # switched on by train.Trainer): by default forward() returns real [B,Q,H/4,W/4] f32
        # logit tensors, with or without grad, in train() or eval() mode
        self.emit_factors = False

    def embed(self, h, dtype):
        """(LN(h), mask embedding MLP_3(LN(h))) -- HF:m2f:2040-2048."""
        x = self.norm(h)
        e = F.relu(self.mask_embed[0](x))
        e = F.relu(self.mask_embed[1](e))
        return x, self.mask_embed[2](e).to(dtype)

    def predict(self, h, mf_nhwc, Hm, Wm, target_hw, sink=None):
        x, e = self.embed(h, mf_nhwc.dtype)
        logits = ops.mask_head(e, mf_nhwc, Hm, Wm, sink=sink)
        words = ops.attn_bitmask(logits, target_hw) if target_hw is not None else None
        return x, logits, words

    def level_mask(self, h, mf_level, target_hw):
        """Attention bitmask of the next layer from the factors: the logits at the level's
        size are E . resize(F) (bilinear resizing commutes with the mask head's product,
        HF:m2f:2049-2055), resize(F) given as the hi | lo bf16 pair of
        ops.feature_resize_hilo (csrc/match_factors.hip level_bitmask_kernel: the logits are
        thresholded in registers, never stored)."""
        _, e = self.embed(h, mf_level.dtype)
        return ops.level_bitmask_hilo(e, mf_level, *target_hw)

    def forward(self, ms_feats, mask_features):
        d = self.cfg.hidden_dim
        B, _, Hm, Wm = mask_features.shape
        dev = mask_features.device
        mf = mask_features.to(_compute_dtype(mask_features)).permute(0, 2, 3, 1).reshape(B, Hm * Wm, -1).contiguous()
        # Batched prediction heads (training on the device): every step's mask embedding and
        # logits are computed WITHOUT autograd inside the loop (they only steer the next
        # layer's attention mask and the matching), and the heads run once more, batched
        # over the S steps, with autograd: norm + 3-layer MLP over [S, B, Q] rows, whose
        # embeddings E [S, B, Q, C] and mf are the factors the set criterion differentiates
        # through (logits._vs_src; ops.MatchedPointLogitsFunction).  The backward is one
        # launch per head instead of S, and the shared weights' gradients need no adds.
        batched = bool(mf.requires_grad and torch.is_grad_enabled() and mf.is_cuda and self.batched_heads)
        sink = None
        if not batched:
            # the mask-head calls sum their pixel-embedding gradient in one buffer (ops.GradSink)
            sink = ops.GradSink() if (mf.requires_grad and torch.is_grad_enabled() and mf.is_cuda) else None
            if sink is not None:
                mf = sink.source(mf)
        mems, mem_pos, sizes, msinks = [], [], [], []
        for i in range(3):
            # once per level (shared by the decoder rounds): token-major memory and memory + pos
            f, (Hl, Wl) = ms_feats[i]                       # token-major [B, Hl*Wl, C]
            sizes.append((int(Hl), int(Wl)))
            pos = sine_pos_tokens(B, Hl, Wl, d // 2, dev, f.dtype)
            m = f + self.level_embed.weight[i][None, None, :].to(f.dtype)
            ms = None
            if m.is_cuda and torch.is_grad_enabled() and m.requires_grad:
                # the layers reading this level sum their K / V input gradients in one
                # buffer (ops.GradSink, linear._InProjFn)
                ms = ops.GradSink()
                m = ms.source(m)
            msinks.append(ms)
            mems.append(m)
            mem_pos.append(m + pos)
        qpos = self.query_embed.weight.unsqueeze(0).expand(B, -1, -1)
        psink = None
        if qpos.is_cuda and torch.is_grad_enabled() and qpos.requires_grad:
            psink = ops.GradSink()                   # every layer's qpos gradient in one buffer
            qpos = psink.source(qpos)
        h = self.query_feat.weight.unsqueeze(0).expand(B, -1, -1)
        n = len(self.layers)

        # (C in {128, 256}: the grouped mask-head kernel of the matched maps)
        fact = (batched and self.emit_factors and self.training and self.factored_masks and mf.dtype == torch.bfloat16 and mf.shape[-1] in (128, 256))
        mf_levels = {}

        def step(hh, target_hw):
            if not batched:
                return self.predict(hh, mf, Hm, Wm, target_hw, sink)
            with torch.no_grad():
                if not fact:
                    return self.predict(hh, mf.detach(), Hm, Wm, target_hw)
                if target_hw is None:
                    return None, None, None
                lv = mf_levels.get(target_hw)
                if lv is None:
                    lv = mf_levels[target_hw] = ops.feature_resize_hilo(mf.detach(), Hm, Wm, *target_hw)
                return None, None, self.level_mask(hh, lv, target_hw)

        hs = [h]
        inter, logits, words = step(h, sizes[0] if n else None)
        inters, masks = [inter], [logits]
        self.trace = []
        for idx, layer in enumerate(self.layers):
            lvl = idx % 3
            if self.record:
                self.trace.append(words)
            if self.mask_override is not None:
                words = pack_bitmask(self.mask_override[idx].to(dev))
            h = layer(h, qpos, mems[lvl], mem_pos[lvl], words, psink, msinks[lvl])
            hs.append(h)
            nxt = sizes[(idx + 1) % 3] if idx + 1 < n else None
            inter, logits, words = step(h, nxt)
            inters.append(inter)
            masks.append(logits)
        if batched:
            X, E = self.embed(torch.stack(hs), mf.dtype)                                # [S,B,Q,D], [S,B,Q,C]
            inters = list(X.unbind(0))
            if fact:
                masks = [ops.FactoredLogits(E, mf, s_, Hm, Wm) for s_ in range(len(hs))]
            else:
                for s_, m in enumerate(masks):
                    m._vs_src = (E, mf, s_)
        return inters, masks


def pack_bitmask(blocked: torch.Tensor) -> torch.Tensor:
    """bool [B,Q,K] (True = blocked) -> int32 words [B,Q,ceil(K/32)] in the kernels' format."""
    B, Q, K = blocked.shape
    nw = (K + 31) // 32
    pad = torch.zeros(B, Q, nw * 32, dtype=torch.int64, device=blocked.device)
    pad[..., :K] = blocked.to(torch.int64)
    bits = (pad.view(B, Q, nw, 32) << torch.arange(32, device=blocked.device)).sum(-1)
    return torch.where(bits >= 2 ** 31, bits - 2 ** 32, bits).to(torch.int32)


class Mask2Former(nn.Module):
    """Swin + Mask2Former forward: returns (mask logits per decoder step [B,Q,H/4,W/4]
    f32, class logits per step [B,Q,num_labels+1]).  Exception: with
    `decoder.emit_factors` set (train.Trainer sets it for the visionseg SetCriterion) and
    the model in train() mode with grad on, bf16, the mask logits are ops.FactoredLogits
    (E . F never materialised; `.materialize()` gives the tensor)."""

    def __init__(self, cfg: M2FConfig):
        super().__init__()
        self.cfg = cfg
        self.backbone = SwinBackbone(cfg)
        chans = [cfg.embed_dim * 2 ** i for i in range(len(cfg.depths))]
        self.pixel_decoder = PixelDecoder(cfg, chans)
        self.decoder = Decoder(cfg)
        self.class_head = nn.Linear(cfg.hidden_dim, cfg.num_labels + 1)

    def forward(self, pixel_values):
        # pure-bf16 mode (bf16 parameters): feed the backbone in the parameter dtype
        feats = self.backbone(pixel_values.to(self.backbone.patch_embed.proj.weight.dtype))
        mask_features, ms = self.pixel_decoder(feats)
        inters, masks = self.decoder(ms, mask_features)
        # one launch for all decoder steps (HF:m2f:2479-2481 per step), widened to f32 once
        # (the criterion's softmax / CE run in f32; a per-step .float() was 10 + 10 launches)
        classes = list(self.class_head(torch.stack(inters)).float().unbind(0))
        return masks, classes

    @torch.no_grad()
    def init_weights(self, seed: int = 0):
        """Training init in the spirit of upstream Mask2Former (trunc-normal Linear,
        xavier decoder projections, Deformable-DETR MSDA init, zero rel-bias)."""
        g = torch.Generator().manual_seed(seed)
        for name, m in self.named_modules():
            if isinstance(m, nn.Linear):
                w = torch.empty_like(m.weight, device="cpu")
                nn.init.trunc_normal_(w, std=0.02, generator=g)
                m.weight.copy_(w)
                if m.bias is not None:
                    m.bias.zero_()
            elif isinstance(m, nn.LayerNorm):
                m.weight.fill_(1.0)
                m.bias.zero_()
            elif isinstance(m, CrossAttn):
                w = torch.empty_like(m.in_proj_weight, device="cpu")
                nn.init.xavier_uniform_(w, generator=g)
                m.in_proj_weight.copy_(w)
                m.in_proj_bias.zero_()
            elif isinstance(m, nn.Embedding):
                w = torch.empty_like(m.weight, device="cpu")
                nn.init.normal_(w, generator=g)
                m.weight.copy_(w)
        for m in self.modules():
            if isinstance(m, MSDeformAttn):
                m.sampling_offsets.weight.zero_()
                th = torch.arange(m.heads, dtype=torch.float32) * (2.0 * math.pi / m.heads)
                grid = torch.stack([th.cos(), th.sin()], -1)
                grid = (grid / grid.abs().max(-1, keepdim=True)[0]).view(m.heads, 1, 1, 2).repeat(1, m.levels, m.points, 1)
                for i in range(m.points):
                    grid[:, :, i, :] *= i + 1
                m.sampling_offsets.bias.copy_(grid.view(-1))
                m.attention_weights.weight.zero_()
                m.attention_weights.bias.zero_()
            elif isinstance(m, WindowAttention):
                m.rel_table.zero_()
        return self


def unpack_bitmask_like(words: torch.Tensor, n_keys: int) -> torch.Tensor:
    """int32 words [B,Q,nw] -> bool [B,Q,n_keys] (True = blocked)."""
    w = words.to(torch.int64) & 0xFFFFFFFF
    bits = (w.unsqueeze(-1) >> torch.arange(32, device=w.device)) & 1
    return bits.flatten(-2)[..., :n_keys].bool()
