"""ORACLE (test infrastructure only) — CPU restatement of the hot-path operators.

Index/byte ops are numpy (bit-exact targets); floating-point ops are torch fp32 on CPU.
Each function cites the line of the in-container HF oracle (transformers 5.15.0) it
restates — see oracle/__init__.py for the pinning story.  Nothing here is imported by
the product package.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

# ----------------------------------------------------------------------------------
# a2: Swin pad / cyclic shift / window partition / window reverse (bit-exact)
# ----------------------------------------------------------------------------------


def padded_size(n: int, ws: int) -> int:
    """HF:swin:609-615 — pad bottom/right up to a multiple of the window size."""
    return n + (ws - n % ws) % ws


def window_partition_np(x: np.ndarray, ws: int, shift: int) -> np.ndarray:
    """Pad -> roll(-shift) -> partition.  HF:swin:609-626 (maybe_pad, cyclic_shift),
    HF:swin:486-495 (window_partition), order of operations HF:swin:546-551.

    x: [B, H, W, C] (any dtype) -> [B * nWh * nWw, ws*ws, C]; window index is
    (b, wy, wx) row-major, token index inside a window is (ty, tx) row-major.
    Padded pixels are zero (F.pad with zeros, HF:swin:614)."""
    B, H, W, C = x.shape
    Hp, Wp = padded_size(H, ws), padded_size(W, ws)
    xp = np.zeros((B, Hp, Wp, C), dtype=x.dtype)
    xp[:, :H, :W] = x
    if shift > 0:
        xp = np.roll(xp, shift=(-shift, -shift), axis=(1, 2))
    nh, nw = Hp // ws, Wp // ws
    win = xp.reshape(B, nh, ws, nw, ws, C).transpose(0, 1, 3, 2, 4, 5)
    return np.ascontiguousarray(win.reshape(B * nh * nw, ws * ws, C))


def window_reverse_np(win: np.ndarray, B: int, H: int, W: int, ws: int, shift: int) -> np.ndarray:
    """Inverse of window_partition_np: reverse -> roll(+shift) -> crop.
    HF:swin:498-505 (window_reverse), HF:swin:560-566 (roll back, crop)."""
    C = win.shape[-1]
    Hp, Wp = padded_size(H, ws), padded_size(W, ws)
    nh, nw = Hp // ws, Wp // ws
    x = win.reshape(B, nh, nw, ws, ws, C).transpose(0, 1, 3, 2, 4, 5).reshape(B, Hp, Wp, C)
    if shift > 0:
        x = np.roll(x, shift=(shift, shift), axis=(1, 2))
    return np.ascontiguousarray(x[:, :H, :W])


def shift_region_ids_np(Hp: int, Wp: int, ws: int, shift: int) -> np.ndarray:
    """HF:swin:584-602 — region id h_region*3 + w_region on the padded grid."""
    h = np.arange(Hp)
    w = np.arange(Wp)
    hr = (h >= Hp - ws).astype(np.int64) + (h >= Hp - shift).astype(np.int64)
    wr = (w >= Wp - ws).astype(np.int64) + (w >= Wp - shift).astype(np.int64)
    return hr[:, None] * 3 + wr[None, :]


def shift_attn_mask_np(Hp: int, Wp: int, ws: int, shift: int) -> np.ndarray:
    """HF:swin:584-607 — [nW, N, N] float32 additive mask: 0 where the two tokens of a
    window share a shift region, -100 otherwise.  (mask[w, i, j] = id[j] - id[i] != 0)."""
    ids = shift_region_ids_np(Hp, Wp, ws, shift).astype(np.float32)[None, :, :, None]
    mw = window_partition_np(ids, ws, 0).reshape(-1, ws * ws)  # no roll on the id map
    diff = mw[:, None, :] - mw[:, :, None]
    return np.where(diff != 0, np.float32(-100.0), np.float32(0.0)).astype(np.float32)


def rel_position_index_np(ws: int) -> np.ndarray:
    """HF:swin:350-365 — [N*N] int64 index into the (2ws-1)^2 relative-bias table."""
    coords = np.stack(np.meshgrid(np.arange(ws), np.arange(ws), indexing="ij")).reshape(2, -1)
    rel = coords[:, :, None] - coords[:, None, :]
    rel = rel.transpose(1, 2, 0).copy()
    rel[:, :, 0] += ws - 1
    rel[:, :, 1] += ws - 1
    rel[:, :, 0] *= 2 * ws - 1
    return rel.sum(-1).reshape(-1).astype(np.int64)


# ----------------------------------------------------------------------------------
# a5: Swin window attention core (fp32)
# ----------------------------------------------------------------------------------


def rel_bias(rel_table: torch.Tensor, ws: int) -> torch.Tensor:
    """HF:swin:367-370 — gather the table into [heads, N, N]."""
    N = ws * ws
    idx = torch.from_numpy(rel_position_index_np(ws))
    return rel_table[idx].view(N, N, -1).permute(2, 0, 1).contiguous()


def window_attention_ref(q, k, v, rel_table, ws: int, shift_mask=None, scale=None):
    """HF:swin:373-398 (eager_attention_forward) + HF:swin:418-468 (bias/mask combine).

    q, k, v: [Bw, heads, N, d] fp32.  shift_mask: [nW, N, N] or None (window w of the
    batch uses mask[w % nW]).  Returns [Bw, N, heads*d]."""
    Bw, heads, N, d = q.shape
    if scale is None:
        scale = d ** -0.5
    s = torch.matmul(q, k.transpose(2, 3)) * scale
    s = s + rel_bias(rel_table, ws).unsqueeze(0)
    if shift_mask is not None:
        nW = shift_mask.shape[0]
        s = s + shift_mask.unsqueeze(1).unsqueeze(0).expand(Bw // nW, -1, -1, -1, -1).reshape(Bw, 1, N, N)
    p = torch.softmax(s, dim=-1, dtype=torch.float32).to(v.dtype)     # HF:swin:392
    o = torch.matmul(p, v)
    return o.transpose(1, 2).reshape(Bw, N, heads * d)


# ----------------------------------------------------------------------------------
# a8: multi-scale deformable attention sampling (fp32), explicit bilinear gather
# ----------------------------------------------------------------------------------


def _bilinear_corners(loc_x, loc_y, Hl: int, Wl: int):
    """Sampling-position arithmetic of upstream `ms_deform_attn_im2col_bilinear`
    (h = loc_y*H - 0.5, w = loc_x*W - 0.5; zero outside), which equals the oracle's
    grid_sample(align_corners=False, padding_mode='zeros') at HF:m2f:807,822-824."""
    h = loc_y * Hl - 0.5
    w = loc_x * Wl - 0.5
    inside = (h > -1) & (w > -1) & (h < Hl) & (w < Wl)
    h0 = torch.floor(h)
    w0 = torch.floor(w)
    lh = h - h0
    lw = w - w0
    hh = 1 - lh
    hw = 1 - lw
    h0i = h0.long()
    w0i = w0.long()
    out = []
    for dy, dx, wt in ((0, 0, hh * hw), (0, 1, hh * lw), (1, 0, lh * hw), (1, 1, lh * lw)):
        yy = h0i + dy
        xx = w0i + dx
        ok = inside & (yy >= 0) & (yy <= Hl - 1) & (xx >= 0) & (xx <= Wl - 1)
        idx = (yy.clamp(0, Hl - 1) * Wl + xx.clamp(0, Wl - 1))
        out.append((idx, wt * ok.to(wt.dtype)))
    return out


def msda_ref(value, spatial_shapes, sampling_locations, attention_weights):
    """HF:m2f:798-837 (multi_scale_deformable_attention) restated as an explicit
    4-tap gather, differentiable through torch autograd (the backward oracle).

    value [B, S, H, D]; spatial_shapes list[(H_l, W_l)]; sampling_locations
    [B, Q, H, L, P, 2] (x, y in [0,1]); attention_weights [B, Q, H, L, P]
    -> [B, Q, H*D]."""
    B, S, H, D = value.shape
    _, Q, _, L, P, _ = sampling_locations.shape
    start = 0
    acc = None
    for lvl, (Hl, Wl) in enumerate(spatial_shapes):
        vl = value[:, start:start + Hl * Wl].permute(0, 2, 1, 3)  # [B, H, HW, D]
        start += Hl * Wl
        loc = sampling_locations[:, :, :, lvl].permute(0, 2, 1, 3, 4)  # [B, H, Q, P, 2]
        aw = attention_weights[:, :, :, lvl].permute(0, 2, 1, 3)  # [B, H, Q, P]
        lx = loc[..., 0].reshape(B, H, Q * P)
        ly = loc[..., 1].reshape(B, H, Q * P)
        samp = 0
        for idx, wt in _bilinear_corners(lx, ly, Hl, Wl):
            g = torch.gather(vl, 2, idx.unsqueeze(-1).expand(B, H, Q * P, D))
            samp = samp + g * wt.unsqueeze(-1)
        contrib = (samp.view(B, H, Q, P, D) * aw.unsqueeze(-1)).sum(3)  # [B, H, Q, D]
        acc = contrib if acc is None else acc + contrib
    return acc.permute(0, 2, 1, 3).reshape(B, Q, H * D)


# ----------------------------------------------------------------------------------
# a11: mask head (query embedding x pixel embedding) + attention-mask derivation
# ----------------------------------------------------------------------------------


def mask_head_ref(mask_embed, pixel_embed, target_hw):
    """HF:m2f:2040-2056 — logits = einsum('bqc,bchw->bqhw'); the attention mask is
    bilinear(align_corners=False) resize to `target_hw`, sigmoid < 0.5 -> True=blocked.

    Returns (logits [B,Q,H,W] fp32, blocked bool [B,Q,h*w]); the head-repeat of
    HF:m2f:2053 is left to the consumer (it is a broadcast)."""
    logits = torch.einsum("bqc,bchw->bqhw", mask_embed, pixel_embed)
    am = F.interpolate(logits, size=target_hw, mode="bilinear", align_corners=False)
    blocked = (am.sigmoid().flatten(2) < 0.5)
    return logits, blocked


def unblock_full_rows(blocked: torch.Tensor) -> torch.Tensor:
    """HF:m2f:1912-1914 — rows blocked at every key are un-blocked entirely."""
    where = (blocked.sum(-1) != blocked.shape[-1])
    return blocked & where.unsqueeze(-1)


# ----------------------------------------------------------------------------------
# a10: masked cross-attention core (fp32)
# ----------------------------------------------------------------------------------


def masked_attention_ref(q, k, v, blocked, scale=None):
    """Core of nn.MultiheadAttention with a boolean attn_mask as the decoder calls it
    (HF:m2f:1644-1650): softmax(q k^T * d^-1/2 + (-inf where blocked)) v.

    q [B, H, Q, d], k/v [B, H, S, d], blocked [B, Q, S] (shared by all heads, already
    passed through `unblock_full_rows`).  Returns [B, Q, H*d]."""
    B, H, Q, d = q.shape
    if scale is None:
        scale = d ** -0.5
    s = torch.matmul(q * scale, k.transpose(-1, -2))
    s = s.masked_fill(blocked.unsqueeze(1), float("-inf"))
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, v)
    return o.permute(0, 2, 1, 3).reshape(B, Q, H * d)


# ----------------------------------------------------------------------------------
# sine position embedding and MSDA reference points
# ----------------------------------------------------------------------------------


def sine_pos_embed(B: int, H: int, W: int, num_feats: int, temperature: int = 10000,
                   scale: float = 2 * math.pi, dtype=torch.float32) -> torch.Tensor:
    """HF:m2f:864-904 with normalize=True and no mask -> [B, 2*num_feats, H, W]."""
    y = torch.arange(1, H + 1, dtype=dtype)[None, :, None].expand(B, H, W)
    x = torch.arange(1, W + 1, dtype=dtype)[None, None, :].expand(B, H, W)
    eps = 1e-6
    y = y / (y[:, -1:, :] + eps) * scale
    x = x / (x[:, :, -1:] + eps) * scale
    dim_t = torch.arange(num_feats, dtype=torch.int64).to(dtype)
    dim_t = temperature ** (2 * torch.div(dim_t, 2, rounding_mode="floor") / num_feats)
    px = x[:, :, :, None] / dim_t
    py = y[:, :, :, None] / dim_t
    px = torch.stack((px[:, :, :, 0::2].sin(), px[:, :, :, 1::2].cos()), dim=4).flatten(3)
    py = torch.stack((py[:, :, :, 0::2].sin(), py[:, :, :, 1::2].cos()), dim=4).flatten(3)
    return torch.cat((py, px), dim=3).permute(0, 3, 1, 2)


def reference_points(spatial_shapes, B: int, dtype=torch.float32) -> torch.Tensor:
    """HF:m2f:1127-1156 with all valid ratios 1 -> [B, S, L, 2] (x, y)."""
    refs = []
    for (Hl, Wl) in spatial_shapes:
        ry, rx = torch.meshgrid(torch.linspace(0.5, Hl - 0.5, Hl, dtype=dtype),
                                torch.linspace(0.5, Wl - 0.5, Wl, dtype=dtype), indexing="ij")
        ry = ry.reshape(-1)[None] / Hl
        rx = rx.reshape(-1)[None] / Wl
        refs.append(torch.stack((rx, ry), -1))
    r = torch.cat(refs, 1)
    L = len(spatial_shapes)
    return r[:, :, None].expand(B, -1, L, -1).contiguous()
