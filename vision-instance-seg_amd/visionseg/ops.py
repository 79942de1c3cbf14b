"""PyTorch-facing operators over the HIP C ABI (autograd Functions + functional API).

Mirrors the operator surface the reference's path reaches:
  * `MSDeformAttnFunction.apply(value, spatial_shapes, level_start_index,
    sampling_locations, attention_weights, im2col_step)` — same argument meaning as the
    upstream MaskDINO/Mask2Former `ops/functions/ms_deform_attn_func.py` wrapper; the
    functional `ms_deform_attn(value, spatial_shapes, sampling_locations,
    attention_weights)` has the argument order of the oracle's
    `multi_scale_deformable_attention` (HF:m2f:798).
  * `window_partition(x, window, shift)` / `window_reverse(windows, H, W, window, shift)`
    fuse F.pad + torch.roll + HF `window_partition`/`window_reverse` (HF:swin:486-505,
    546-566, 609-626).

Every op runs on the current HIP stream of its inputs' device and raises if the
kernels library is missing or an input is on the CPU.
"""
from __future__ import annotations

import collections
import contextlib
import ctypes
import os

import torch
import torch.nn.functional as F

from . import _lib as L
from .profiling import timed


def _shapes_list(spatial_shapes):
    if isinstance(spatial_shapes, torch.Tensor):
        spatial_shapes = spatial_shapes.tolist()  # host sync; pass a list on hot paths
    return [(int(h), int(w)) for h, w in spatial_shapes]


def _level_arrays(shapes):
    import ctypes
    n = len(shapes)
    sh = (ctypes.c_int64 * (2 * n))(*[v for hw in shapes for v in hw])
    st = []
    s = 0
    for h, w in shapes:
        st.append(s)
        s += h * w
    starts = (ctypes.c_int64 * n)(*st)
    return sh, starts, s


# MSDA backward variant (A/B switch, VS_MSDA_BWD): "carry" (default; f32 atomics into
# grad_value: the MFMA query-tile product for bf16, the binned query-tile kernel for f32,
# then a cast) or "tiled" (deterministic: grad_value by destination tiles with plain LDS
# read-modify-write, no float atomics, written once in the value dtype; pays for its
# inverse index with integer atomics, ~30 G/s on gfx950: at 4x1024^2, tools/kbench.py
# --only msda, smooth offsets, 4.4 ms against the binned kernel's 0.96 ms).
_MSDA_BWD = os.environ.get("VS_MSDA_BWD", "carry")


class MSDeformAttnFunction(torch.autograd.Function):
    """value [B,S,H,32] (f32/bf16), sampling_locations [B,Q,H,L,P,2], attention_weights
    [B,Q,H,L,P] (f32) -> [B,Q,H*32] in value's dtype."""

    @staticmethod
    def forward(ctx, value, spatial_shapes, level_start_index, sampling_locations, attention_weights,
                im2col_step=64):
        shapes = _shapes_list(spatial_shapes)
        L.require_hip(value, sampling_locations, attention_weights)
        value = value.contiguous()
        loc = sampling_locations.float().contiguous()
        aw = attention_weights.float().contiguous()
        B, S, H, D = value.shape
        _, Q, _, Lv, P, _ = loc.shape
        tot = sum(h * w for h, w in shapes)
        if tot != S:
            raise ValueError(f"spatial shapes cover {tot} positions, value has {S}")
        sh_t, st_t = L.level_tensors(shapes)
        nb = (value.numel() + B * Q * H * D) * value.element_size() + (loc.numel() + aw.numel()) * 4
        with timed("msda_fwd", value, bytes_=nb, flops=2.0 * aw.numel() * (4 * D + D)):
            out = L.tops().msda_fwd(value, sh_t, st_t, loc, aw, int(im2col_step or 64))
        ctx.shapes = shapes
        ctx.save_for_backward(value, loc, aw)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        value, loc, aw = ctx.saved_tensors
        B, S, H, D = value.shape
        _, Q, _, Lv, P, _ = loc.shape
        g = grad_out.to(value.dtype).contiguous()
        if _MSDA_BWD == "tiled":
            gl = torch.empty_like(loc)
            ga = torch.empty_like(aw)
            sh, st, _ = _level_arrays(ctx.shapes)
            # grad_value by destination tiles (csrc/msda.hip msda_tile_*): atomic-free,
            # written once in value's dtype
            gv = torch.empty_like(value)
            nbytes = int(L.lib().vs_msda_backward_tiled_workspace_bytes(B, H, Lv, Q, P, sh))
            if nbytes < 0:
                raise ValueError("bad sizes for the tiled MSDA backward")
            ws = torch.empty(nbytes, device=value.device, dtype=torch.uint8)
            nb = (2 * value.numel() + g.numel()) * value.element_size() + (loc.numel() + aw.numel()) * 8
            with timed("msda_bwd", value, bytes_=nb, flops=2.0 * aw.numel() * 10 * D):
                L.check(L.lib().vs_msda_backward_tiled(L.dtype_code(value), L.ptr(value), sh, st, L.ptr(loc),
                                                       L.ptr(aw), L.ptr(g), L.ptr(gv), L.ptr(gl), L.ptr(ga),
                                                       L.ptr(ws), B, S, H, D, Lv, Q, P, L.stream(value)),
                        "msda_backward_tiled")
            return gv, None, None, gl, ga, None
        sh_t, st_t = L.level_tensors(ctx.shapes)
        nb = (value.numel() + g.numel()) * value.element_size() + (loc.numel() + aw.numel()) * 8 + value.numel() * 4
        with timed("msda_bwd", value, bytes_=nb, flops=2.0 * aw.numel() * 10 * D):
            gv, gl, ga = L.tops().msda_bwd(value, sh_t, st_t, loc, aw, g, 64, True)
        return gv.to(value.dtype), None, None, gl, ga, None


def ms_deform_attn(value, spatial_shapes, sampling_locations, attention_weights):
    """Functional form with the oracle's argument order (HF:m2f:798)."""
    shapes = _shapes_list(spatial_shapes)
    return MSDeformAttnFunction.apply(value, shapes, None, sampling_locations, attention_weights, 64)


class MSDAPrepFunction(torch.autograd.Function):
    """(offsets [B,Q,H*L*P*2], logits [B,Q,H*L*P], ref [B,Q,L,2] f32) -> (sampling
    locations [B,Q,H,L,P,2] f32, attention weights [B,Q,H,L,P] f32) as
    `ref + offsets.float() / (W_l, H_l)` and `softmax(logits.float())` over L*P
    (HF:m2f:994-1002; csrc/msda_prep.hip).  ref gets no gradient (a buffer).
    logits=None: `off` is the packed projection [B,Q,H*L*P*3] (offsets then logits, one
    GEMM's output); its gradient is then written as one tensor (the kernel takes row
    strides), not as two slice gradients that autograd zero-fills and adds."""

    @staticmethod
    def forward(ctx, off, logits, ref, shapes, heads, points):
        nl = len(shapes)
        lp = nl * points
        ctx.packed = logits is None
        if ctx.packed:
            if off.shape[-1] != heads * lp * 3:
                raise ValueError(f"packed projection width {off.shape[-1]} != {heads * lp * 3}")
            off, logits = off[..., :heads * lp * 2], off[..., heads * lp * 2:]
        L.require_hip(off, logits, ref)
        B, Q = off.shape[0], off.shape[1]
        if off.dtype != logits.dtype:
            raise ValueError("offsets / logits dtypes differ")
        if off.shape[-1] != heads * lp * 2 or logits.shape[-1] != heads * lp:
            raise ValueError(f"projection widths {off.shape[-1]}, {logits.shape[-1]} != {heads * lp * 2}, "
                             f"{heads * lp}")
        n_off, n_lg = heads * lp * 2, heads * lp
        off2 = off.reshape(B * Q, n_off) if off.stride(-1) == 1 else off.contiguous().view(B * Q, n_off)
        lg2 = logits.reshape(B * Q, n_lg) if logits.stride(-1) == 1 else logits.contiguous().view(B * Q, n_lg)
        if B * Q and (off2.stride(1) != 1 or lg2.stride(1) != 1 or off2.stride(0) < n_off or lg2.stride(0) < n_lg):
            off2, lg2 = off2.contiguous(), lg2.contiguous()
        ref = ref.float()
        if tuple(ref.shape) != (B, Q, nl, 2):
            raise ValueError(f"reference points {tuple(ref.shape)} != {(B, Q, nl, 2)}")
        if (ref.stride(3) != 1 or ref.stride(2) != 2 or ref.stride(1) != 2 * nl or ref.stride(0) % 2
                or ref.data_ptr() % 8):
            ref = ref.contiguous()
        loc = torch.empty(B, Q, heads, nl, points, 2, device=off.device, dtype=torch.float32)
        aw = torch.empty(B, Q, heads, nl, points, device=off.device, dtype=torch.float32)
        sh, _, _ = _level_arrays(shapes)
        with timed("msda_prep_fwd", off, bytes_=(off.numel() + logits.numel()) * off.element_size()
                   + (loc.numel() + aw.numel()) * 4):
            L.check(L.lib().vs_msda_prep_forward(L.dtype_code(off), L.ptr(off2), max(off2.stride(0), n_off),
                                                 L.ptr(lg2), max(lg2.stride(0), n_lg), L.ptr(ref), ref.stride(0), sh, L.ptr(loc), L.ptr(aw),
                                                 B, Q, heads, nl, points, L.stream(off)), "msda_prep_forward")
        ctx.save_for_backward(aw)
        ctx.geom = (B, Q, heads, nl, points, off.dtype, tuple(shapes))
        return loc, aw

    @staticmethod
    def backward(ctx, gloc, gaw):
        (aw,) = ctx.saved_tensors
        B, Q, heads, nl, points, dt, shapes = ctx.geom
        lp = nl * points
        gloc = aw.new_zeros(*aw.shape, 2) if gloc is None else gloc.float().contiguous()
        gaw = torch.zeros_like(aw) if gaw is None else gaw.float().contiguous()
        if ctx.packed:
            gproj = torch.empty(B, Q, heads * lp * 3, device=aw.device, dtype=dt)
            goff, glg = gproj[..., :heads * lp * 2], gproj[..., heads * lp * 2:]
        else:
            goff = torch.empty(B, Q, heads * lp * 2, device=aw.device, dtype=dt)
            glg = torch.empty(B, Q, heads * lp, device=aw.device, dtype=dt)
        sh, _, _ = _level_arrays(shapes)
        with timed("msda_prep_bwd", aw, bytes_=(gloc.numel() + gaw.numel() + aw.numel()) * 4
                   + (goff.numel() + glg.numel()) * goff.element_size()):
            L.check(L.lib().vs_msda_prep_backward(L.dtype_code(goff), L.ptr(gloc), L.ptr(gaw), L.ptr(aw), sh,
                                                  L.ptr(goff), goff.stride(1), L.ptr(glg), glg.stride(1), B, Q, heads,
                                                  nl, points, L.stream(aw)), "msda_prep_backward")
        if ctx.packed:
            return gproj, None, None, None, None, None
        return goff, glg, None, None, None, None


def msda_prep(offsets, logits, ref, spatial_shapes, heads: int, points: int):
    """Sampling locations and attention weights of MSDeformAttn from its two projections
    (see MSDAPrepFunction; logits=None: `offsets` is the packed projection)."""
    return MSDAPrepFunction.apply(offsets, logits, ref, _shapes_list(spatial_shapes), int(heads), int(points))


def _padded(n, ws):
    return n + (ws - n % ws) % ws


class _WindowPartition(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ws, shift):
        L.require_hip(x)
        x = x.contiguous()
        B, H, W, C = x.shape
        out = _window_partition_raw(x, ws, shift)
        ctx.meta = (B, H, W, C, ws, shift)
        return out

    @staticmethod
    def backward(ctx, g):
        B, H, W, C, ws, shift = ctx.meta
        return _window_reverse_raw(g.contiguous(), B, H, W, C, ws, shift), None, None


def _window_reverse_raw(win, B, H, W, C, ws, shift):
    with timed("window_reverse", win, bytes_=(win.numel() + B * H * W * C) * win.element_size()):
        return L.tops().swin_window_bwd(win, B, H, W, ws, shift)


def _window_partition_raw(x, ws, shift):
    B, H, W, C = x.shape
    n_out = B * _padded(H, ws) * _padded(W, ws) * C
    with timed("window_partition", x, bytes_=(x.numel() + n_out) * x.element_size()):
        return L.tops().swin_window_fwd(x, ws, shift)


class _WindowReverse(torch.autograd.Function):
    @staticmethod
    def forward(ctx, win, B, H, W, ws, shift):
        L.require_hip(win)
        win = win.contiguous()
        C = win.shape[-1]
        ctx.meta = (ws, shift)
        return _window_reverse_raw(win, B, H, W, C, ws, shift)

    @staticmethod
    def backward(ctx, g):
        ws, shift = ctx.meta
        return _window_partition_raw(g.contiguous(), ws, shift), None, None, None, None, None


def window_partition(x, window: int, shift: int = 0):
    """x [B,H,W,C] -> [B*nW, window^2, C]: zero pad to a multiple of `window`, roll by
    -shift, partition (HF:swin:546-551).  Bit-exact."""
    return _WindowPartition.apply(x, int(window), int(shift))


def window_reverse(windows, batch: int, height: int, width: int, window: int, shift: int = 0):
    """Inverse of window_partition: [B*nW, window^2, C] -> [B,H,W,C] (HF:swin:558-566)."""
    return _WindowReverse.apply(windows, int(batch), int(height), int(width), int(window), int(shift))


def table_grad_from_partials(part):
    """f32 partials [P, heads, T] of the relative-position-table gradient (one per window,
    from the window-attention backward) -> their sum [heads, T] through the column-sum
    kernel (csrc/norm.hip; ATen's dim-0 sum took 82 us for the 5476 x 507 partials of a C2
    stage-1 block).  Rows of heads*T % 8 != 0 are summed 8 partial rows at a time as one
    row of 8 heads*T columns, the remainder rows (< 8) added after."""
    P, H, T = part.shape
    R = H * T
    flat = part.reshape(P, R)
    if R % 8 == 0 and R <= 16384:
        return column_sum(flat).view(H, T)
    q = P // 8
    if q == 0 or 8 * R > 16384:
        return part.sum(0)
    s = column_sum(flat[:8 * q].reshape(q, 8 * R)).view(8, R).sum(0)
    if P % 8:
        s = s + flat[8 * q:].sum(0)
    return s.view(H, T)


def rel_table_grad(part, dtype):
    """f32 partials [P, heads, T] of the relative-position-table gradient -> the table
    gradient [T, heads] in `dtype` (the table's layout): one column-sum pass over the rows
    folded to a multiple-of-8 width and one fold / transpose / cast pass
    (vs_rel_table_grad); table_grad_from_partials + transpose + cast (4-5 launches) where
    the rows do not fold (P % F != 0)."""
    P, H, T = part.shape
    R = H * T
    F = next(f for f in (1, 2, 4, 8) if (f * R) % 8 == 0)
    if P % F or F * R > 16384 or dtype not in (torch.float32, torch.bfloat16):
        return table_grad_from_partials(part).t().contiguous().to(dtype)
    part = part.contiguous()
    out = torch.empty(T, H, device=part.device, dtype=dtype)
    ws = torch.empty(int(L.lib().vs_rel_table_grad_workspace_bytes(P, H, T)), device=part.device, dtype=torch.uint8)
    L.check(L.lib().vs_rel_table_grad(L.dtype_code(out), L.ptr(part), L.ptr(out), L.ptr(ws), P, H, T,
                                      L.stream(part)), "rel_table_grad")
    return out


class WindowAttentionFunction(torch.autograd.Function):
    """Swin window attention core with the relative-position bias and the shifted-window
    mask fused (HF:swin:373-398, 418-468, 584-607).

    qkv [Bw, N, 3*C] (fused q;k;v Linear output of the partitioned windows, C =
    heads*32), rel_table [(2ws-1)^2, heads] -> [Bw, N, C].  fp8=True (bf16 qkv, window^2
    <= 160): the e4m3 MFMA path of config C5 (vs_window_attn_forward_fp8)."""

    @staticmethod
    def forward(ctx, qkv, rel_table, heads, window, shift, nwin_h, nwin_w, scale, fp8=False):
        L.require_hip(qkv, rel_table)
        if fp8 and (qkv.dtype != torch.bfloat16 or window * window > 160):
            raise ValueError(f"fp8 window attention needs bf16 qkv and window^2 <= 160 (got {qkv.dtype}, "
                             f"window {window})")
        qkv = qkv.contiguous()
        table = rel_table.float().contiguous()
        Bw, N, C3 = qkv.shape
        C = C3 // 3
        if C != heads * 32 or N != window * window:
            raise ValueError(f"qkv {tuple(qkv.shape)} does not match heads={heads} (x32) window={window}")
        with timed("window_attn_fwd_fp8" if fp8 else "window_attn_fwd", qkv,
                   bytes_=(qkv.numel() + Bw * N * C) * qkv.element_size() + Bw * heads * N * 4,
                   flops=4.0 * Bw * heads * N * N * 32):
            out, lse = L.tops().win_attn_fwd(qkv, table, heads, window, shift, nwin_h, nwin_w, float(scale),
                                             bool(fp8))
        ctx.meta = (heads, window, shift, nwin_h, nwin_w, float(scale), rel_table.dtype, bool(fp8))
        ctx.save_for_backward(qkv, table, out, lse)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        qkv, table, out, lse = ctx.saved_tensors
        heads, window, shift, nwin_h, nwin_w, scale, tdtype, fp8 = ctx.meta
        Bw, N, C3 = qkv.shape
        g = grad_out.to(qkv.dtype).contiguous()
        with timed("window_attn_bwd_fp8" if fp8 else "window_attn_bwd", qkv,
                   bytes_=(3 * qkv.numel() + 2 * out.numel()) * qkv.element_size(),
                   flops=10.0 * Bw * heads * N * N * 32):
            gqkv, part = L.tops().win_attn_bwd(qkv, table, out, lse, g, heads, window, shift, nwin_h, nwin_w,
                                               scale, bool(fp8), True)
        gtable = rel_table_grad(part, tdtype)
        return gqkv, gtable, None, None, None, None, None, None, None


class WindowAttentionImageFunction(torch.autograd.Function):
    """WindowAttentionFunction with the window reverse folded into the kernels
    (vs_window_attn_forward_image / _backward_image): the output (and its gradient) in the
    image layout [B, H, W, C] -- un-rolled, padding cropped -- so neither the reverse nor
    the partition of the output gradient runs as its own pass over HBM.  bf16 MFMA / fp8
    kernels; qkv and lse stay in the window layout."""

    @staticmethod
    def forward(ctx, qkv, rel_table, heads, window, shift, nwin_h, nwin_w, height, width, scale, fp8=False,
                table32=None):
        """table32: rel_table's values already in f32 (not differentiated: the gradient goes to
        rel_table)."""
        L.require_hip(qkv, rel_table)
        qkv = qkv.contiguous()
        table = table32.contiguous() if table32 is not None else rel_table.float().contiguous()
        Bw, N, C3 = qkv.shape
        if C3 != 3 * heads * 32 or N != window * window:
            raise ValueError(f"qkv {tuple(qkv.shape)} does not match heads={heads} (x32) window={window}")
        with timed("window_attn_fwd_fp8" if fp8 else "window_attn_fwd", qkv,
                   bytes_=(qkv.numel() + Bw * N * C3 // 3) * qkv.element_size() + Bw * heads * N * 4,
                   flops=4.0 * Bw * heads * N * N * 32):
            out, lse = L.tops().win_attn_fwd_img(qkv, table, heads, window, shift, nwin_h, nwin_w, height, width,
                                                 float(scale), bool(fp8))
        ctx.meta = (heads, window, shift, nwin_h, nwin_w, height, width, float(scale), rel_table.dtype, bool(fp8))
        ctx.save_for_backward(qkv, table, out, lse)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        qkv, table, out, lse = ctx.saved_tensors
        heads, window, shift, nwin_h, nwin_w, height, width, scale, tdtype, fp8 = ctx.meta
        Bw, N, C3 = qkv.shape
        g = grad_out.to(qkv.dtype).contiguous()
        with timed("window_attn_bwd_fp8" if fp8 else "window_attn_bwd", qkv,
                   bytes_=(3 * qkv.numel() + 2 * Bw * N * C3 // 3) * qkv.element_size(),
                   flops=10.0 * Bw * heads * N * N * 32):
            gqkv, part = L.tops().win_attn_bwd_img(qkv, table, out, lse, g, heads, window, shift, nwin_h, nwin_w,
                                                   height, width, scale, bool(fp8))
        gtable = rel_table_grad(part, tdtype)
        return gqkv, gtable, None, None, None, None, None, None, None, None, None, None


def window_attention_image(qkv, rel_table, heads: int, window: int, shift: int, batch: int, height: int,
                           width: int, scale: float | None = None, fp8: bool = False, table32=None):
    """Window attention of the partitioned qkv [B*nW, ws^2, 3C] with the output in the image
    layout [B, H, W, C] (= window_reverse(window_attention(...))): the reverse folded into
    the bf16 kernels; the f32 parity mode (and VS_WIN_ATTN_SCALAR) keeps the separate
    reverse."""
    if scale is None:
        scale = 32 ** -0.5
    nwin_h, nwin_w = -(-height // window), -(-width // window)
    if (qkv.is_cuda and qkv.dtype == torch.bfloat16 and window * window <= 160
            and os.environ.get("VS_WIN_ATTN_SCALAR", "0") == "0"):
        return WindowAttentionImageFunction.apply(qkv, rel_table, int(heads), int(window), int(shift), nwin_h, nwin_w,
                                                  int(height), int(width), float(scale), bool(fp8), table32)
    o = window_attention(qkv, rel_table, heads, window, shift, nwin_h, nwin_w, scale, fp8)
    return window_reverse(o, batch, height, width, window, shift)


def window_attention(qkv, rel_table, heads: int, window: int, shift: int, nwin_h: int, nwin_w: int,
                     scale: float | None = None, fp8: bool = False):
    if scale is None:
        scale = 32 ** -0.5
    return WindowAttentionFunction.apply(qkv, rel_table, int(heads), int(window), int(shift), int(nwin_h),
                                         int(nwin_w), float(scale), bool(fp8))


class MaskHeadFunction(torch.autograd.Function):
    """logits [B,Q,H,W] f32 = einsum('bqc,bchw->bqhw') with the pixel embedding given
    channels-last (HF:m2f:2051).  Forward: hand-written MFMA kernel.  Backward (bf16):
    one fused MFMA kernel producing dE = dL.P and dP = dL^T.E in a single pass over dL;
    f32 parity mode uses vendor GEMMs for the backward."""

    @staticmethod
    def forward(ctx, mask_embed, pixel_nhwc, height, width, sink=None):
        L.require_hip(mask_embed, pixel_nhwc)
        ctx.sink = sink
        E = mask_embed.contiguous()
        P = pixel_nhwc.to(E.dtype).contiguous()
        B, Q, C = E.shape
        if P.shape != (B, height * width, C):
            raise ValueError(f"pixel embedding {tuple(P.shape)} != {(B, height * width, C)}")
        with timed("mask_head_fwd", E, bytes_=(E.numel() + P.numel()) * E.element_size() + B * Q * height * width * 4,
                   flops=2.0 * B * Q * C * height * width):
            out = L.tops().mask_head_fwd(E, P, height, width)
        ctx.save_for_backward(E, P)
        ctx.pdtype = pixel_nhwc.dtype
        return out

    @staticmethod
    def backward(ctx, g):
        E, P = ctx.saved_tensors
        B, Q, C = E.shape
        N = P.shape[1]
        sink = ctx.sink
        if E.dtype == torch.bfloat16 and C in (128, 256):
            # the fused kernel takes <= 128 queries: more (MaskDINO's 300 + denoising
            # queries) run as chunks of 128 that accumulate dP in place
            acc = sink is not None and sink.buf is not None
            if sink is not None and not acc:
                sink.buf = torch.empty_like(P)
            gP = sink.buf if sink is not None else torch.empty_like(P)
            nb = g.numel() * 4 + (E.numel() * 2 + P.numel() * 2) * 2 + (P.numel() * 2 if acc else 0)
            with timed("mask_head_bwd", E, bytes_=nb, flops=4.0 * B * Q * C * N):
                gE = L.tops().mask_head_bwd(g, E, P, gP, bool(acc))
            if sink is not None:
                return gE, None, None, None, None
            return gE, gP.to(ctx.pdtype), None, None, None
        # f32 parity mode (and shapes outside the fused kernel): vendor GEMMs
        gl = g.reshape(B, Q, -1).to(E.dtype)
        gE = torch.bmm(gl, P) if ctx.needs_input_grad[0] else None
        gP = torch.bmm(gl.transpose(1, 2), E).to(ctx.pdtype) if ctx.needs_input_grad[1] else None
        if sink is not None and gP is not None:
            sink.buf = gP if sink.buf is None else sink.buf + gP
            gP = None
        return gE, gP, None, None, None


def mask_head(mask_embed, pixel_nhwc, height: int, width: int, sink=None):
    """sink (GradSink): the pixel-embedding gradient of every call sharing the sink is
    summed in one buffer inside the backward kernel (pass `pixel_nhwc` through
    `sink.source(...)` once); without a sink each call returns its own gradient."""
    out = MaskHeadFunction.apply(mask_embed, pixel_nhwc, int(height), int(width), sink)
    # the factors, for losses that only read a few rows of the logits (matched_point_logits)
    out._vs_src = (mask_embed, pixel_nhwc)
    return out


def mask_head_factors(masks_list):
    """(E [S,B,Q,C], P [B,HW,C]) if every logits tensor came from `mask_head` with one
    shared pixel embedding, else None."""
    srcs = [getattr(m, "_vs_src", None) for m in masks_list]
    if not srcs or any(s is None for s in srcs) or any(s[1] is not srcs[0][1] for s in srcs):
        return None
    if all(len(s) == 3 and s[0] is srcs[0][0] and s[2] == i for i, s in enumerate(srcs)) \
            and srcs[0][0].shape[0] == len(srcs):
        return srcs[0][0], srcs[0][1]        # (E [S,B,Q,C], P): the decoder's batched heads
    return torch.stack([s[0] for s in srcs]), srcs[0][1]


class MatchedPointLogitsFunction(torch.autograd.Function):
    """Point samples of the matched mask logits, differentiable w.r.t. the mask head's
    factors instead of the logits.

    The set criterion's mask losses (HF:m2f:671-724) read the logits of the MATCHED
    (step, image, target) pairs at sampled points only, so the gradient of the full
    [B, Q, H, W] logits of every decoder step is zero except on <= Kc of Q query rows.
    Autograd through the logits would zero-fill and scatter those full-size gradients and
    run the mask-head backward over all Q rows, once per step.  Here the backward scatters
    the point gradients into the matched maps only (G [B, S*Kc, H, W]: vs_point_scatter,
    LDS bands, no global atomics) and applies the einsum's adjoint to them directly, all
    steps at once:
        dE[s, b, q_sk] = G[b, (s, k)] . P[b]                     ([S*Kc, HW] x [HW, C])
        dP[b]          = sum_{s,k} G[b, (s, k)]^T E[s, b, q_sk]  ([HW, S*Kc] x [S*Kc, C])
    -- for bf16 the fused mask-head backward kernel with the S*Kc pairs as its queries
    (one pass over G), else two batched GEMMs.
    pred: the matched maps [S*B*Kc, 1, H, W] (detached), coords [S*B*Kc, n, 2] in [0, 1),
    qsel int64 [S, B, Kc], E [S, B, Q, C], P [B, H*W, C] -> logits at the points [S*B*Kc, n]."""

    @staticmethod
    def forward(ctx, pred, coords, qsel, E, P):
        grid = 2.0 * coords.unsqueeze(2) - 1.0
        out = point_sample(pred, coords)
        ctx.save_for_backward(grid, qsel, E, P)
        ctx.map_shape = tuple(pred.shape)
        return out

    @staticmethod
    def backward(ctx, g):
        grid, qsel, E, P = ctx.saved_tensors
        S, B, Kc = qsel.shape
        N, _, H, W = ctx.map_shape
        Q, C = E.shape[2], E.shape[3]
        n = g.shape[-1]
        # point gradients -> dense maps of the matched pairs, [B, S*Kc, H, W] f32
        # (csrc/mask_head.hip point_scatter_kernel: LDS bands, no global atomics)
        G = torch.empty(B, S * Kc, H, W, device=g.device, dtype=torch.float32)
        gc = g.float().contiguous()
        gr = grid.contiguous()
        with timed("point_scatter", gc, bytes_=gc.numel() * 12 + G.numel() * 4):
            L.check(L.lib().vs_point_scatter(L.ptr(gc), L.ptr(gr), L.ptr(G), S, B, Kc, n, H, W, L.stream(gc)),
                    "point_scatter")
        bq = qsel.transpose(0, 1)                                                       # [B, S, Kc]
        Esel = torch.gather(E.transpose(0, 1), 2, bq[..., None].expand(B, S, Kc, C)).reshape(B, S * Kc, C)
        if P.dtype == torch.bfloat16 and C in (128, 256) and S * Kc <= 128:
            # the fused mask-head backward with the S*Kc matched pairs as its queries:
            # dE_sel = G.P and dP = G^T.E_sel in one pass over G
            dP = torch.empty_like(P)
            Ec = Esel.contiguous()
            with timed("mask_head_bwd", Ec, bytes_=G.numel() * 4 + (Ec.numel() * 2 + P.numel() * 2) * 2,
                       flops=4.0 * B * S * Kc * C * H * W):
                dEs = L.tops().mask_head_bwd(G, Ec, P, dP, False)
        else:
            Gb = G.view(B, S * Kc, H * W).to(P.dtype)
            dEs = torch.bmm(Gb, P)                                                      # [B, S*Kc, C]
            dP = torch.bmm(Gb.transpose(1, 2), Esel.to(P.dtype))                        # [B, HW, C]
        dE = torch.zeros(S, B, Q, C, device=E.device, dtype=E.dtype)
        dE.scatter_add_(2, qsel[..., None].expand(S, B, Kc, C), dEs.view(B, S, Kc, C).transpose(0, 1).to(E.dtype))
        return None, None, None, dE, dP.to(P.dtype)


class FactoredLogits:
    """Mask logits of decoder step `s` kept as the mask head's factors, never materialised
    at full resolution: L[b, q, n] = E[s, b, q, :] . F[b, n, :] (E [S, B, Q, C] the batched
    heads' mask embeddings with their autograd history, F [B, H*W, C] the channels-last
    pixel embedding).  The training step reads the logits only through linear resamplings
    (the matcher's points, the attention masks' resize) and the matched rows, each computed
    from the factors (csrc/match_factors.hip, `matched_maps`); `materialize()` gives the
    full tensor for any other consumer."""

    def __init__(self, E, F, s: int, height: int, width: int):
        self.E, self.F, self.s, self.H, self.W = E, F, int(s), int(height), int(width)
        self._vs_src = (E, F, self.s)

    @property
    def shape(self):
        return torch.Size((self.E.shape[1], self.E.shape[2], self.H, self.W))

    @property
    def device(self):
        return self.E.device

    dtype = torch.float32

    def detach(self):
        return FactoredLogits(self.E.detach(), self.F.detach(), self.s, self.H, self.W)

    def materialize(self):
        return mask_head(self.E[self.s], self.F, self.H, self.W)

    def float(self):
        return self               # the logits are f32 already (the mask head's output dtype)


def factored(masks_list) -> bool:
    """True when `masks_list` is exactly the decoder's factored output: every entry a
    FactoredLogits over the SAME factors (E, F), entry s holding step s, one entry per step
    of E.  The consumers (SetCriterion.match, matched_maps) read E and F from the first
    entry for every step, so a subset or a reordered list must be materialised instead."""
    if not masks_list or not all(isinstance(m, FactoredLogits) for m in masks_list):
        return False
    m0 = masks_list[0]

    def same(a, b):          # the same tensor, or a detached view of it (FactoredLogits.detach)
        return a.data_ptr() == b.data_ptr() and a.shape == b.shape and a.stride() == b.stride()

    return (int(m0.E.shape[0]) == len(masks_list)
            and all(same(m.E, m0.E) and same(m.F, m0.F) and m.s == i for i, m in enumerate(masks_list)))


def materialize_masks(masks_list):
    return [m.materialize() if isinstance(m, FactoredLogits) else m for m in masks_list]


def feature_resize_hilo(F_nhwc, height: int, width: int, th: int, tw: int):
    """Bilinear (align_corners=False) resize of the channels-last pixel embedding bf16
    [B, H*W, C] to [B, th*tw, 2C] as hi | lo bf16 pairs (csrc/match_factors.hip): E . (hi + lo)
    = the resized logits of HF:m2f:2049-2055 to ~2^-17 relative."""
    L.require_hip(F_nhwc)
    Fc = F_nhwc.contiguous()
    if Fc.dtype != torch.bfloat16:
        raise TypeError("feature_resize_hilo takes the bf16 pixel embedding")
    B, N, C = Fc.shape
    if N != height * width:
        raise ValueError("feature_resize_hilo: pixel embedding is not [B, H*W, C]")
    out = torch.empty(B, th * tw, 2 * C, device=Fc.device, dtype=torch.bfloat16)
    with timed("feature_resize_hilo", Fc, bytes_=out.numel() * 2 + min(Fc.numel(), out.numel() * 2) * 2):
        L.check(L.lib().vs_feature_resize_hilo(L.ptr(Fc), L.ptr(out), B, int(height), int(width), C, int(th), int(tw),
                                               L.stream(Fc)), "feature_resize_hilo")
    return out


def level_bitmask_hilo(E, level_features, height: int, width: int):
    """Attention bitmask (attn_bitmask's format and rule) of E bf16 [B, Q, C] . resize(F) at a
    level of height x width keys, resize(F) = feature_resize_hilo's [B, h*w, 2C] pair; the
    level logits are never stored (csrc/match_factors.hip level_bitmask_kernel)."""
    Ec, Fl = E.contiguous(), level_features.contiguous()
    L.require_hip(Ec, Fl)
    B, Q, C = Ec.shape
    if Ec.dtype != torch.bfloat16 or tuple(Fl.shape) != (B, height * width, 2 * C):
        raise ValueError("level_bitmask_hilo: bf16 E [B, Q, C] and features [B, h*w, 2C] expected")
    words = torch.empty(B, Q, (height * width + 31) // 32, device=Ec.device, dtype=torch.int32)
    with timed("level_bitmask", Ec, bytes_=Fl.numel() * 2 + words.numel() * 4, flops=4.0 * B * Q * C * height * width):
        L.check(L.lib().vs_level_bitmask_hilo(L.ptr(Ec), L.ptr(Fl), L.ptr(words), B, Q, C, int(height), int(width),
                                              L.stream(Ec)), "level_bitmask_hilo")
    return words


def feature_sample_hilo(F_nhwc, height: int, width: int, grid):
    """The pixel embedding bf16 [B, H*W, C] at grid points f32 [B, P, 2] in [-1, 1]
    (grid_sample bilinear, zeros padding, align_corners=False) -> [B, P, 2C] hi | lo bf16."""
    L.require_hip(F_nhwc, grid)
    Fc = F_nhwc.contiguous()
    g = grid.float().contiguous()
    B, N, C = Fc.shape
    P = int(g.shape[1])
    if Fc.dtype != torch.bfloat16 or N != height * width or tuple(g.shape) != (B, P, 2):
        raise ValueError("feature_sample_hilo: bf16 [B, H*W, C] features and [B, P, 2] grid expected")
    out = torch.empty(B, P, 2 * C, device=Fc.device, dtype=torch.bfloat16)
    with timed("feature_sample_hilo", Fc, bytes_=out.numel() * 2 * 3):
        L.check(L.lib().vs_feature_sample_hilo(L.ptr(Fc), L.ptr(g), L.ptr(out), B, int(height), int(width), C, P,
                                               L.stream(Fc)), "feature_sample_hilo")
    return out


def match_cost_factors(E, point_features, probs, target_classes, target_labels, mask_weight, class_weight,
                       dice_weight):
    """Hungarian-matcher cost for all decoder steps from the mask head's factors
    (csrc/match_factors.hip): E bf16 [S, B, Q, C], point_features = feature_sample_hilo at
    the matcher's points [B, P, 2C], probs f32 [S, B, Q, C+1], target_classes int64
    [B, Kc], target_labels f32 [B, Kc, P] -> cost f32 [S, B, Q, Kc] (= match_cost over the
    logits E_s . F, HF:m2f:434-481)."""
    Ec = E.contiguous()
    Fp = point_features.contiguous()
    L.require_hip(Ec, Fp, probs, target_classes, target_labels)
    S, B, Q, C = Ec.shape
    pr = probs.float().contiguous()
    tc = target_classes.to(torch.int64).contiguous()
    tl = target_labels.float().contiguous()
    Kc, P = int(tl.shape[1]), int(tl.shape[2])
    if (Ec.dtype != torch.bfloat16 or tuple(Fp.shape) != (B, P, 2 * C) or tuple(tc.shape) != (B, Kc)
            or tuple(pr.shape[:3]) != (S, B, Q)):
        raise ValueError("match_cost_factors: inconsistent shapes")
    ws = torch.empty(int(L.lib().vs_match_cost_factors_workspace_bytes(S, B, Q, P, Kc)), device=Ec.device,
                     dtype=torch.uint8)
    cost = torch.empty(S, B, Q, Kc, device=Ec.device, dtype=torch.float32)
    with timed("match_cost_factors", Ec, bytes_=Fp.numel() * 2 + tl.numel() * 4 + Ec.numel() * 2,
               flops=4.0 * S * B * Q * P * C):
        L.check(L.lib().vs_match_cost_factors(L.ptr(Ec), L.ptr(Fp), S, L.ptr(pr), int(pr.shape[3]), L.ptr(tc),
                                              L.ptr(tl), L.ptr(cost), L.ptr(ws), B, Q, C, P, Kc,
                                              float(mask_weight), float(class_weight), float(dice_weight),
                                              L.stream(Ec)), "match_cost_factors")
    return cost


def mask_head_grouped(E, F_nhwc, height: int, width: int, group: int):
    """mask_head of E bf16 [B, Q, C] (Q = R * group) over F [B, H*W, C] with the output rows
    in (r, image, g) order: f32 [R, B, group, H, W] (csrc/mask_head.hip, grouped stores)."""
    Ec, Fc = E.contiguous(), F_nhwc.contiguous()
    L.require_hip(Ec, Fc)
    B, Q, C = Ec.shape
    if Ec.dtype != torch.bfloat16 or Fc.dtype != torch.bfloat16 or tuple(Fc.shape) != (B, height * width, C):
        raise ValueError("mask_head_grouped: bf16 E [B, Q, C] and F [B, H*W, C] expected")
    out = torch.empty(Q // group, B, group, height, width, device=Ec.device, dtype=torch.float32)
    with timed("mask_head_fwd", Ec, bytes_=Fc.numel() * 2 + out.numel() * 4, flops=2.0 * B * Q * C * height * width):
        L.check(L.lib().vs_mask_head_forward_grouped(L.ptr(Ec), L.ptr(Fc), L.ptr(out), B, Q, C, int(height),
                                                     int(width), int(group), L.stream(Ec)), "mask_head_grouped")
    return out


class RowPointLogitsFunction(torch.autograd.Function):
    """Point samples of SELECTED rows of one mask-head output, differentiable w.r.t. the
    head's factors: the single-step form of MatchedPointLogitsFunction for a criterion
    that pairs R queries per image with targets (MaskDINO: the matched queries of a step,
    or its denoising queries).  logits [M, H, W] detached f32 (the head's output, all rows),
    rows int64 [B*R] (the selected row of each point set), coords [B*R, n, 2] in [0, 1),
    Esel [B, R, C] the selected rows' mask embeddings, P [B, HW, C] -> [B*R, n]; the forward
    gathers the points straight from the selected rows (csrc/mask_head.hip
    point_sample_rows_kernel: no copy of the selected maps).  Backward: point gradients
    scattered into [B, R, H, W] (point_scatter, no
    atomics), the mask head's adjoint on those R rows only (the fused bf16 backward, dP
    accumulated in `sink`'s buffer when one is given) -- instead of grid_sample's atomic
    backward over the maps and the mask-head backward over all Q rows of a zero-filled
    full-size gradient."""

    @staticmethod
    def forward(ctx, logits, rows, coords, Esel, P, sink=None):
        M, H, W = logits.shape
        B, R = Esel.shape[:2]
        out = point_sample_rows(logits, rows, coords)
        grid = 2.0 * coords.unsqueeze(2) - 1.0
        ctx.save_for_backward(grid, Esel, P)
        ctx.geom = (B, R, H, W)
        ctx.sink = sink
        return out

    @staticmethod
    def backward(ctx, g):
        grid, Esel, P = ctx.saved_tensors
        B, R, H, W = ctx.geom
        n = g.shape[-1]
        G = torch.empty(B, R, H, W, device=g.device, dtype=torch.float32)
        gc = g.float().contiguous()
        gr = grid.contiguous()
        with timed("point_scatter", gc, bytes_=gc.numel() * 12 + G.numel() * 4):
            L.check(L.lib().vs_point_scatter(L.ptr(gc), L.ptr(gr), L.ptr(G), 1, B, R, n, H, W, L.stream(gc)),
                    "point_scatter")
        C = Esel.shape[-1]
        sink = ctx.sink
        if P.dtype == torch.bfloat16 and C in (128, 256):
            acc = sink is not None and sink.buf is not None
            if sink is not None and not acc:
                sink.buf = torch.empty_like(P)
            dP = sink.buf if sink is not None else torch.empty_like(P)
            Ec = Esel.contiguous()
            with timed("mask_head_bwd", Ec, bytes_=G.numel() * 4 + (Ec.numel() * 2 + P.numel() * 2) * 2,
                       flops=4.0 * B * R * C * H * W):
                dE = L.tops().mask_head_bwd(G, Ec, P, dP, bool(acc))
            return None, None, None, dE, (None if sink is not None else dP), None
        Gb = G.view(B, R, H * W).to(P.dtype)
        dE = torch.bmm(Gb, P)
        dP = torch.bmm(Gb.transpose(1, 2), Esel.to(P.dtype))
        if sink is not None:
            sink.buf = dP if sink.buf is None else sink.buf + dP
            dP = None
        return None, None, None, dE.to(Esel.dtype), dP, None


class StepRowPointLogitsFunction(torch.autograd.Function):
    """RowPointLogitsFunction for S prediction sets at once (MaskDINO: the matched queries
    of every decoder step, or the denoising queries of every step): logits = S detached
    f32 [M_s, H, W] maps, rows int64 [S, B*R] (each set's selected row in its step's maps),
    coords [S*B*R, n, 2], Esel [B, S*R, C] (image b's selected rows, step-major), P
    [B, HW, C] -> [S*B*R, n] (set order (s, b, r)).  Backward: ONE point scatter into
    [B, S*R, H, W] and ONE mask-head adjoint over the S*R rows (instead of S of each: the
    fused kernel reads P once, not S times)."""

    @staticmethod
    def forward(ctx, rows, coords, Esel, P, sink, *logits):
        S = len(logits)
        H, W = logits[0].shape[-2:]
        B, SR = Esel.shape[:2]
        R = SR // S
        n = coords.shape[1]
        out = torch.empty(S * B * R, n, device=coords.device, dtype=torch.float32)
        for s_, lg in enumerate(logits):
            out[s_ * B * R:(s_ + 1) * B * R] = point_sample_rows(lg, rows[s_], coords[s_ * B * R:(s_ + 1) * B * R])
        grid = 2.0 * coords.unsqueeze(2) - 1.0
        ctx.save_for_backward(grid, Esel, P)
        ctx.geom = (S, B, R, H, W)
        ctx.sink = sink
        return out

    @staticmethod
    def backward(ctx, g):
        grid, Esel, P = ctx.saved_tensors
        S, B, R, H, W = ctx.geom
        n = g.shape[-1]
        G = torch.empty(B, S * R, H, W, device=g.device, dtype=torch.float32)
        gc = g.float().contiguous()
        gr = grid.contiguous()
        with timed("point_scatter", gc, bytes_=gc.numel() * 12 + G.numel() * 4):
            L.check(L.lib().vs_point_scatter(L.ptr(gc), L.ptr(gr), L.ptr(G), S, B, R, n, H, W, L.stream(gc)),
                    "point_scatter")
        C = Esel.shape[-1]
        sink = ctx.sink
        nones = (None,) * S
        if P.dtype == torch.bfloat16 and C in (128, 256):
            acc = sink is not None and sink.buf is not None
            if sink is not None and not acc:
                sink.buf = torch.empty_like(P)
            dP = sink.buf if sink is not None else torch.empty_like(P)
            Ec = Esel.contiguous()
            with timed("mask_head_bwd", Ec, bytes_=G.numel() * 4 + (Ec.numel() * 2 + P.numel() * 2) * 2,
                       flops=4.0 * B * S * R * C * H * W):
                dE = L.tops().mask_head_bwd(G, Ec, P, dP, bool(acc))
            return (None, None, dE, (None if sink is not None else dP), None) + nones
        Gb = G.view(B, S * R, H * W).to(P.dtype)
        dE = torch.bmm(Gb, P)
        dP = torch.bmm(Gb.transpose(1, 2), Esel.to(P.dtype))
        if sink is not None:
            sink.buf = dP if sink.buf is None else sink.buf + dP
            dP = None
        return (None, None, dE.to(Esel.dtype), dP, None) + nones


def step_row_point_logits(logits, rows, coords, Esel, P, sink=None):
    """StepRowPointLogitsFunction (logits: a list of S detached [M_s, H, W] maps)."""
    return StepRowPointLogitsFunction.apply(rows, coords, Esel, P, sink, *logits)


def row_point_logits(logits, rows, coords, Esel, P, sink=None):
    """RowPointLogitsFunction (device tensors; sink: a GradSink whose source P is)."""
    return RowPointLogitsFunction.apply(logits, rows, coords, Esel, P, sink)


def point_sample_rows(maps, rows, coords):
    """maps f32 [M, H, W], rows int64 [N] (or None: set n reads map n), coords f32 [N, P, 2]
    in [0, 1] -> [N, P]: the bilinear sample (grid_sample, align_corners=False, zeros) of map
    rows[n] at each of its points (csrc/mask_head.hip point_sample_rows_kernel)."""
    L.require_hip(maps, coords)
    M, H, W = maps.shape
    N, P = coords.shape[:2]
    mc = maps if (maps.dtype == torch.float32 and maps.is_contiguous()) else maps.float().contiguous()
    rc = rows.to(torch.int64).contiguous() if rows is not None else None
    if rc is None and N > M:
        raise ValueError(f"{N} point sets but {M} maps and no rows")
    cc = coords if (coords.dtype == torch.float32 and coords.is_contiguous()) else coords.float().contiguous()
    out = torch.empty(N, P, device=maps.device, dtype=torch.float32)
    with timed("point_sample_rows", mc, bytes_=cc.numel() * 4 + out.numel() * 4 * 5):
        L.check(L.lib().vs_point_sample_rows(L.ptr(mc), L.ptr(rc) if rc is not None else None, L.ptr(cc), L.ptr(out),
                                             M, H, W, N, P, L.stream(mc)), "point_sample_rows")
    return out


def point_sample(feat, coords):
    """point_sample (HF:m2f:245-275) of one map per point set: feat f32 [N, 1, H, W] (or
    [N, H, W]), coords [N, P, 2] in [0, 1] -> [N, P] -- grid_sample(align_corners=False,
    zeros) on the HIP point gather for device tensors (ATen's grid_sampler_2d took 95 us per
    call at the criterion's 80 x 256^2 maps / 37 632 points), torch on the CPU or where
    autograd must differentiate through it."""
    if not feat.is_cuda or (feat.requires_grad and torch.is_grad_enabled()):
        return F.grid_sample(feat.view(feat.shape[0], 1, *feat.shape[-2:]), 2.0 * coords.unsqueeze(2) - 1.0,
                             align_corners=False).squeeze(3).squeeze(1)
    return point_sample_rows(feat.reshape(feat.shape[0], *feat.shape[-2:]), None, coords)


def point_sample_masks(masks, coords, grid_space=False, sets_per_coord=1, rows=None):
    """Bilinear point samples (grid_sample, align_corners=False, zeros) of bool / u8 target
    masks [M, H, W] without an f32 copy of them (csrc/mask_head.hip, vs_point_sample_masks).
    grid_space=False: coords f32 [N, P, 2] in [0, 1], set n reads masks[rows[n]] (rows None:
    masks[n]) -> [N, P].  grid_space=True: coords f32 [G, P, 2] in [-1, 1], set n reads
    masks[n] at point set n // sets_per_coord -> [G * sets_per_coord, P]."""
    L.require_hip(masks, coords)
    M, H, W = masks.shape
    mc = masks.contiguous()
    mc = mc.view(torch.uint8) if mc.dtype == torch.bool else mc.to(torch.uint8)
    cc = coords.float().contiguous()
    P = cc.shape[1]
    N = cc.shape[0] * sets_per_coord if grid_space else cc.shape[0]
    if rows is not None:
        rows = rows.to(torch.int64).contiguous()
    elif N > M:
        raise ValueError(f"{N} point sets but {M} masks and no rows")
    out = torch.empty(N, P, device=masks.device, dtype=torch.float32)
    with timed("point_sample_masks", mc, bytes_=cc.numel() * 4 + out.numel() * 4 * 2):
        L.check(L.lib().vs_point_sample_masks(L.ptr(mc), L.ptr(rows) if rows is not None else None, L.ptr(cc),
                                              L.ptr(out), M, H, W, N, P, int(bool(grid_space)), int(sets_per_coord),
                                              L.stream(mc)), "point_sample_masks")
    return out


def topk_rows(values, k):
    """values f32 [N, n] -> int64 [N, k]: per row the indices of the k largest values, in
    ascending index order (csrc/topk.hip radix select; replaces `torch.topk(values, k)[1]`
    of the importance sampling, HF:m2f:689-724 -- the points are used as a set)."""
    L.require_hip(values)
    vc = values.float().contiguous()
    N, n = vc.shape
    assert 0 < k <= n
    out = torch.empty(N, k, device=vc.device, dtype=torch.int64)
    with timed("topk_rows", vc, bytes_=vc.numel() * 4 * 5 + out.numel() * 8):
        L.check(L.lib().vs_topk_rows(L.ptr(vc), L.ptr(out), N, n, k, L.stream(vc)), "topk_rows")
    return out


def matched_maps(masks_list, qsel):
    """(maps [S*B*Kc, 1, H, W] f32 of mask_list[s][b, qsel[s, b, k]], factors): detached
    maps + the mask head's factors (E, P) when every step's logits came from `mask_head`
    (the loss then differentiates through `point_logits` -> MatchedPointLogitsFunction),
    else the maps with their autograd history and factors None.  FactoredLogits: the
    matched rows only, E_sel . F in one grouped mask-head launch."""
    S, B, Kc = qsel.shape
    if factored(masks_list):
        m0 = masks_list[0]
        E, Fm = m0.E, m0.F
        C = E.shape[-1]
        with torch.no_grad():
            Esel = torch.gather(E.detach().transpose(0, 1), 2, qsel.transpose(0, 1)[..., None].expand(B, S, Kc, C))
            maps = mask_head_grouped(Esel.reshape(B, S * Kc, C), Fm.detach(), m0.H, m0.W, Kc)
        return maps.view(S * B * Kc, 1, m0.H, m0.W), (E, Fm)
    masks_list = materialize_masks(masks_list)      # a partial / reordered factored list
    bidx = torch.arange(B, device=qsel.device)[:, None].expand(B, Kc)
    fac = mask_head_factors(masks_list)
    with torch.no_grad() if fac is not None else contextlib.nullcontext():
        pred = torch.stack([masks_list[s][bidx, qsel[s]] for s in range(S)])            # [S,B,Kc,H,W]
    H, W = pred.shape[-2:]
    return pred.reshape(S * B * Kc, 1, H, W).float(), fac


def point_logits(maps, coords, qsel, fac):
    """Logits of `matched_maps` at coords [S*B*Kc, n, 2] in [0,1) (bilinear, zero padding:
    point_sample HF:m2f:245-275) -> [S*B*Kc, n] f32."""
    if fac is None:
        return F.grid_sample(maps, 2.0 * coords.unsqueeze(2) - 1.0, align_corners=False).squeeze(3).squeeze(1)
    return MatchedPointLogitsFunction.apply(maps, coords, qsel, fac[0], fac[1])


class _SinkSource(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, sink):
        ctx.sink = sink
        ctx.shape = x.shape
        ctx.set_materialize_grads(False)
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        # runs after every consumer of the output: their in-place sum is in sink.buf (kept
        # in the consumers' row layout: viewed back to the source's shape here)
        buf, ctx.sink.buf = ctx.sink.buf, None
        if buf is not None:
            buf = buf.view(ctx.shape)
        if g is not None:
            buf = g if buf is None else buf + g
        return buf, None


class GradSink:
    """Gradient side channel for a tensor consumed by several mask-head calls: the calls
    accumulate its gradient into `buf` in place (csrc/mask_head.hip ACC mode) and return
    none; the source node hands the sum to autograd once."""

    def __init__(self):
        self.buf = None

    def source(self, x):
        return _SinkSource.apply(x, self)


def attn_bitmask(logits, target_hw):
    """Blocked-key bitmask of the next decoder layer from mask logits [B,Q,H,W]
    (HF:m2f:2049-2055 + the fully-blocked-row fix HF:m2f:1912-1914) -> int32 words
    [B, Q, ceil(th*tw/32)] (bit k%32 of word k/32 set = key k blocked)."""
    L.require_hip(logits)
    lg = logits.detach().float().contiguous()
    B, Q, H, W = lg.shape
    th, tw = int(target_hw[0]), int(target_hw[1])
    with timed("attn_bitmask", lg, bytes_=min(lg.numel(), B * Q * th * tw * 4) * 4 + B * Q * ((th * tw + 31) // 32) * 4):
        return L.tops().attn_bitmask(lg, th, tw)


def unpack_bitmask(words, n_keys: int):
    """[..., nwords] int32 -> bool [..., n_keys] (True = blocked); test/debug helper."""
    w = words.to(torch.int64) & 0xFFFFFFFF
    bits = (w.unsqueeze(-1) >> torch.arange(32, device=w.device)) & 1
    return bits.flatten(-2)[..., :n_keys].bool()


class MaskedAttentionFunction(torch.autograd.Function):
    """softmax over unblocked keys of (q.k)*scale, times V (HF:m2f:1644-1650 core).
    q [B,Q,heads*32], k/v [B,S,heads*32], words from `attn_bitmask` -> [B,Q,heads*32]."""

    @staticmethod
    def forward(ctx, q, k, v, words, heads, scale):
        L.require_hip(q, k, v, words)
        q, k, v = q.contiguous(), k.to(q.dtype).contiguous(), v.to(q.dtype).contiguous()
        B, Q, C = q.shape
        S = k.shape[1]
        if C != heads * 32 or k.shape != (B, S, C) or v.shape != (B, S, C):
            raise ValueError("masked attention shape mismatch")
        if words.shape != (B, Q, (S + 31) // 32):
            raise ValueError(f"bitmask {tuple(words.shape)} does not cover {S} keys")
        nb = (q.numel() * 2 + k.numel() + v.numel()) * q.element_size() + words.numel() * 4
        with timed("masked_attn_fwd", q, bytes_=nb, flops=4.0 * B * heads * Q * S * 32):
            out, lse = L.tops().masked_xattn_fwd(q, k, v, words, heads, float(scale))
        ctx.meta = (heads, float(scale))
        ctx.save_for_backward(q, k, v, words, out, lse)
        return out

    @staticmethod
    def backward(ctx, g):
        q, k, v, words, out, lse = ctx.saved_tensors
        heads, scale = ctx.meta
        B, Q, C = q.shape
        S = k.shape[1]
        nb = (q.numel() * 4 + 2 * k.numel() + 2 * v.numel()) * q.element_size() + words.numel() * 4
        with timed("masked_attn_bwd", q, bytes_=nb, flops=10.0 * B * heads * Q * S * 32):
            try:
                gq, gk, gv = L.tops().masked_xattn_bwd(q, k, v, words, out, lse, g, heads, scale)
            except RuntimeError as e:
                raise RuntimeError(f"{e} (q {q.dtype} {tuple(q.shape)}, k {k.dtype} {tuple(k.shape)}, out "
                                   f"{out.dtype}, lse {lse.dtype}, grad {g.dtype} {tuple(g.shape)})") from e
        return gq, gk, gv, None, None, None


def masked_attention(q, k, v, words, heads: int, scale: float | None = None):
    if scale is None:
        scale = 32 ** -0.5
    return MaskedAttentionFunction.apply(q, k, v, words, int(heads), float(scale))


def pack_blocked(blocked):
    """bool [..., S] (True = blocked) -> int32 words [..., ceil(S/32)], bit j%32 of word j/32
    set = key j blocked (the layout of attn_bitmask / the self-attention kernels)."""
    S = blocked.shape[-1]
    nw = (S + 31) // 32
    b = F.pad(blocked.to(torch.int64), (0, nw * 32 - S)).view(*blocked.shape[:-1], nw, 32)
    w = (b << torch.arange(32, device=blocked.device, dtype=torch.int64)).sum(-1)
    return torch.where(w >= 2 ** 31, w - 2 ** 32, w).to(torch.int32).contiguous()


_NO_WORDS: dict = {}


class SelfAttentionFunction(torch.autograd.Function):
    """Decoder self-attention core (HF:m2f:1659-1664; MaskDINO's DN-masked self-attention):
    softmax over the unblocked keys of (q.k) * scale, times V.  q / k / v [B, Q, heads*32] bf16;
    words: None, or int32 [Q, nw] shared by the batch / [B, Q, nw] (pack_blocked).  One
    forward and one backward launch (csrc/self_attn.hip), f32 softmax and dS, P / dS as
    exact bf16 hi + lo pairs in the products."""

    @staticmethod
    def forward(ctx, q, k, v, words, heads, scale):
        L.require_hip(q, k, v)
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        B, Q, C = q.shape
        S = k.shape[1]
        if words is None:
            key = q.device
            words = _NO_WORDS.get(key)
            if words is None:
                words = _NO_WORDS[key] = torch.empty(0, device=q.device, dtype=torch.int32)
        nb = (2 * q.numel() + k.numel() + v.numel()) * 2 + q.numel() * 4 + words.numel() * 4
        with timed("self_attn_fwd", q, bytes_=nb, flops=4.0 * B * heads * Q * S * 32):
            out, out32, lse = L.tops().self_attn_fwd(q, k, v, words, heads, float(scale))
        ctx.meta = (heads, float(scale))
        ctx.save_for_backward(q, k, v, words, out32, lse)
        return out

    @staticmethod
    def backward(ctx, g):
        q, k, v, words, out32, lse = ctx.saved_tensors
        heads, scale = ctx.meta
        B, Q, C = q.shape
        S = k.shape[1]
        nb = (4 * q.numel() + 2 * k.numel() + 2 * v.numel()) * 2 + out32.numel() * 4 + words.numel() * 4
        with timed("self_attn_bwd", q, bytes_=nb, flops=10.0 * B * heads * Q * S * 32):
            gq, gk, gv = L.tops().self_attn_bwd(q, k, v, words, out32, lse, g, heads, scale)
        return gq, gk, gv, None, None, None


def self_attention(q, k, v, heads: int, scale: float | None = None, words=None):
    """Decoder self-attention core on the HIP kernels: bf16 -> SelfAttentionFunction; f32
    (the parity kernel mode) -> the scalar masked-attention kernels with explicit words
    (all-zero when there is no mask).  No SDPA, no fallback."""
    if scale is None:
        scale = 32 ** -0.5
    if q.dtype == torch.bfloat16:
        return SelfAttentionFunction.apply(q, k.to(q.dtype), v.to(q.dtype), words, int(heads), float(scale))
    B, Q, _ = q.shape
    S = k.shape[1]
    if words is None:
        words = torch.zeros(B, Q, (S + 31) // 32, device=q.device, dtype=torch.int32)
    elif words.dim() == 2:
        words = words.unsqueeze(0).expand(B, -1, -1).contiguous()
    return masked_attention(q, k, v, words, heads, scale)


# ------------------------------------------------------------------ LayerNorm / bias grad
class WindowRows:
    """Window-layout rows of the image tokens of a [B, H, W] grid, for the Swin window
    partition folded into the LayerNorm before it (HF:swin:546-551: zero pad to multiples
    of ws, roll by -shift, partition): rows int32 [B*H*W] = the window row of image token
    m, pad int64 = the window rows of the zero padding, total = B * nWh * nWw * ws^2."""

    def __init__(self, B, H, W, ws, shift, device):
        self.B, self.H, self.W, self.ws, self.shift = B, H, W, ws, shift
        nwh, nww = -(-H // ws), -(-W // ws)
        Hp, Wp = nwh * ws, nww * ws
        self.total = B * Hp * Wp
        with torch.no_grad():
            y = torch.arange(H, device=device).view(1, H, 1)
            x = torch.arange(W, device=device).view(1, 1, W)
            b = torch.arange(B, device=device).view(B, 1, 1)
            py, px = (y - shift) % Hp, (x - shift) % Wp            # padded-grid position of each pixel
            row = ((b * nwh + py // ws) * nww + px // ws) * (ws * ws) + (py % ws) * ws + px % ws
            self.rows = row.reshape(-1).to(torch.int32).contiguous()
            hit = torch.zeros(self.total, dtype=torch.bool, device=device)
            hit[self.rows.long()] = True
            self.pad = torch.nonzero(~hit).view(-1)

    def tensors(self):
        return [self.rows, self.pad]


_WROWS: "collections.OrderedDict" = collections.OrderedDict()


def window_rows(B, H, W, ws, shift, device):
    """WindowRows for the shape, made once per (shape, device) and kept in an LRU of 64:
    the eager warm-up before a HIP graph capture (trainer, predictor) makes every entry
    the capture reads, the most recently used, so none is evicted before the capture
    (making one needs a host sync, which a capture refuses; see model.cached_constants
    for the lifetime of the tensors a graph reads)."""
    key = (B, H, W, ws, shift, str(device))
    wr = _WROWS.get(key)
    if wr is None:
        wr = WindowRows(B, H, W, ws, shift, device)
        _WROWS[key] = wr
        while len(_WROWS) > 64:
            _WROWS.popitem(last=False)
    else:
        _WROWS.move_to_end(key)
    return wr


def window_rows_constants():
    return [t for wr in _WROWS.values() for t in wr.tensors()]


def _to_windows(y, wr):
    """The window partition of a [B*H*W, C] tensor as the row-mapped kernels lay it out."""
    return window_partition(y.view(wr.B, wr.H, wr.W, -1), wr.ws, wr.shift).view(wr.total, -1)


class LayerNormFunction(torch.autograd.Function):
    """F.layer_norm over the last dim of a token-major [..., C] tensor (csrc/norm.hip);
    x, weight, bias share one dtype (f32 or bf16)."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps, wrows=None, quant=False):
        """wrows (WindowRows): y in the window layout [wrows.total, C] (the partition folded
        into the kernel's stores; padding rows zero).  quant (bf16, with wrows): also y's MX
        fp8 copy (e4m3, e8m0 scales) -> (y, y_q, y_qscales), the copy not differentiable."""
        L.require_hip(x, weight, bias)
        C = x.shape[-1]
        xc = x.contiguous()
        M = xc.numel() // C
        mean = torch.empty(M, device=x.device, dtype=torch.float32)
        rstd = torch.empty(M, device=x.device, dtype=torch.float32)
        with timed("layer_norm_fwd", xc, bytes_=2 * xc.numel() * xc.element_size()):
            if quant == "rows":              # row-scaled e4m3 copy for the vendor rowwise fp8 GEMM
                rows = wrows.total if wrows is not None else M
                y = torch.empty(rows, C, device=x.device, dtype=xc.dtype)
                yq = torch.empty(rows, C, device=x.device, dtype=torch.uint8)
                ys = torch.empty(rows, 1, device=x.device, dtype=torch.float32)
                L.check(L.lib().vs_layer_norm_forward_qr(L.ptr(xc), L.ptr(weight), L.ptr(bias), L.ptr(y), L.ptr(yq),
                                                         L.ptr(ys), L.ptr(mean), L.ptr(rstd), M, C, float(eps),
                                                         L.ptr(wrows.rows) if wrows is not None else None,
                                                         L.stream(xc)), "layer_norm_forward_qr")
                if wrows is None:
                    y = y.view(xc.shape)
                elif wrows.pad.numel():
                    y.index_fill_(0, wrows.pad, 0)
                    yq.index_fill_(0, wrows.pad, 0)
                    ys.index_fill_(0, wrows.pad, 1.0)
                yq = yq.view(torch.float8_e4m3fn)
            elif quant:
                y = torch.empty(wrows.total, C, device=x.device, dtype=xc.dtype)
                yq = torch.empty(wrows.total, C, device=x.device, dtype=torch.uint8)
                ys = torch.empty(wrows.total, C // 32, device=x.device, dtype=torch.uint8)
                L.check(L.lib().vs_layer_norm_forward_rows_q(L.ptr(xc), L.ptr(weight), L.ptr(bias), L.ptr(y),
                                                             L.ptr(yq), L.ptr(ys), L.ptr(mean), L.ptr(rstd), M, C,
                                                             float(eps), L.ptr(wrows.rows), L.stream(xc)),
                        "layer_norm_forward_rows_q")
                if wrows.pad.numel():
                    y.index_fill_(0, wrows.pad, 0)
                    yq.index_fill_(0, wrows.pad, 0)
                    ys.index_fill_(0, wrows.pad, 127)          # scale 1 (0xff would be NaN)
            elif wrows is None:
                y = torch.empty_like(xc)
                L.check(L.lib().vs_layer_norm_forward(L.dtype_code(xc), L.ptr(xc), L.ptr(weight), L.ptr(bias),
                                                      L.ptr(y), L.ptr(mean), L.ptr(rstd), M, C, float(eps),
                                                      L.stream(xc)), "layer_norm_forward")
            else:
                y = torch.empty(wrows.total, C, device=x.device, dtype=xc.dtype)
                L.check(L.lib().vs_layer_norm_forward_rows(L.dtype_code(xc), L.ptr(xc), L.ptr(weight), L.ptr(bias),
                                                           L.ptr(y), L.ptr(mean), L.ptr(rstd), M, C, float(eps),
                                                           L.ptr(wrows.rows), L.stream(xc)), "layer_norm_forward_rows")
                if wrows.pad.numel():
                    y.index_fill_(0, wrows.pad, 0)
        ctx.wrows = wrows
        ctx.save_for_backward(xc, weight, mean, rstd)
        if quant:
            ctx.mark_non_differentiable(yq, ys)
            return y, yq, ys
        return y

    @staticmethod
    def backward(ctx, gy, *_):
        xc, weight, mean, rstd = ctx.saved_tensors
        C = xc.shape[-1]
        M = xc.numel() // C
        gy = gy.to(xc.dtype).contiguous()
        gx = torch.empty_like(xc)
        gw = torch.empty_like(weight)
        gb = torch.empty_like(weight)
        ws = torch.empty(int(L.lib().vs_layer_norm_backward_workspace_bytes(M, C)), device=xc.device,
                         dtype=torch.uint8)
        with timed("layer_norm_bwd", xc, bytes_=3 * xc.numel() * xc.element_size()):
            if ctx.wrows is None:
                L.check(L.lib().vs_layer_norm_backward(L.dtype_code(xc), L.ptr(gy), L.ptr(xc), L.ptr(weight),
                                                       L.ptr(mean), L.ptr(rstd), L.ptr(gx), L.ptr(gw), L.ptr(gb),
                                                       L.ptr(ws), M, C, L.stream(xc)), "layer_norm_backward")
            else:
                L.check(L.lib().vs_layer_norm_backward_rows(L.dtype_code(xc), L.ptr(gy), L.ptr(xc), L.ptr(weight),
                                                            L.ptr(mean), L.ptr(rstd), None, L.ptr(gx), L.ptr(gw),
                                                            L.ptr(gb), None, L.ptr(ws), M, C, L.ptr(ctx.wrows.rows),
                                                            L.stream(xc)), "layer_norm_backward_rows")
        return gx, gw, gb, None, None, None


def attach_colsum(g: torch.Tensor, colsum: torch.Tensor) -> None:
    """Record the column sums over the leading dims of gradient `g` (computed by the kernel
    that produced g) so a consumer needing them -- the bias gradient of the Linear whose
    output received g -- skips a second read of g.  Keyed to g's version counter: an
    in-place update of g afterwards (e.g. autograd accumulating into it) invalidates it."""
    g._vs_colsum = (colsum, g._version)


def take_colsum(g: torch.Tensor):
    """The column sums recorded by attach_colsum if still valid for g, else None.  The record
    is removed: the caller returns the sums as a bias gradient, and a second reference to them
    makes autograd's AccumulateGrad copy them instead of adopting them as .grad (36 copy
    launches per C2 step)."""
    rec = getattr(g, "_vs_colsum", None)
    if rec is None:
        return None
    del g._vs_colsum
    if rec[1] != g._version or rec[0].shape[0] != g.shape[-1]:
        return None
    return rec[0]


class AddLayerNormFunction(torch.autograd.Function):
    """(s, y) = (x + r, layer_norm(x + r)) in one pass (csrc/norm.hip, RES variant); the
    backward adds the gradient of s (residual path) inside the LayerNorm backward."""

    @staticmethod
    def forward(ctx, x, r, weight, bias, eps, sink=None, wrows=None, quant=False):
        """wrows (WindowRows): y in the window layout (see LayerNormFunction); s stays in x's.
        quant (bf16): also y's MX fp8 copy -> (s, y, y_q, y_qscales)."""
        L.require_hip(x, r, weight, bias)
        ctx.sink = sink if sink is not None and sink.armed else None
        # an unused output (the post-norm decoder drops s) gets no gradient instead of a
        # zero-filled one (a fill kernel + the residual-add read of zeros, per block)
        ctx.set_materialize_grads(False)
        C = x.shape[-1]
        xc, rc = x.contiguous(), r.to(x.dtype).contiguous()
        M = xc.numel() // C
        s = torch.empty_like(xc)
        mean = torch.empty(M, device=x.device, dtype=torch.float32)
        rstd = torch.empty(M, device=x.device, dtype=torch.float32)
        with timed("add_layer_norm_fwd", xc, bytes_=4 * xc.numel() * xc.element_size()):
            if quant == "rows":              # row-scaled e4m3 copy for the vendor rowwise fp8 GEMM
                rows = wrows.total if wrows is not None else M
                y = torch.empty(rows, C, device=x.device, dtype=xc.dtype)
                yq = torch.empty(rows, C, device=x.device, dtype=torch.uint8)
                ys = torch.empty(rows, 1, device=x.device, dtype=torch.float32)
                L.check(L.lib().vs_add_layer_norm_forward_qr(L.ptr(xc), L.ptr(rc), L.ptr(weight), L.ptr(bias),
                                                             L.ptr(s), L.ptr(y), L.ptr(yq), L.ptr(ys), L.ptr(mean),
                                                             L.ptr(rstd), M, C, float(eps),
                                                             L.ptr(wrows.rows) if wrows is not None else None,
                                                             L.stream(xc)), "add_layer_norm_forward_qr")
                if wrows is None:
                    y = y.view(xc.shape)
                elif wrows.pad.numel():
                    y.index_fill_(0, wrows.pad, 0)
                    yq.index_fill_(0, wrows.pad, 0)
                    ys.index_fill_(0, wrows.pad, 1.0)
                yq = yq.view(torch.float8_e4m3fn)
            elif quant:
                rows = wrows.total if wrows is not None else M
                y = torch.empty(rows, C, device=x.device, dtype=xc.dtype)
                yq = torch.empty(rows, C, device=x.device, dtype=torch.uint8)
                ys = torch.empty(rows, C // 32, device=x.device, dtype=torch.uint8)
                L.check(L.lib().vs_add_layer_norm_forward_q(L.ptr(xc), L.ptr(rc), L.ptr(weight), L.ptr(bias),
                                                            L.ptr(s), L.ptr(y), L.ptr(yq), L.ptr(ys), L.ptr(mean),
                                                            L.ptr(rstd), M, C, float(eps),
                                                            L.ptr(wrows.rows) if wrows is not None else None,
                                                            L.stream(xc)), "add_layer_norm_forward_q")
                if wrows is None:
                    y = y.view(xc.shape)
                elif wrows.pad.numel():
                    y.index_fill_(0, wrows.pad, 0)
                    yq.index_fill_(0, wrows.pad, 0)
                    ys.index_fill_(0, wrows.pad, 127)
            elif wrows is None:
                y = torch.empty_like(xc)
                L.check(L.lib().vs_add_layer_norm_forward(L.dtype_code(xc), L.ptr(xc), L.ptr(rc), L.ptr(weight),
                                                          L.ptr(bias), L.ptr(s), L.ptr(y), L.ptr(mean), L.ptr(rstd),
                                                          M, C, float(eps), L.stream(xc)), "add_layer_norm_forward")
            else:
                y = torch.empty(wrows.total, C, device=x.device, dtype=xc.dtype)
                L.check(L.lib().vs_add_layer_norm_forward_rows(L.dtype_code(xc), L.ptr(xc), L.ptr(rc), L.ptr(weight),
                                                               L.ptr(bias), L.ptr(s), L.ptr(y), L.ptr(mean),
                                                               L.ptr(rstd), M, C, float(eps), L.ptr(wrows.rows),
                                                               L.stream(xc)), "add_layer_norm_forward_rows")
                if wrows.pad.numel():
                    y.index_fill_(0, wrows.pad, 0)
        ctx.wrows = wrows
        ctx.save_for_backward(s, weight, mean, rstd)
        if quant:
            ctx.mark_non_differentiable(yq, ys)
            return s, y, yq, ys
        return s, y

    @staticmethod
    def backward(ctx, gs, gy, *_):
        s, weight, mean, rstd = ctx.saved_tensors
        C = s.shape[-1]
        M = s.numel() // C
        if gy is None:
            gy = torch.zeros_like(s)
        gy = gy.to(s.dtype).contiguous()
        gx = torch.empty_like(s)
        gw = torch.empty_like(weight)
        gb = torch.empty_like(weight)
        ws = torch.empty(int(L.lib().vs_layer_norm_backward_workspace_bytes(M, C)), device=s.device,
                         dtype=torch.uint8)
        # the column sums of gx come out of the same pass (C <= 1024: LDS budget); they are
        # the bias gradient of the Linear that produced r (see attach_colsum)
        cs = torch.empty(C, device=s.device, dtype=s.dtype) if C <= 1024 else None
        with timed("layer_norm_bwd", s, bytes_=(3 + (gs is not None)) * s.numel() * s.element_size()):
            gsc = gs.to(s.dtype).contiguous() if gs is not None else None
            if ctx.wrows is None:
                L.check(L.lib().vs_layer_norm_backward_ex(L.dtype_code(s), L.ptr(gy), L.ptr(s), L.ptr(weight),
                                                          L.ptr(mean), L.ptr(rstd),
                                                          L.ptr(gsc) if gsc is not None else None, L.ptr(gx), L.ptr(gw),
                                                          L.ptr(gb), L.ptr(cs) if cs is not None else None, L.ptr(ws),
                                                          M, C, L.stream(s)), "layer_norm_backward_ex")
            else:
                L.check(L.lib().vs_layer_norm_backward_rows(L.dtype_code(s), L.ptr(gy), L.ptr(s), L.ptr(weight),
                                                            L.ptr(mean), L.ptr(rstd),
                                                            L.ptr(gsc) if gsc is not None else None, L.ptr(gx),
                                                            L.ptr(gw), L.ptr(gb), L.ptr(cs) if cs is not None else None,
                                                            L.ptr(ws), M, C, L.ptr(ctx.wrows.rows), L.stream(s)),
                        "layer_norm_backward_rows")
        if cs is not None:
            attach_colsum(gx, cs)
        gxx = gx
        if ctx.sink is not None and ctx.needs_input_grad[0]:
            ctx.sink.g = gx            # the armed consumer of x adds it in its dX GEMM
            gxx = None
        return gxx, gx, gw, gb, None, None, None, None


def add_layer_norm(x, r, weight, bias, eps: float = 1e-5, sink: ResidualSink | None = None, wrows=None,
                   quant: bool = False):
    """(x + r, layer_norm(x + r)) for token-major [..., C] tensors (see AddLayerNormFunction;
    `sink`: see ResidualSink; `wrows`: y in the window layout; `quant`: + y's MX fp8 copy)."""
    return AddLayerNormFunction.apply(x, r, weight, bias, eps, sink, wrows, quant)


def layer_norm(x, weight, bias, eps: float = 1e-5, wrows=None, quant: bool = False):
    return LayerNormFunction.apply(x, weight, bias, eps, wrows, quant)


def layer_norm_supported(x, weight) -> bool:
    C = x.shape[-1]
    return (x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and weight.dtype == x.dtype
            and C % 8 == 0 and C <= 2048)


# widest row of the column-sum / activation-backward kernels (column blocks of 2048 on
# grid.y, csrc/norm.hip kColBlock): covers the Swin-L MLP hidden widths 3072 / 6144
COLSUM_MAX_N = 16384


def column_sum(x2d, out=None):
    """x [M, N] -> [N] (x's dtype, f32 accumulation): the bias gradient of a token-major
    Linear (csrc/norm.hip).  `out`: a contiguous [N] tensor of x's dtype to write into."""
    L.require_hip(x2d)
    x2d = x2d.contiguous()
    M, N = x2d.shape
    if out is None:
        out = torch.empty(N, device=x2d.device, dtype=x2d.dtype)
    elif out.shape != (N,) or out.dtype != x2d.dtype or not out.is_contiguous():
        raise ValueError("column_sum: out must be a contiguous [N] tensor of the input dtype")
    ws = torch.empty(int(L.lib().vs_column_sum_workspace_bytes(M, N)), device=x2d.device, dtype=torch.uint8)
    with timed("column_sum", x2d, bytes_=x2d.numel() * x2d.element_size()):
        L.check(L.lib().vs_column_sum(L.dtype_code(x2d), L.ptr(x2d), L.ptr(out), L.ptr(ws), M, N, L.stream(x2d)),
                "column_sum")
    return out


def column_sum_segments(x3d, sizes):
    """x [B, S, N] -> f32 [len(sizes), N]: column sums over every image's rows of each
    consecutive segment (sizes sum to S) -- the per-level sums of a multi-scale token
    sequence (csrc/norm.hip colsum_seg_kernel)."""
    L.require_hip(x3d)
    x3d = x3d.contiguous()
    B, S, N = x3d.shape
    sizes = [int(v) for v in sizes]
    if sum(sizes) != S or not 1 <= len(sizes) <= 8:
        raise ValueError(f"column_sum_segments: segment sizes {sizes} do not cover S = {S} (1..8 segments)")
    starts = [0]
    for v in sizes:
        starts.append(starts[-1] + v)
    seg = (ctypes.c_int * len(starts))(*starts)
    out = torch.empty(len(sizes), N, device=x3d.device, dtype=torch.float32)
    ws = torch.empty(int(L.lib().vs_column_sum_segments_workspace_bytes(B, N, len(sizes))), device=x3d.device,
                     dtype=torch.uint8)
    with timed("column_sum", x3d, bytes_=x3d.numel() * x3d.element_size()):
        L.check(L.lib().vs_column_sum_segments(L.dtype_code(x3d), L.ptr(x3d), L.ptr(out), L.ptr(ws), B, S, N, seg,
                                               len(sizes), L.stream(x3d)), "column_sum_segments")
    return out


class ResidualSink:
    """Hands a post-norm residual block's residual-path gradient to the GEMM that also
    consumes the block input, so that GEMM adds it in its epilogue (beta = 1) instead of
    autograd adding the two input gradients with a separate full-size kernel.

    Protocol (one object per forward call): the consumer (first op of the branch, e.g.
    the encoder FFN's fc1 or the MSDeformAttn input projections) `arm()`s the sink in its
    forward when it takes its fused path; `add_layer_norm(x, branch, ..., sink)` then
    returns no gradient for x and stores it here in its backward (which runs first: the
    consumer's output feeds the branch); the consumer `take()`s it in its backward.  If
    either side takes a plain path the sink is never armed or never filled, and autograd
    adds the gradients as usual."""

    __slots__ = ("armed", "g")

    def __init__(self):
        self.armed = False
        self.g = None

    def arm(self):
        self.armed = True

    def take(self):
        g, self.g = self.g, None
        return g


class ActBackwardSink:
    """The activation backward of one MLP (fc1 -> GELU / ReLU -> fc2) folded into fc2's dX
    GEMM (token_gemm gelu_pre / relu_out: the epilogue reads the saved pre-activation, resp.
    the ReLU output = fc2's own input), so dH is never written and read back by a separate
    activation pass.  Protocol (one object per MLP call, owned by the caller, whose activation
    output feeds fc2 ONLY): the activation's producer records the tensor (`pre`); fc2's Linear
    takes the sink in its forward when its dX runs on the token GEMM and, in its backward
    (which runs first), returns dpre = (dY W2) * act'(pre) and sets `done`; the activation's
    backward then passes that gradient through unchanged.  Either side on another path leaves
    the sink unused and autograd runs the plain composition."""

    __slots__ = ("kind", "pre", "done")

    def __init__(self, kind: str = "gelu"):
        assert kind in ("gelu", "relu")
        self.kind = kind
        self.pre = None
        self.done = False


GeluBackwardSink = ActBackwardSink


class _ActColsumFunction(torch.autograd.Function):
    """y = act(x) (torch's ReLU / exact GELU forward); the backward is one HIP pass
    (vs_act_backward_colsum) that also records the column sums of dx (attach_colsum): the
    bias gradient of the Linear that produced x, which then reads no dY for it.  gelu_sink
    (GeluBackwardSink): x is offered to the consumer; when it folded the derivative into its
    dX GEMM the incoming gradient IS dx (passed through; the producing Linear then takes its
    bias gradient from the split-K kernel)."""

    @staticmethod
    def forward(ctx, x, act, gelu_sink=None):
        ctx.act = act
        ctx.gs = gelu_sink if act == 1 and gelu_sink is not None and gelu_sink.kind == "gelu" else None
        if ctx.gs is not None:
            ctx.gs.pre = x
        ctx.save_for_backward(x)
        return F.gelu(x) if act == 1 else F.relu(x)

    @staticmethod
    def backward(ctx, gy):
        gs = getattr(ctx, "gs", None)            # (shared with _GeluRowQuantFunction: no sink there)
        if gs is not None and gs.done:
            gs.done = False
            return gy, None, None
        (x,) = ctx.saved_tensors
        N = x.shape[-1]
        M = x.numel() // N
        gy = gy.to(x.dtype).contiguous()
        gx = torch.empty_like(x)
        cs = torch.empty(N, device=x.device, dtype=x.dtype)
        ws = torch.empty(int(L.lib().vs_column_sum_workspace_bytes(M, N)), device=x.device, dtype=torch.uint8)
        with timed("act_bwd_colsum", x, bytes_=3 * x.numel() * x.element_size()):
            L.check(L.lib().vs_act_backward_colsum(L.dtype_code(x), int(ctx.act), L.ptr(gy), L.ptr(x), L.ptr(gx),
                                                   L.ptr(cs), L.ptr(ws), M, N, L.stream(x)), "act_backward_colsum")
        attach_colsum(gx, cs)
        return gx, None, None


class _GeluRowQuantFunction(torch.autograd.Function):
    """y = gelu(x) (exact erf) plus y's row-wise e4m3 copy (q, scale) for the next vendor
    fp8 GEMM, from one HIP pass over x (vs_gelu_row_quantize_fp8); q / scale are not
    differentiable (straight-through: the next Linear's backward uses y).  Backward: that of
    _ActColsumFunction (dx and the preceding Linear's bias gradient in one pass)."""

    @staticmethod
    def forward(ctx, x):
        ctx.act = 1
        ctx.save_for_backward(x)
        y, q, sc = row_quantize_fp8(x, gelu=True)
        ctx.mark_non_differentiable(q, sc)
        return y.view(x.shape), q, sc

    @staticmethod
    def backward(ctx, gy, gq=None, gs=None):
        return _ActColsumFunction.backward(ctx, gy)[0]


def gelu_row_quant(x):
    """(gelu(x), e4m3 rows of it, f32 row scales) -- see _GeluRowQuantFunction; x a
    contiguous bf16 device tensor with a gradient path."""
    return _GeluRowQuantFunction.apply(x)


def activation(x, kind: str, gelu_sink=None):
    """F.gelu / F.relu whose backward feeds the preceding Linear's bias gradient (see
    _ActColsumFunction) on contiguous f32 / bf16 device tensors with N % 8 == 0 (gelu_sink:
    see GeluBackwardSink)."""
    act = {"relu": 0, "gelu": 1}[kind]
    N = x.shape[-1]
    if (x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and N % 8 == 0 and N <= COLSUM_MAX_N
            and x.is_contiguous() and torch.is_grad_enabled() and x.requires_grad and not torch.is_autocast_enabled()):
        return _ActColsumFunction.apply(x, act, gelu_sink)
    return F.gelu(x) if act == 1 else F.relu(x)


# ------------------------------------------------------------------ per-parameter clip
class FlatParams:
    """f32 parameters (or gradients) packed into one flat device buffer, each starting
    16-B aligned, with the chunk table of csrc/optim.hip for per-parameter clipping."""

    CHUNK = 1 << 16

    def __init__(self, shapes, device):
        self.shapes = [tuple(s) for s in shapes]
        self.offsets, off = [], 0
        for s in self.shapes:
            n = 1
            for d in s:
                n *= int(d)
            self.offsets.append((off, n))
            off += (n + 3) // 4 * 4
        self.total = off
        rows = []
        for (o, n) in self.offsets:
            first = len(rows)
            count = max(1, (n + self.CHUNK - 1) // self.CHUNK)
            for c in range(count):
                rows.append([o + c * self.CHUNK, max(0, min(self.CHUNK, n - c * self.CHUNK)), first, count])
        self.num_chunks = len(rows)
        self.table = torch.tensor(rows, dtype=torch.int32).to(device)
        self.device = torch.device(device)
        self.ws = torch.empty(int(L.lib().vs_segment_clip_workspace_bytes(self.num_chunks)) if self.device.type == "cuda"
                              else 0, device=device, dtype=torch.uint8)

    def buffer(self):
        return torch.zeros(self.total, device=self.device, dtype=torch.float32)

    def views(self, flat):
        return [flat[o:o + n].view(s) for (o, n), s in zip(self.offsets, self.shapes)]

    def clip_(self, flat, max_norm: float, eps: float = 1e-6):
        """In place: every parameter's slice scaled to L2 norm <= max_norm (clip_grad_norm_
        per parameter, detectron2 "norm")."""
        L.require_hip(flat)
        with timed("segment_clip", flat, bytes_=3 * self.total * 4):
            L.check(L.lib().vs_segment_clip(L.ptr(flat), L.ptr(self.table), self.num_chunks, float(max_norm),
                                            float(eps), L.ptr(self.ws), L.stream(flat)), "segment_clip")


# ------------------------------------------------------------------ matching
def lsa_max_targets(num_queries: int) -> int:
    return int(L.lib().vs_lsa_max_targets(int(num_queries)))


def linear_sum_assignment_batch(cost, targets_per_image):
    """cost [S, B, Q, Kmax] f32 (device) + per-image target counts (host ints) ->
    int32 [S, B, Kmax]: the query matched to each target, -1 past the count
    (csrc/match.hip; scipy linear_sum_assignment semantics per (step, image))."""
    import ctypes
    L.require_hip(cost)
    c = cost.float().contiguous()
    S, B, Q, K = c.shape
    ks = (ctypes.c_int * B)(*[int(k) for k in targets_per_image])
    out = torch.empty(S, B, K, device=c.device, dtype=torch.int32)
    with timed("lsa", c, bytes_=c.numel() * 4):
        L.check(L.lib().vs_lsa_batch(L.ptr(c), ks, S, B, Q, K, L.ptr(out), L.stream(c)), "lsa_batch")
    return out


def linear_sum_assignment_padded(cost, counts):
    """cost [S, B, Q, K] f32 (device) + per-image target counts int32 [B] ON THE DEVICE ->
    int32 [S, B, K] (-1 past each count).  The launch does not depend on the counts, so a
    captured graph serves any counts <= K (csrc/match.hip vs_lsa_batch_device_counts)."""
    L.require_hip(cost, counts)
    c = cost.float().contiguous()
    S, B, Q, K = c.shape
    cnt = counts.to(torch.int32).contiguous()
    if cnt.numel() != B:
        raise ValueError(f"counts has {cnt.numel()} entries for a batch of {B}")
    out = torch.empty(S, B, K, device=c.device, dtype=torch.int32)
    with timed("lsa", c, bytes_=c.numel() * 4):
        L.check(L.lib().vs_lsa_batch_device_counts(L.ptr(c), L.ptr(cnt), S, B, Q, K, L.ptr(out), L.stream(c)),
                "lsa_batch_device_counts")
    return out


def match_cost(masks_list, probs, target_classes, points, target_labels, mask_weight, class_weight, dice_weight):
    """Hungarian-matcher cost for all decoder steps (csrc/match.hip match_cost_kernel).
    masks_list: S x f32 [B,Q,H,W]; probs f32 [S,B,Q,C+1]; target_classes int64 [B,Kc];
    points f32 [B,P,2] in [-1,1]; target_labels f32 [B,Kc,P] -> cost f32 [S,B,Q,Kc]."""
    ms = [m.float().contiguous() for m in masks_list]
    L.require_hip(*ms, probs, target_classes, points, target_labels)
    S = len(ms)
    B, Q, H, W = ms[0].shape
    pr = probs.float().contiguous()
    tc = target_classes.to(torch.int64).contiguous()
    pts = points.float().contiguous()
    tl = target_labels.float().contiguous()
    Kc, P = int(tl.shape[1]), int(tl.shape[2])
    if tuple(pts.shape) != (B, P, 2) or tuple(tc.shape) != (B, Kc) or tuple(pr.shape[:3]) != (S, B, Q):
        raise ValueError("match_cost: inconsistent shapes")
    cost = torch.empty(S, B, Q, Kc, device=pr.device, dtype=torch.float32)
    ptrs = (ctypes.c_void_p * S)(*[m.data_ptr() for m in ms])
    with timed("match_cost", pr, bytes_=sum(m.numel() for m in ms) * 4):
        L.check(L.lib().vs_match_cost(ptrs, S, L.ptr(pr), int(pr.shape[3]), L.ptr(tc), L.ptr(pts), L.ptr(tl),
                                      L.ptr(cost), B, Q, H, W, P, Kc, float(mask_weight), float(class_weight),
                                      float(dice_weight), L.stream(pr)), "match_cost")
    return cost


# ------------------------------------------------------------------ GroupNorm (channels-last)
class GroupNormNHWCFunction(torch.autograd.Function):
    """group_norm (+ optional ReLU) of an NCHW tensor stored channels-last, groups of 8
    channels (csrc/groupnorm.hip); returns a channels-last NCHW tensor."""

    @staticmethod
    def forward(ctx, x, weight, bias, groups, eps, relu):
        L.require_hip(x, weight, bias)
        B, C, H, W = x.shape
        xt = x.permute(0, 2, 3, 1)
        if not xt.is_contiguous():
            xt = xt.contiguous()
        y = torch.empty_like(xt)
        mean = torch.empty(B * groups, device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        ws = torch.empty(int(L.lib().vs_group_norm_workspace_bytes(B, H * W, C, groups)), device=x.device,
                         dtype=torch.uint8)
        with timed("group_norm_fwd", xt, bytes_=3 * xt.numel() * xt.element_size()):
            L.check(L.lib().vs_group_norm_forward(L.dtype_code(xt), L.ptr(xt), L.ptr(weight), L.ptr(bias), L.ptr(y),
                                                  L.ptr(mean), L.ptr(rstd), L.ptr(ws), B, H * W, C, groups,
                                                  float(eps), int(relu), L.stream(xt)), "group_norm_forward")
        ctx.save_for_backward(xt, weight, bias, mean, rstd)
        ctx.cfg = (groups, bool(relu))
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gy):
        xt, weight, bias, mean, rstd = ctx.saved_tensors
        groups, relu = ctx.cfg
        B, H, W, C = xt.shape
        gyt = gy.permute(0, 2, 3, 1).to(xt.dtype)
        if not gyt.is_contiguous():
            gyt = gyt.contiguous()
        gx = torch.empty_like(xt)
        gw, gb = torch.empty_like(weight), torch.empty_like(bias)
        ws = torch.empty(int(L.lib().vs_group_norm_workspace_bytes(B, H * W, C, groups)), device=xt.device,
                         dtype=torch.uint8)
        with timed("group_norm_bwd", xt, bytes_=5 * xt.numel() * xt.element_size()):
            L.check(L.lib().vs_group_norm_backward(L.dtype_code(xt), L.ptr(gyt), L.ptr(xt), L.ptr(weight), L.ptr(bias),
                                                   L.ptr(mean), L.ptr(rstd), L.ptr(gx), L.ptr(gw), L.ptr(gb),
                                                   L.ptr(ws), B, H * W, C, groups, int(relu), L.stream(xt)),
                    "group_norm_backward")
        return gx.permute(0, 3, 1, 2), gw, gb, None, None, None


def group_norm_nhwc(x, weight, bias, groups: int, eps: float = 1e-5, relu: bool = False):
    return GroupNormNHWCFunction.apply(x, weight, bias, int(groups), float(eps), bool(relu))


class GroupNormNCHWFunction(torch.autograd.Function):
    """group_norm (+ optional ReLU) of an NCHW-contiguous tensor (csrc/groupnorm.hip NCHW
    kernels: a group is C/G contiguous channel planes); returns an NCHW-contiguous tensor."""

    @staticmethod
    def forward(ctx, x, weight, bias, groups, eps, relu):
        L.require_hip(x, weight, bias)
        B, C, H, W = x.shape
        x = x.contiguous()
        y = torch.empty_like(x)
        mean = torch.empty(B * groups, device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        ws = torch.empty(int(L.lib().vs_group_norm_nchw_workspace_bytes(B, C, groups)), device=x.device,
                         dtype=torch.uint8)
        with timed("group_norm_nchw_fwd", x, bytes_=3 * x.numel() * x.element_size()):
            L.check(L.lib().vs_group_norm_nchw_forward(L.dtype_code(x), L.ptr(x), L.ptr(weight), L.ptr(bias),
                                                       L.ptr(y), L.ptr(mean), L.ptr(rstd), L.ptr(ws), B, C, H * W,
                                                       groups, float(eps), int(relu), L.stream(x)),
                    "group_norm_nchw_forward")
        ctx.save_for_backward(x, weight, bias, mean, rstd)
        ctx.cfg = (groups, bool(relu))
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight, bias, mean, rstd = ctx.saved_tensors
        groups, relu = ctx.cfg
        B, C, H, W = x.shape
        gy = gy.to(x.dtype).contiguous()
        gx = torch.empty_like(x)
        gw, gb = torch.empty_like(weight), torch.empty_like(bias)
        ws = torch.empty(int(L.lib().vs_group_norm_nchw_workspace_bytes(B, C, groups)), device=x.device,
                         dtype=torch.uint8)
        with timed("group_norm_nchw_bwd", x, bytes_=5 * x.numel() * x.element_size()):
            L.check(L.lib().vs_group_norm_nchw_backward(L.dtype_code(x), L.ptr(gy), L.ptr(x), L.ptr(weight),
                                                        L.ptr(bias), L.ptr(mean), L.ptr(rstd), L.ptr(gx), L.ptr(gw),
                                                        L.ptr(gb), L.ptr(ws), B, C, H * W, groups, int(relu),
                                                        L.stream(x)), "group_norm_nchw_backward")
        return gx, gw, gb, None, None, None


def group_norm_nchw(x, weight, bias, groups: int, eps: float = 1e-5, relu: bool = False):
    return GroupNormNCHWFunction.apply(x, weight, bias, int(groups), float(eps), bool(relu))


# ------------------------------------------------------------------ FPN merge (upsample + add)
class UpsampleAddFunction(torch.autograd.Function):
    """out = cur + bilinear_upsample(src) (csrc/upsample.hip): cur NCHW [B,C,H,W]
    contiguous, src token-major [B, Hs*Ws, C] (rows contiguous, any batch stride)."""

    @staticmethod
    def forward(ctx, cur, src, Hs, Ws):
        L.require_hip(cur, src)
        B, C, H, W = cur.shape
        cur = cur.contiguous()
        src = src.to(cur.dtype)
        if src.stride(2) != 1 or src.stride(1) != C:
            src = src.contiguous()
        if tuple(src.shape) != (B, Hs * Ws, C):
            raise ValueError(f"src {tuple(src.shape)} != {(B, Hs * Ws, C)}")
        out = torch.empty_like(cur)
        with timed("upsample_add", cur, bytes_=(2 * cur.numel() + src.numel()) * cur.element_size()):
            L.check(L.lib().vs_upsample_add_forward(L.dtype_code(cur), L.ptr(cur), L.ptr(src), L.ptr(out), B, C, H,
                                                    W, int(Hs), int(Ws), src.stride(0), L.stream(cur)),
                    "upsample_add_forward")
        ctx.geom = (B, C, H, W, int(Hs), int(Ws))
        ctx.src_dtype = src.dtype
        return out

    @staticmethod
    def backward(ctx, g):
        B, C, H, W, Hs, Ws = ctx.geom
        g = g.contiguous()
        gs = torch.empty(B, Hs * Ws, C, device=g.device, dtype=g.dtype)
        with timed("upsample_bwd", g, bytes_=(g.numel() + gs.numel()) * g.element_size()):
            L.check(L.lib().vs_upsample_backward(L.dtype_code(g), L.ptr(g), L.ptr(gs), B, C, H, W, Hs, Ws,
                                                 L.stream(g)), "upsample_backward")
        return g, gs.to(ctx.src_dtype), None, None


def upsample_add(cur, src_tokens, Hs: int, Ws: int):
    return UpsampleAddFunction.apply(cur, src_tokens, int(Hs), int(Ws))


class UpsampleAddNHWCFunction(torch.autograd.Function):
    """UpsampleAddFunction on channels-last planes (csrc/upsample.hip NHWC forms): cur an
    NCHW-shaped tensor stored channels-last, src token-major [B, Hs*Ws, C]; returns a
    channels-last NCHW view."""

    @staticmethod
    def forward(ctx, cur, src, Hs, Ws):
        L.require_hip(cur, src)
        B, C, H, W = cur.shape
        ct = cur.permute(0, 2, 3, 1)
        if not ct.is_contiguous():
            ct = ct.contiguous()
        src = src.to(cur.dtype)
        if src.stride(2) != 1 or src.stride(1) != C or src.stride(0) % 8 or src.data_ptr() % 16:
            src = src.contiguous()
        if tuple(src.shape) != (B, Hs * Ws, C):
            raise ValueError(f"src {tuple(src.shape)} != {(B, Hs * Ws, C)}")
        out = torch.empty_like(ct)
        with timed("upsample_add_nhwc", ct, bytes_=(2 * ct.numel() + src.numel()) * ct.element_size()):
            L.check(L.lib().vs_upsample_add_forward_nhwc(L.dtype_code(ct), L.ptr(ct), L.ptr(src), L.ptr(out), B, C,
                                                         H, W, int(Hs), int(Ws), src.stride(0), L.stream(ct)),
                    "upsample_add_forward_nhwc")
        ctx.geom = (B, C, H, W, int(Hs), int(Ws))
        ctx.src_dtype = src.dtype
        return out.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, g):
        B, C, H, W, Hs, Ws = ctx.geom
        gt = g.permute(0, 2, 3, 1)
        if not gt.is_contiguous():
            gt = gt.contiguous()
        gs = torch.empty(B, Hs * Ws, C, device=g.device, dtype=g.dtype)
        with timed("upsample_bwd_nhwc", gt, bytes_=(gt.numel() + gs.numel()) * gt.element_size()):
            L.check(L.lib().vs_upsample_backward_nhwc(L.dtype_code(gt), L.ptr(gt), L.ptr(gs), B, C, H, W, Hs, Ws,
                                                      L.stream(gt)), "upsample_backward_nhwc")
        return g, gs.to(ctx.src_dtype), None, None


def upsample_add_nhwc(cur, src_tokens, Hs: int, Ws: int):
    return UpsampleAddNHWCFunction.apply(cur, src_tokens, int(Hs), int(Ws))


# ------------------------------------------------------------------ token-Linear weight gradient
def token_wgrad(gy, x, out_dtype, bias: bool = False, out=None, bias_out=None):
    """dW [N, K] = gy^T x for token-major gy [T, N], x [T, K] (bf16, rows strided, unit
    column stride), f32 accumulation, out_dtype; bias=True also returns db [N] = column sums
    of gy (csrc/token_wgrad.hip).  `out` / `bias_out`: contiguous [N, K] / [N] tensors of
    out_dtype to write into (e.g. row blocks of a fused parameter's gradients)."""
    L.require_hip(gy, x)
    T, N = gy.shape
    K = x.shape[1]
    dev = gy.device
    nb = int(L.lib().vs_token_wgrad_workspace_bytes(T, N, K))
    ws = torch.empty(nb, device=dev, dtype=torch.uint8)
    if out is None:
        out = torch.empty(N, K, device=dev, dtype=out_dtype)
    db = (bias_out if bias_out is not None else torch.empty(N, device=dev, dtype=out_dtype)) if bias else None
    with timed("token_wgrad", gy, flops=2.0 * T * N * K, bytes_=T * (N + K) * 2):
        L.check(L.lib().vs_token_wgrad(L.dtype_code(out), L.ptr(gy), gy.stride(0), L.ptr(x), x.stride(0), L.ptr(out),
                                       L.ptr(db) if bias else None, L.ptr(ws), T, N, K, L.stream(gy)), "token_wgrad")
    return (out, db) if bias else out


class WgradProblem(ctypes.Structure):
    """vs_wgrad_problem (include/visionseg.h)."""
    _fields_ = [("grad_y", ctypes.c_void_p), ("x", ctypes.c_void_p), ("dw", ctypes.c_void_p),
                ("db", ctypes.c_void_p), ("ld_grad_y", ctypes.c_longlong), ("ld_x", ctypes.c_longlong),
                ("tokens", ctypes.c_longlong), ("N", ctypes.c_int), ("K", ctypes.c_int)]


def token_wgrad_grouped(items, out_dtype):
    """Several independent token-Linear weight gradients in one launch (+ one reduction launch
    when some are split): items = [(gy [T, N], x [T, K], dw [N, K], db [N] or None)], gy / x bf16
    with unit column stride, dw / db contiguous of out_dtype, all written
    (vs_token_wgrad_grouped)."""
    if not items:
        return
    L.require_hip(items[0][0])
    n = len(items)
    arr = (WgradProblem * n)()
    flops = 0.0
    for k, (gy, x, dw, db) in enumerate(items):
        pw = dw.data_ptr()
        pb = db.data_ptr() if db is not None else None
        arr[k] = WgradProblem(gy.data_ptr(), x.data_ptr(), pw, pb, gy.stride(0), x.stride(0), gy.shape[0],
                              gy.shape[1], x.shape[1])
        flops += 2.0 * gy.shape[0] * gy.shape[1] * x.shape[1]
    gy0 = items[0][0]
    nb = int(L.lib().vs_token_wgrad_grouped_workspace_bytes(arr, n))
    ws = torch.empty(max(nb, 16), device=gy0.device, dtype=torch.uint8)
    code = L.dtype_code(torch.empty(0, dtype=out_dtype))
    with timed("token_wgrad", gy0, flops=flops, bytes_=sum(it[0].shape[0] * (it[0].shape[1] + it[1].shape[1]) * 2
                                                           for it in items)):
        L.check(L.lib().vs_token_wgrad_grouped(code, arr, n, L.ptr(ws), L.stream(gy0)), "token_wgrad_grouped")


class TransposeItem(ctypes.Structure):
    """vs_transpose_item (include/visionseg.h)."""
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("rows", ctypes.c_int), ("cols", ctypes.c_int)]


def transpose_batched(pairs):
    """dst.copy_(src.t()) for every (src [R, C], dst [C, R]) pair -- contiguous bf16 device
    tensors, R % 8 == 0, C % 8 == 0 -- in one launch (vs_transpose_batched)."""
    if not pairs:
        return
    L.require_hip(pairs[0][0])
    arr = (TransposeItem * len(pairs))()
    for k, (src, dst) in enumerate(pairs):
        assert src.is_contiguous() and dst.is_contiguous() and dst.shape == (src.shape[1], src.shape[0])
        arr[k] = TransposeItem(src.data_ptr(), dst.data_ptr(), src.shape[0], src.shape[1])
    L.check(L.lib().vs_transpose_batched(L.VS_BF16, arr, len(pairs), L.stream(pairs[0][0])), "transpose_batched")


# ------------------------------------------------------------------ 3 x 3 conv (channels-last)
def conv3x3_nhwc_ok(x, weight) -> bool:
    """Shapes / dtypes csrc/conv3x3.hip covers: bf16 device tensors, a [Co, Ci, 3, 3] weight
    with Ci and Co multiples of 128 (forward, input and weight gradients)."""
    return (x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16
            and tuple(weight.shape[2:]) == (3, 3) and weight.shape[1] == x.shape[1]
            and x.shape[1] % 128 == 0 and weight.shape[0] % 128 == 0)


def conv3x3_layouts(weight, fwd=True, bwd=False):
    """weight [Co, Ci, 3, 3] -> (w_fwd [Co, 3, 3, Ci] or None, w_bwd [Ci, 3, 3, Co] flipped or None)."""
    L.require_hip(weight)
    Co, Ci = weight.shape[:2]
    w = weight.contiguous()
    wf = torch.empty(Co, 3, 3, Ci, device=w.device, dtype=w.dtype) if fwd else None
    wb = torch.empty(Ci, 3, 3, Co, device=w.device, dtype=w.dtype) if bwd else None
    L.check(L.lib().vs_conv3x3_weight_layouts(L.ptr(w), L.ptr(wf) if wf is not None else None,
                                              L.ptr(wb) if wb is not None else None, Co, Ci, L.stream(w)),
            "conv3x3_weight_layouts")
    return wf, wb


def conv3x3_raw(xt, w_layout, bias=None):
    """y [B, H, W, Co] = conv3x3(xt [B, H, W, Ci]) with the weights in the vs_conv3x3_forward
    layout [Co, 3, 3, Ci] (the input gradient: grad_y and the w_bwd layout)."""
    L.require_hip(xt, w_layout)
    B, H, W, Ci = xt.shape
    Co = w_layout.shape[0]
    y = torch.empty(B, H, W, Co, device=xt.device, dtype=xt.dtype)
    with timed("conv3x3_igemm", xt, flops=2.0 * B * H * W * Co * 9 * Ci):
        L.check(L.lib().vs_conv3x3_forward(L.ptr(xt), L.ptr(w_layout), L.ptr(bias) if bias is not None else None,
                                           L.ptr(y), B, H, W, Ci, Co, L.stream(xt)), "conv3x3_forward")
    return y


def conv3x3_wgrad(gyt, xt, dtype):
    """dW [Co, Ci, 3, 3] (dtype) = sum over pixels of gyt [B, H, W, Co] x the 3 x 3
    neighbourhoods of xt [B, H, W, Ci] (vs_conv3x3_wgrad)."""
    B, H, W, Ci = xt.shape
    Co = gyt.shape[3]
    nb = int(L.lib().vs_conv3x3_wgrad_workspace_bytes(B, H, W, Ci, Co))
    if nb <= 0:
        raise ValueError(f"conv3x3_wgrad: unsupported shape {tuple(xt.shape)} -> {Co}")
    ws = torch.empty(nb, device=xt.device, dtype=torch.uint8)
    gw = torch.empty(Co, Ci, 3, 3, device=xt.device, dtype=dtype)
    with timed("conv3x3_wgrad", xt, flops=2.0 * B * H * W * Co * 9 * Ci):
        L.check(L.lib().vs_conv3x3_wgrad(L.dtype_code(gw), L.ptr(gyt), L.ptr(xt), L.ptr(gw), L.ptr(ws), B, H, W, Ci,
                                         Co, L.stream(xt)), "conv3x3_wgrad")
    return gw


class Conv3x3NHWCFunction(torch.autograd.Function):
    """nn.functional.conv2d(x, weight, bias, stride=1, padding=1) for a 3 x 3 kernel on a
    channels-last bf16 NCHW tensor (csrc/conv3x3.hip): the pixel decoder's output conv
    (HF:m2f:1394-1419).  Returns a channels-last NCHW view."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        L.require_hip(x, weight)
        if not conv3x3_nhwc_ok(x, weight):
            raise ValueError(f"conv3x3_nhwc: unsupported x {tuple(x.shape)} {x.dtype}, weight {tuple(weight.shape)}")
        xt = x.permute(0, 2, 3, 1)
        if not xt.is_contiguous():
            xt = xt.contiguous()
        wf, _ = conv3x3_layouts(weight)
        b = bias.to(x.dtype).contiguous() if bias is not None else None
        y = conv3x3_raw(xt, wf, b)
        ctx.save_for_backward(xt, weight)
        ctx.has_bias = bias is not None
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gy):
        xt, weight = ctx.saved_tensors
        gyt = gy.permute(0, 2, 3, 1).to(xt.dtype)
        if not gyt.is_contiguous():
            gyt = gyt.contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            _, wb = conv3x3_layouts(weight, fwd=False, bwd=True)
            gx = conv3x3_raw(gyt, wb).permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1]:
            gw = conv3x3_wgrad(gyt, xt, weight.dtype)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = gyt.sum((0, 1, 2), dtype=torch.float32).to(weight.dtype)
        return gx, gw, gb


def conv3x3_nhwc(x, weight, bias=None):
    return Conv3x3NHWCFunction.apply(x, weight, bias)


# ---------------------------------------------------------------------------------------
# token GEMM (csrc/token_gemm.hip): the Swin blocks' Linears, bf16 or block-scaled MX fp8
# ---------------------------------------------------------------------------------------
TGEMM_FP8, TGEMM_GELU, TGEMM_QOUT, TGEMM_GELU_BWD, TGEMM_RELU_BWD = 1, 2, 4, 8, 16


def mx_quantize(x: torch.Tensor):
    """bf16 [..., K] (K % 32 == 0) -> (e4m3 bytes uint8 [..., K], e8m0 scale bytes uint8
    [..., K / 32]): one power-of-two scale per 32 elements along K (vs_mx_quantize)."""
    L.require_hip(x)
    if x.dtype != torch.bfloat16 or x.shape[-1] % 32:
        raise ValueError("mx_quantize: bf16 rows with K % 32 == 0")
    x = x.contiguous()
    K = x.shape[-1]
    rows = x.numel() // K
    q = torch.empty(x.shape, device=x.device, dtype=torch.uint8)
    s = torch.empty(*x.shape[:-1], K // 32, device=x.device, dtype=torch.uint8)
    with timed("mx_quantize", x, bytes_=x.numel() * 3 + s.numel()):
        L.check(L.lib().vs_mx_quantize(L.ptr(x), L.ptr(q), L.ptr(s), rows, K, L.stream(x)), "mx_quantize")
    return q, s


def row_quantize_fp8(x: torch.Tensor, gelu: bool = False):
    """bf16 [..., K] -> (q float8_e4m3fn [rows, K], scale f32 [rows, 1]) with x ~= q * scale
    per row (power-of-two scales; csrc/fp8_rows.hip), the operand form of the vendor
    rowwise fp8 GEMM (torch._scaled_mm).  gelu=True: quantises gelu(x) (exact erf) and also
    returns it in bf16: (y, q, scale)."""
    L.require_hip(x)
    if x.dtype != torch.bfloat16 or x.shape[-1] % 8:
        raise ValueError("row_quantize_fp8: bf16 rows with K % 8 == 0")
    x = x.contiguous()
    K = x.shape[-1]
    rows = x.numel() // K
    q = torch.empty(rows, K, device=x.device, dtype=torch.float8_e4m3fn)
    sc = torch.empty(rows, 1, device=x.device, dtype=torch.float32)
    if gelu:
        y = torch.empty_like(x)
        with timed("gelu_row_quantize", x, bytes_=x.numel() * 5 + rows * 4):
            L.check(L.lib().vs_gelu_row_quantize_fp8(L.ptr(x), L.ptr(y), L.ptr(q), L.ptr(sc), rows, K, L.stream(x)),
                    "gelu_row_quantize_fp8")
        return y, q, sc
    with timed("row_quantize", x, bytes_=x.numel() * 3 + rows * 4):
        L.check(L.lib().vs_row_quantize_fp8(L.ptr(x), L.ptr(q), L.ptr(sc), rows, K, L.stream(x)), "row_quantize_fp8")
    return q, sc


def token_gemm(x, w, bias=None, gelu: bool = False, x_scales=None, w_scales=None, quant_out: bool = False,
               gelu_pre=None, relu_out=None):
    """y = x w^T + bias over token rows (x [..., K], w [N, K]; bf16, or -- with scales --
    e4m3 bytes from mx_quantize) -> bf16 [..., N]; gelu=True -> (gelu(y), y) with the exact
    erf GELU in the epilogue (y = the bf16 pre-activation); quant_out=True (with gelu) ->
    (gelu(y), y, (e4m3 bytes, e8m0 scales) of gelu(y), as mx_quantize would make them).
    gelu_pre ([..., N] bf16, no bias): the GELU BACKWARD in the epilogue -> bf16(x w^T) *
    gelu'(gelu_pre), each product rounded once (VS_TGEMM_GELU_BWD: fc2's dX of an MLP);
    relu_out (the same for a ReLU, given its OUTPUT): bf16(x w^T) * [relu_out > 0]."""
    fp8 = x_scales is not None
    if relu_out is not None:
        if gelu_pre is not None:
            raise ValueError("token_gemm: one activation backward")
        gelu_pre, act_mode = relu_out, TGEMM_RELU_BWD
    else:
        act_mode = TGEMM_GELU_BWD
    L.require_hip(x, w)
    K = x.shape[-1]
    N = w.shape[0]
    if w.shape[1] != K or N % 4 or (fp8 and (w_scales is None or K % 128)) or (not fp8 and K % 8) \
            or (quant_out and (not gelu or N % 32)) \
            or (gelu_pre is not None and (fp8 or gelu or bias is not None or N % 8 or gelu_pre.dtype != torch.bfloat16
                                          or gelu_pre.numel() != x.numel() // K * N)):
        raise ValueError(f"token_gemm: bad shapes x {tuple(x.shape)} w {tuple(w.shape)} fp8={fp8}")
    x2 = x.reshape(-1, K).contiguous()
    w = w.contiguous()
    # the kernel's 16-B LDS-DMA rows, 8-B bias and 4-B scale loads: a view with a storage
    # offset that breaks them is copied to a fresh (aligned) buffer
    if x2.data_ptr() % 16:
        x2 = x2.clone()
    if w.data_ptr() % 16:
        w = w.clone()
    if bias is not None:
        bias = bias.contiguous()
        if bias.data_ptr() % 8:
            bias = bias.clone()
    M = x2.shape[0]
    y = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    pre = torch.empty_like(y) if gelu else None
    yq = torch.empty(M, N, device=x.device, dtype=torch.uint8) if quant_out else None
    yqs = torch.empty(M, N // 32, device=x.device, dtype=torch.uint8) if quant_out else None
    mode = (TGEMM_FP8 if fp8 else 0) | (TGEMM_GELU if gelu else 0) | (TGEMM_QOUT if quant_out else 0)
    if gelu_pre is not None:
        mode |= act_mode
        pre = gelu_pre.reshape(M, N).contiguous()
        if pre.data_ptr() % 16:
            pre = pre.clone()
    esz = 1 if fp8 else 2
    nb = (M * K + N * K) * esz + M * N * 2 * (2 if gelu or gelu_pre is not None else 1) + \
        (M * N * 33 // 32 if quant_out else 0)
    with timed("token_gemm_fp8" if fp8 else "token_gemm", x2, bytes_=nb, flops=2.0 * M * N * K):
        L.check(L.lib().vs_token_gemm(mode, L.ptr(x2), L.ptr(x_scales.contiguous()) if fp8 else None,
                                      L.ptr(w), L.ptr(w_scales.contiguous()) if fp8 else None,
                                      L.ptr(bias) if bias is not None else None, L.ptr(y),
                                      L.ptr(pre) if gelu or gelu_pre is not None else None,
                                      L.ptr(yq) if quant_out else None,
                                      L.ptr(yqs) if quant_out else None, M, N, K, L.stream(x2)), "token_gemm")
    shape = (*x.shape[:-1], N)
    if quant_out:
        return y.view(shape), pre.view(shape), (yq.view(shape), yqs.view(*x.shape[:-1], N // 32))
    if gelu:
        return y.view(shape), pre.view(shape)
    return y.view(shape)
