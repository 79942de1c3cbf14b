"""Token-major Linear with a split-K weight gradient.

The backbone and pixel-decoder Linears see tens to hundreds of thousands of tokens
(Swin-T stage 1 at 1024^2, batch 4: K = 268k) but only a few hundred output features,
so the weight gradient dW[out,in] = dY^T X is a tall-K GEMM whose M x N is a handful
of macro-tiles: one launch of the library kernel fills ~10 of the 256 CUs.  Here the
K (token) axis is cut into S chunks and run as one batched GEMM with f32 outputs
[S, out, in] (every CU busy), then reduced over S in f32 and rounded once.  Forward and
dX are the plain library GEMMs.  Parameter names are nn.Linear's, so checkpoints and
visionseg.convert are unaffected.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib as L
from . import ops

import ctypes
import os

# Linears over at least this many tokens take the token path (_LinearFn: the token GEMM where
# its shape rule picks it, token_wgrad with the fused bias column sums, residual sinks).  4096
# (round 6) takes in Swin-T stage 4 (4 x 32 x 32 tokens), whose bias gradients were ATen
# reductions (16 launches, 0.30 ms of the C2 step, profiles/r6_step_graph_c2_selfattn.txt);
# measured +0.4 % img/s against 16384 at the end of round 5 (profiles/r5_min_tokens_ab.txt)
MIN_TOKENS = int(os.environ.get("VS_SPLITK_MIN_TOKENS", "4096"))

GEMM_TABLE = os.environ.get("VS_GEMM_TABLE") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                             "tuning", "tunableop_mi355x.csv")


def load_gemm_table(path: str = GEMM_TABLE) -> bool:
    """Use the shipped vendor-GEMM solution table (PyTorch TunableOp over hipBLASLt /
    rocBLAS, tuned on MI355X for the bench configs by tools/retune.sh) for every later
    GEMM of this process, without tuning: shapes it lacks run the default heuristic.

    Loaded through the Python API on purpose: TunableOp inserts the device ordinal into a
    PYTORCH_TUNABLEOP_FILENAME without "%d" ("x.csv" -> "x0.csv" on device 0), so the
    environment variable alone never read this file, and a "%d" name would need one copy
    per GPU.  Returns False (nothing enabled) when the file or a device is missing."""
    if not (os.path.exists(path) and torch.cuda.is_available()):
        return False
    from torch.cuda import tunable
    tunable.enable(True)
    tunable.tuning_enable(False)
    tunable.set_filename(path, False)
    return bool(tunable.read_file(path))


MIN_CHUNK = 1024
TARGET_TILES = 768   # 128x128 output tiles over all chunks (1536: C2 -0.8 %, C5 +1.2 % img/s, round 3)


def split_count(K: int, M: int, N: int) -> int:
    tiles = max(1, -(-M // 128) * -(-N // 128))
    s = max(1, TARGET_TILES // tiles)
    return max(1, min(s, K // MIN_CHUNK))


# The token-Linear weight gradient on the hand-written kernel (csrc/token_wgrad.hip) for
# bf16 operands with >= WGRAD_MIN_TOKENS tokens; VS_TOKEN_WGRAD=0: the vendor batched GEMM.
_TOKEN_WGRAD = os.environ.get("VS_TOKEN_WGRAD", "1") == "1"
WGRAD_MIN_TOKENS = 4096


def _token_wgrad_ok(gy, x, out_dtype) -> bool:
    return (_TOKEN_WGRAD and gy.is_cuda and gy.dtype == x.dtype == torch.bfloat16
            and out_dtype in (torch.float32, torch.bfloat16) and gy.shape[0] >= WGRAD_MIN_TOKENS
            and gy.shape[1] % 8 == 0 and x.shape[1] % 8 == 0 and gy.stride(1) == 1 and x.stride(1) == 1
            and gy.stride(0) % 8 == 0 and x.stride(0) % 8 == 0 and gy.data_ptr() % 16 == 0
            and x.data_ptr() % 16 == 0)


def weight_grad(gy: torch.Tensor, x: torch.Tensor, out_dtype: torch.dtype, out: torch.Tensor | None = None,
                bias: bool = False, bias_out=None):
    """dW = gy^T x for gy [K, M], x [K, N] -> [M, N] (out_dtype), f32 accumulation.  bf16
    token-heavy operands: the hand-written token weight-gradient kernel (ops.token_wgrad);
    otherwise a batched GEMM over S token chunks with f32 outputs, then one HIP epilogue
    that sums the chunks (+ the remainder rows' product) and rounds once (csrc/norm.hip).
    `out`: a contiguous [M, N] tensor of out_dtype to write into (e.g. a row block of a
    fused parameter's gradient).  bias=True: returns (dW, db) with db = gy's column sums
    (f32 accumulation, out_dtype) -- from the same kernel on the token path."""
    if _token_wgrad_ok(gy, x, out_dtype) and (out is None or (out.is_contiguous() and out.dtype == out_dtype
                                                               and out.data_ptr() % 16 == 0)) \
            and (bias_out is None or (bias_out.is_contiguous() and bias_out.data_ptr() % 16 == 0)):
        res = ops.token_wgrad(gy, x, out_dtype, bias=bias, out=out, bias_out=bias_out)
        return res
    gw = _vendor_weight_grad(gy, x, out_dtype, out)
    if bias:
        gy = gy.contiguous()
        if gy.shape[1] % 8 == 0 and gy.shape[1] <= ops.COLSUM_MAX_N and gy.is_cuda:
            return gw, ops.column_sum(gy).to(out_dtype)
        return gw, gy.sum(0, dtype=torch.float32).to(out_dtype)
    return gw


def _vendor_weight_grad(gy, x, out_dtype, out=None):
    K, M = gy.shape
    N = x.shape[1]
    S = split_count(K, M, N)
    if S <= 1 or (M * N) % 4 or out_dtype not in (torch.float32, torch.bfloat16):
        g = (gy.t() @ x).to(out_dtype)
        return g if out is None else out.copy_(g)
    chunk = K // S
    main = chunk * S
    part = torch.bmm(gy[:main].view(S, chunk, M).transpose(1, 2), x[:main].view(S, chunk, N),
                     out_dtype=torch.float32)
    extra = torch.mm(gy[main:].t(), x[main:], out_dtype=torch.float32) if main < K else None
    if out is None:
        out = torch.empty(M, N, device=gy.device, dtype=out_dtype)
    L.check(L.lib().vs_splitk_sum(L.dtype_code(out), L.ptr(part), S, M * N, L.ptr(extra) if extra is not None else None,
                                  L.ptr(out), L.stream(out)), "splitk_sum")
    return out


# Forward of the token Linears: the hand-written token GEMM (csrc/token_gemm.hip) on the
# shapes where it beat the vendor GEMM on the box, by a STATIC shape rule (the same choice in
# every process and on every rank, so the bf16 rounding of a Linear never depends on a
# timing).  From tools/tgemm_bench.py (profiles/r4_tgemm_bench3.txt, M = tokens):
#   * K <= 384 and N < 4K (qkv, proj, and fc2 from a narrow stage): C2 stages 1-3 qkv / proj
#     1.1-1.4x, stage-1 fc2 1.35x; the fc1 shapes (N = 4K) are ties or vendor wins;
#   * M <= 16384, N <= 768, K <= 1536 (C2 stage-3 fc2, stage-4 proj): 1.2-1.3x;
#   * never above 300 000 tokens: C5 stage 1 (589 824) runs 0.8x of the vendor GEMM.
# VS_TGEMM_FWD=0: always the vendor GEMM.
_TGEMM_FWD = os.environ.get("VS_TGEMM_FWD", "1") == "1"


def _use_token_gemm(M: int, N: int, K: int) -> bool:
    if M > 300_000:
        return False
    return (K <= 384 and N < 4 * K) or (M <= 16384 and N <= 768 and K <= 1536)


def _forward_gemm(x, weight, bias):
    """x W^T + b inside _LinearFn.forward (grad mode is off there, so no _tgemm_ok)."""
    N, K = weight.shape
    if not (_TGEMM_FWD and x.is_cuda and x.dtype == weight.dtype == torch.bfloat16 and x.is_contiguous()
            and (bias is None or bias.dtype == torch.bfloat16) and K % 8 == 0 and N % 8 == 0
            and x.numel() // K >= MIN_TOKENS and _use_token_gemm(x.numel() // K, N, K)):
        return F.linear(x, weight, bias)
    return ops.token_gemm(x.reshape(-1, K), weight, bias).view(*x.shape[:-1], N)


def _addmm_into(c, a, b):
    """c + a @ b with the sum formed IN c (beta = 1 in the GEMM epilogue) when c is a
    contiguous tensor of the product's dtype: torch.addmm into a new output first copies c
    there (a full-size copyBuffer per call: ~15 us at the encoder's 87k x 256 tokens).  c is
    a gradient handed over by ops.ResidualSink -- owned by the caller, dead afterwards."""
    if c.dtype == a.dtype and c.is_contiguous():
        return c.addmm_(a, b)
    return torch.addmm(c.to(a.dtype), a, b)


# The input gradient dX = dY W of the token Linears on the token GEMM (with W^T, a [K, N]
# copy of the small weight), by a static shape rule from tools/r5/wgrad_ab.py
# (profiles/r5_wgrad_dgrad_ab.txt): the token GEMM won 1.0-1.5x at every C2 shape except the
# reductions >= 4x the output width below 100k tokens (encoder fc1, stage-4 fc1: ties or
# vendor wins).  VS_TGEMM_DGRAD=0: always the vendor GEMM.
_TGEMM_DGRAD = os.environ.get("VS_TGEMM_DGRAD", "1") == "1"


# Which dX GEMMs take the token GEMM: every T <= 300000 except the wide reductions of smaller
# T.  (Only where the isolated dX measured faster than hipBLASLt's dY W -- Swin-T stage 1 and
# the wide-output encoder fc2, profiles/r5_dgrad_ab.txt -- measured the same C2 step: 135.2 /
# 135.4 vs 135.6 img/s on one box, profiles/r5_dgrad_rule_ab.txt; that variant is gone.)
def _use_token_gemm_dgrad(T: int, K_out: int, N_red: int) -> bool:
    return T <= 300_000 and not (N_red >= 4 * K_out and T <= 100_000)


def _dgrad_on_token_gemm(T: int, weight, dtype) -> bool:
    N, K = weight.shape
    return (_TGEMM_DGRAD and weight.is_cuda and dtype == weight.dtype == torch.bfloat16 and K % 8 == 0
            and N % 8 == 0 and T >= MIN_TOKENS and _use_token_gemm_dgrad(T, K, N))


class _WeightTransposes:
    """W^T [K, N] copies of the token Linears' weights for the dX GEMM on the token GEMM
    (whose operands are both K-contiguous rows): requested in the forward (request), all
    written by ONE batched launch (ops.transpose_batched) at the first use in the backward
    (get).  Before, each dX GEMM made its own weight.t().contiguous(): 53 strided-copy
    launches per C2 step (0.33 ms, profiles/r6_glue_c2.txt).  The weights do not change
    between a forward and its backward (the optimizer steps after).  A request never used
    (a forward without backward) is dropped after `cap` newer ones; get() then falls back to
    its own copy."""

    def __init__(self, cap: int = 1024):
        self.pending = []
        self.cap = cap

    def request(self, weight):
        h = [weight, torch.empty(weight.shape[1], weight.shape[0], device=weight.device, dtype=weight.dtype), False]
        self.pending.append(h)
        if len(self.pending) > self.cap:
            self.pending.pop(0)
        return h

    def flush(self):
        by_dev = {}
        for h in self.pending:
            by_dev.setdefault(h[0].device, []).append(h)
        for hs in by_dev.values():
            ops.transpose_batched([(h[0].detach().contiguous(), h[1]) for h in hs])
            for h in hs:
                h[2] = True
        self.pending = []

    def get(self, h):
        if not h[2]:
            if any(p is h for p in self.pending):
                self.flush()
            else:                     # dropped: a copy of its own
                return h[0].t().contiguous()
        return h[1]


_WT = _WeightTransposes()


def _dgrad_gemm(gy2, weight, wt=None):
    """dX = dY W for dY [T, N] and W [N, K] (no residual term); wt: the _WT request made in
    the forward when this GEMM was known to run on the token GEMM."""
    if _dgrad_on_token_gemm(gy2.shape[0], weight, gy2.dtype) and gy2.is_cuda:
        return ops.token_gemm(gy2.contiguous(), _WT.get(wt) if wt is not None else weight.t().contiguous())
    return gy2 @ weight.to(gy2.dtype)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, sink=None, gelu_sink=None):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        ctx.sink = sink
        if sink is not None:
            sink.arm()
        # the dX GEMM's W^T (only where it runs without the residual term, on the token GEMM)
        T = x.numel() // max(1, x.shape[-1])
        tok = sink is None and _dgrad_on_token_gemm(T, weight, x.dtype)
        ctx.wt = _WT.request(weight) if tok else None
        # x = act(pre) of an MLP: the activation backward rides in the dX GEMM (ops.ActBackwardSink)
        ctx.gs = (gelu_sink if tok and gelu_sink is not None and gelu_sink.pre is not None
                  and gelu_sink.pre.shape == x.shape and gelu_sink.pre.dtype == x.dtype else None)
        return _forward_gemm(x, weight, bias)

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        gy2 = gy.reshape(-1, gy.shape[-1])
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gres = ctx.sink.take() if ctx.sink is not None else None
            if gres is not None:       # the residual path's gradient of x, added by the GEMM (beta = 1)
                gx = _addmm_into(gres.reshape(gy2.shape[0], -1), gy2, weight.to(gy2.dtype)).view(x.shape)
            elif ctx.gs is not None and _dgrad_on_token_gemm(gy2.shape[0], weight, gy2.dtype):
                act = {"gelu_pre" if ctx.gs.kind == "gelu" else "relu_out": ctx.gs.pre}
                gx = ops.token_gemm(gy2.contiguous(), _WT.get(ctx.wt), **act).view(x.shape)
                ctx.gs.done = True
            else:
                gx = _dgrad_gemm(gy2, weight, ctx.wt).view(x.shape)
        ctx.wt = ctx.gs = None
        want_b = ctx.has_bias and ctx.needs_input_grad[2]
        cs = ops.take_colsum(gy) if want_b else None               # from the LayerNorm backward's pass
        if cs is not None:
            gb = cs.to(weight.dtype)
        if ctx.needs_input_grad[1]:
            x2 = x.reshape(-1, x.shape[-1]).to(gy2.dtype)
            if want_b and gb is None and _token_wgrad_ok(gy2, x2, weight.dtype):
                gw, gb = weight_grad(gy2, x2, weight.dtype, bias=True)
            else:
                gw = weight_grad(gy2, x2, weight.dtype)
        if want_b and gb is None:
            if gy2.shape[1] % 8 == 0 and gy2.shape[1] <= ops.COLSUM_MAX_N:
                gb = ops.column_sum(gy2).to(weight.dtype)          # HIP column sum, f32 accumulation
            else:
                gb = gy2.sum(0, dtype=torch.float32).to(weight.dtype)
        return gx, gw, gb, None, None


class _PlaneProjectionFn(torch.autograd.Function):
    """1x1 convolution from NCHW planes to token-major output: out[b, p, o] = sum_i
    W[o, i] y[b, i, p] + bias[o].  Both GEMMs read y in place (its [C, HW] planes are a
    column-major [HW, C] operand), so neither direction needs a layout copy."""

    @staticmethod
    def forward(ctx, y, weight, bias):
        B, Ci, H, W = y.shape
        Co = weight.shape[0]
        y3 = y.contiguous().view(B, Ci, H * W)
        w2 = weight.view(Co, Ci)
        wt = w2.t().unsqueeze(0).expand(B, Ci, Co)
        if bias is not None:
            out = torch.baddbmm(bias.view(1, 1, Co).expand(B, H * W, Co), y3.transpose(1, 2), wt)
        else:
            out = torch.bmm(y3.transpose(1, 2), wt)
        ctx.save_for_backward(y3, weight)
        ctx.has_bias = bias is not None
        ctx.hw = (H, W)
        return out

    @staticmethod
    def backward(ctx, gp):
        y3, weight = ctx.saved_tensors
        B, Ci, HW = y3.shape
        Co = weight.shape[0]
        H, W = ctx.hw
        gp = gp.contiguous()
        w2 = weight.view(Co, Ci).to(gp.dtype)
        gy = gw = gb = None
        if ctx.needs_input_grad[0]:
            gy = torch.bmm(w2.t().unsqueeze(0).expand(B, Ci, Co), gp.transpose(1, 2)).view(B, Ci, H, W)
        if ctx.needs_input_grad[1]:
            gw = _plane_weight_grad(gp, y3.to(gp.dtype), weight.dtype).view_as(weight)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            g2 = gp.view(-1, Co)
            gb = (ops.column_sum(g2) if Co % 8 == 0 and Co <= ops.COLSUM_MAX_N else g2.sum(0, dtype=torch.float32))
            gb = gb.to(weight.dtype)
        return gy, gw, gb


def _plane_weight_grad(gp, y3, out_dtype):
    """dW[o, i] = sum_b gp[b]^T y[b]^T with K = HW per image: each image's pixel axis is
    cut into chunks run as one f32 batched GEMM (y's chunk is a column-major operand
    in place), all partials summed once by the split-K epilogue."""
    B, HW, Co = gp.shape
    Ci = y3.shape[1]
    per = max(1, split_count(B * HW, Co, Ci) // B)
    while per > 1 and HW % per:
        per -= 1
    if per <= 1 or (Co * Ci) % 4 or out_dtype not in (torch.float32, torch.bfloat16):
        return torch.einsum("bpo,bip->oi", gp.float(), y3.float()).to(out_dtype)
    c = HW // per
    parts = [torch.bmm(gp[b].view(per, c, Co).transpose(1, 2), y3[b].view(Ci, per, c).permute(1, 2, 0),
                       out_dtype=torch.float32) for b in range(B)]
    part = torch.cat(parts, 0)
    out = torch.empty(Co, Ci, device=gp.device, dtype=out_dtype)
    L.check(L.lib().vs_splitk_sum(L.dtype_code(out), L.ptr(part), B * per, Co * Ci, None, L.ptr(out),
                                  L.stream(out)), "splitk_sum")
    return out


class _TokenPlaneFn(torch.autograd.Function):
    """1x1 convolution from token-major input to NCHW planes: out[b, o, p] = sum_i W[o, i]
    x[b, p, i] + bias[o] (the pixel decoder's lateral conv on the stage-1 Swin feature,
    HF:m2f:1394-1405).  x^T is read in place as a column-major operand, so the NCHW copy of
    the [B, 96, 256, 256] feature that nn.Conv2d needed (~0.1 ms at C2) is gone; backward:
    dX = dY^T W (dY's planes column-major in place), dW = sum_b dY_b X_b, db = sum dY."""

    @staticmethod
    def forward(ctx, x, weight, bias, H, W):
        B, HW, Ci = x.shape
        Co = weight.shape[0]
        w2 = weight.view(Co, Ci).unsqueeze(0).expand(B, Co, Ci)
        xt = x.transpose(1, 2)                                           # [B, Ci, HW] column-major view
        if bias is not None:
            out = torch.baddbmm(bias.view(1, Co, 1).expand(B, Co, HW), w2, xt)
        else:
            out = torch.bmm(w2, xt)
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return out.view(B, Co, H, W)

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        B, HW, Ci = x.shape
        Co = weight.shape[0]
        g3 = gy.contiguous().view(B, Co, HW).to(x.dtype)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.bmm(g3.transpose(1, 2), weight.view(Co, Ci).to(x.dtype).unsqueeze(0).expand(B, Co, Ci))
        if ctx.needs_input_grad[1]:
            # per-image products in f32 (bmm's f32 output), summed over the batch and rounded
            # once -- a bf16 product per image rounded each image's dW first (round-5 ADVICE)
            gw = (torch.bmm(g3, x, out_dtype=torch.float32) if x.dtype != torch.float32 else torch.bmm(g3, x))
            gw = gw.sum(0).to(weight.dtype).view_as(weight)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = g3.sum((0, 2), dtype=torch.float32).to(weight.dtype)
        return gx, gw, gb, None, None


def token_plane_projection(x, weight, bias, H, W):
    """nn.Conv2d(k=1) of a token-major [B, H*W, Ci] tensor -> NCHW [B, Co, H, W] (see
    _TokenPlaneFn)."""
    return _TokenPlaneFn.apply(x, weight, bias, H, W)


def plane_projection(y, weight, bias=None):
    """nn.Conv2d(k=1) of an NCHW tensor returned as a channels-last NCHW view (memory
    [B, H, W, Co]): the mask projection whose output the mask head reads token-major."""
    B, _, H, W = y.shape
    if torch.is_autocast_enabled():
        dt = torch.get_autocast_dtype("cuda")
        with torch.autocast("cuda", enabled=False):
            out = _PlaneProjectionFn.apply(y.to(dt), weight.to(dt), None if bias is None else bias.to(dt))
    else:
        out = _PlaneProjectionFn.apply(y, weight, bias)
    return out.view(B, H, W, -1).permute(0, 3, 1, 2)


SMALL_MAX_TOKENS = 4096
_SMALL = os.environ.get("VS_SMALL_LINEAR", "1") == "1"      # A/B switch


_SMALL_FUSED = os.environ.get("VS_SMALL_LINEAR_FUSED", "1") == "1"   # A/B: library forward / dX GEMMs
_QKV_FUSED = os.environ.get("VS_SELF_ATTN_FUSED", "1") == "1"      # A/B: add + three small Linears


def _pos_rows(pos, T):
    """(contiguous pos rows, rows): the query-position table itself when pos is its batch
    expand (stride 0 over the batch), else the per-token rows."""
    if pos.dim() == 3 and pos.stride(0) == 0 and pos[0].is_contiguous():
        return pos[0], pos.shape[1]
    return pos.reshape(T, -1).contiguous(), T


def _pos_grad_buffer(psink, T, D, like):
    """(buffer, accumulate) for a consumer's position-row gradient: a fresh [T, D] buffer,
    or -- with a GradSink (ops.GradSink: every consumer of one position table sums into
    one buffer, the source node hands the sum to autograd once) -- the sink's buffer,
    created by the first consumer and accumulated into by the rest."""
    if psink is None:
        return torch.empty(T, D, device=like.device, dtype=torch.bfloat16), False
    if psink.buf is None:
        psink.buf = torch.empty(T, D, device=like.device, dtype=torch.bfloat16)
        return psink.buf, False
    return psink.buf, True


class _SmallLinearFn(torch.autograd.Function):
    """Linear over a few hundred tokens on csrc/small_linear.hip: the forward one launch
    (Y = act((X [+ pos]) W^T + b), vs_small_linear_forward) and the whole backward one
    launch (dX = dY' W and the token-split dW / db in one grid, dY' = dY masked by the
    ReLU output when relu, vs_small_linear_backward) -- autograd ran an add, an addmm, a
    relu forward, and threshold_backward + mm + a single-tile dW GEMM + a bias reduction
    backward.  pos (optional, e.g. the query-position table expanded over the batch) gets
    the same gradient as X.  VS_SMALL_LINEAR_FUSED=0: library forward / dX GEMMs, dW and db
    by vs_small_linear_wgrad."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu=False, pos=None, sink=None, psink=None):
        ctx.has_bias = bias is not None
        ctx.relu = bool(relu)
        ctx.sink = ctx.psink = None
        if not _SMALL_FUSED:
            ctx.prows = 0
            xin = x if pos is None else x + pos
            y = F.linear(xin, weight, bias)
            y = F.relu(y) if relu else y
            ctx.save_for_backward(xin, weight, y if relu else None, None)
            return y
        O, I = weight.shape
        x2 = x.reshape(-1, I).contiguous()
        T = x2.shape[0]
        p2, prows = _pos_rows(pos, T) if pos is not None else (None, 0)
        ctx.prows, ctx.pos_shape = prows, (pos.shape if pos is not None else None)
        y = torch.empty(T, O, device=x.device, dtype=torch.bfloat16)
        L.check(L.lib().vs_small_linear_forward(L.dtype_code(y), L.ptr(x2), L.ptr(p2) if p2 is not None else None,
                                                prows, L.ptr(weight.contiguous()),
                                                L.ptr(bias) if bias is not None else None, int(relu), L.ptr(y),
                                                T, O, I, L.stream(x2)), "small_linear_forward")
        ctx.save_for_backward(x2, weight, y if relu else None, p2)
        ctx.sink, ctx.psink = sink, (psink if pos is not None else None)
        if sink is not None:
            sink.arm()
        return y.view(*x.shape[:-1], O)

    @staticmethod
    def backward(ctx, gy):
        x, weight, y, p2 = ctx.saved_tensors
        O, I = weight.shape
        gy2 = gy.reshape(-1, O).contiguous()
        gx = gw = gb = gpos = None
        want_w = ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2])
        want_pos = len(ctx.needs_input_grad) > 4 and ctx.needs_input_grad[4]
        x2 = x.reshape(-1, I).contiguous()
        if want_w:
            gw = torch.empty(O, I, device=gy2.device, dtype=torch.bfloat16)
            gb = torch.empty(O, device=gy2.device, dtype=torch.bfloat16) if ctx.has_bias else None
        if _SMALL_FUSED:
            T = gy2.shape[0]
            gres = ctx.sink.take() if ctx.sink is not None else None
            if gres is not None:
                gres = gres.reshape(T, I).contiguous()
            if ctx.needs_input_grad[0] or want_pos:
                gx = torch.empty(T, I, device=gy2.device, dtype=torch.bfloat16)
            acc = False
            if want_pos:
                gpos, acc = _pos_grad_buffer(ctx.psink, T, I, gy2)
            if gx is not None or gw is not None:
                L.check(L.lib().vs_small_linear_backward(
                    L.dtype_code(gy2), L.ptr(gy2), L.ptr(x2), L.ptr(p2) if p2 is not None else None, ctx.prows,
                    L.ptr(weight.contiguous()), L.ptr(y) if y is not None else None,
                    L.ptr(gres) if gres is not None else None, L.ptr(gx) if gx is not None else None,
                    L.ptr(gpos) if gpos is not None else None, int(acc),
                    L.ptr(gw) if gw is not None else None, L.ptr(gb) if gb is not None else None,
                    T, O, I, L.stream(gy2)), "small_linear_backward")
            if gx is not None:
                gx = gx.view(*gy.shape[:-1], I) if ctx.needs_input_grad[0] else None
            if gpos is not None:
                gpos = None if ctx.psink is not None else gpos.view(*gy.shape[:-1], I)
        else:
            if y is not None:
                gy2 = gy2 * (y.reshape(-1, O) > 0).to(gy2.dtype)
            if ctx.needs_input_grad[0] or want_pos:
                gx = (gy2 @ weight).view(*gy.shape[:-1], I)
                gpos = gx if want_pos else None
                gx = gx if ctx.needs_input_grad[0] else None
            if want_w:
                L.check(L.lib().vs_small_linear_wgrad(L.dtype_code(gw), L.ptr(gy2), L.ptr(x2), L.ptr(gw),
                                                      L.ptr(gb) if gb is not None else None, gy2.shape[0], O, I,
                                                      L.stream(gy2)), "small_linear_wgrad")
        if not ctx.needs_input_grad[1]:
            gw = None
        if not (ctx.has_bias and ctx.needs_input_grad[2]):
            gb = None
        return gx, gw, gb, None, gpos, None, None


class _InProjFn(torch.autograd.Function):
    """The cross-attention input projections of one decoder layer, q = xq W_q^T + b_q,
    k = xk W_k^T + b_k, v = xv W_v^T + b_v, with W = [W_q; W_k; W_v] and b one parameter
    each (nn.MultiheadAttention's in_proj_weight / in_proj_bias; HF:m2f:1644-1650).  The
    backward writes the three row blocks of dW and db straight into one [3D, D] / [3D]
    gradient each -- slicing the parameters in the forward made autograd zero-fill a
    full-size gradient per slice and add the three (2 fills + 2 adds per parameter and
    layer).  q: a few hundred tokens (dW, db by the one-launch small wgrad kernel); k, v:
    the level memory (split-K dW, HIP column sums)."""

    @staticmethod
    def forward(ctx, xq, xk, xv, weight, bias, q_pos=None, sink=None, psink=None, kv_sink=None):
        D = weight.shape[1]
        # kv_sink (ops.GradSink of the level memory m, with xk = m + pos and xv = m): dxk and
        # dxv are summed into the sink's buffer by the dX GEMMs themselves (beta = 1), over
        # every layer that reads this level -- no add of the two, no add across layers
        ctx.kv_sink = kv_sink
        W = (weight[:D], weight[D:2 * D], weight[2 * D:])
        B = (bias[:D], bias[D:2 * D], bias[2 * D:])
        T = xq.numel() // D
        # the query rows on the small-token kernels (one launch each way, q_pos in the
        # operand loads): bf16, a few hundred tokens
        ctx.small = bool(_SMALL and _SMALL_FUSED and xq.dtype == weight.dtype == torch.bfloat16
                         and T <= SMALL_MAX_TOKENS and D % 64 == 0)
        ctx.prows = 0
        ctx.sink = ctx.psink = None
        if ctx.small:
            ctx.sink, ctx.psink = sink, (psink if q_pos is not None else None)
            if sink is not None:
                sink.arm()
            x2 = xq.reshape(-1, D).contiguous()
            p2, ctx.prows = _pos_rows(q_pos, T) if q_pos is not None else (None, 0)
            q = torch.empty(T, D, device=xq.device, dtype=torch.bfloat16)
            L.check(L.lib().vs_small_linear_forward(L.dtype_code(q), L.ptr(x2),
                                                    L.ptr(p2) if p2 is not None else None, ctx.prows,
                                                    L.ptr(W[0]), L.ptr(B[0]), 0, L.ptr(q), T, D, D,
                                                    L.stream(x2)), "small_linear_forward")
            q = q.view(xq.shape)
            ctx.save_for_backward(x2, xk, xv, weight, p2)
        else:
            xq_ = xq if q_pos is None else xq + q_pos
            q = F.linear(xq_, W[0], B[0])
            ctx.save_for_backward(xq_, xk, xv, weight, None)
        return (q,) + tuple(F.linear(x, w, b) for x, w, b in zip((xk, xv), W[1:], B[1:]))

    @staticmethod
    def backward(ctx, gq, gk, gv):
        xq, xk, xv, weight, p2 = ctx.saved_tensors
        D = weight.shape[1]
        gw = torch.empty_like(weight)
        gb = torch.empty(3 * D, device=weight.device, dtype=weight.dtype)
        gx = []
        gpos = None
        want_pos = len(ctx.needs_input_grad) > 5 and ctx.needs_input_grad[5]
        for i, (g, x) in enumerate(((gq, xq), (gk, xk), (gv, xv))):
            g2 = g.reshape(-1, D).contiguous()
            x2 = x.reshape(-1, D).contiguous()
            w_i = weight[i * D:(i + 1) * D]
            rows = slice(i * D, (i + 1) * D)
            if i == 0 and ctx.small:
                T = g2.shape[0]
                need_x = ctx.needs_input_grad[0] or want_pos
                gxq = torch.empty(T, D, device=g2.device, dtype=torch.bfloat16) if need_x else None
                gpos, acc = _pos_grad_buffer(ctx.psink, T, D, g2) if want_pos else (None, False)
                gres = ctx.sink.take() if ctx.sink is not None else None
                if gres is not None:
                    gres = gres.reshape(T, D).contiguous()
                L.check(L.lib().vs_small_linear_backward(
                    L.dtype_code(g2), L.ptr(g2), L.ptr(x2), L.ptr(p2) if p2 is not None else None, ctx.prows,
                    L.ptr(w_i), None, L.ptr(gres) if gres is not None else None,
                    L.ptr(gxq) if gxq is not None else None, L.ptr(gpos) if gpos is not None else None, int(acc),
                    L.ptr(gw[rows]), L.ptr(gb[rows]), T, D, D, L.stream(g2)), "small_linear_backward")
                gx.append(gxq.view(gq.shape) if ctx.needs_input_grad[0] else None)
                gpos = gpos.view(gq.shape) if (gpos is not None and ctx.psink is None) else None
                continue
            if i > 0 and ctx.kv_sink is not None:
                ks = ctx.kv_sink
                if ks.buf is None:
                    ks.buf = g2 @ w_i
                else:
                    ks.buf.addmm_(g2, w_i)
                gx.append(None)
            else:
                gxi = (g2 @ w_i).view(x.shape) if (ctx.needs_input_grad[i] or (i == 0 and want_pos)) else None
                if i == 0 and want_pos:
                    gpos = gxi
                gx.append(gxi if ctx.needs_input_grad[i] else None)
            x2 = x2.to(g2.dtype)
            if _token_wgrad_ok(g2, x2, weight.dtype) and weight.dtype == g2.dtype:
                weight_grad(g2, x2, weight.dtype, out=gw[rows], bias=True, bias_out=gb[rows])
                continue
            weight_grad(g2, x2, weight.dtype, out=gw[rows])
            if D % 8 == 0 and D <= 2048 and g2.dtype == weight.dtype:
                ops.column_sum(g2, out=gb[rows])
            else:
                gb[rows].copy_(g2.sum(0, dtype=torch.float32))
        return gx[0], gx[1], gx[2], gw, gb, gpos, None, None, None


def in_projection(xq, xk, xv, weight, bias, q_pos=None, sink=None, psink=None, kv_sink=None):
    """(q, k, v) of nn.MultiheadAttention's packed in-projection (see _InProjFn), the query
    input being xq + q_pos when q_pos is given (HF:m2f with_pos_embed); plain slicing off
    the device / under autocast / without grad."""
    D = weight.shape[1]
    if (xq.is_cuda and torch.is_grad_enabled() and weight.requires_grad and not torch.is_autocast_enabled()
            and xq.dtype == weight.dtype == xk.dtype == xv.dtype == bias.dtype
            and (q_pos is None or (q_pos.shape == xq.shape and q_pos.dtype == xq.dtype))):
        return _InProjFn.apply(xq, xk, xv, weight, bias, q_pos, sink, psink, kv_sink)
    if q_pos is not None:
        xq = xq + q_pos
    return (F.linear(xq, weight[:D], bias[:D]), F.linear(xk, weight[D:2 * D], bias[D:2 * D]),
            F.linear(xv, weight[2 * D:], bias[2 * D:]))


class _ValueQueryProjFn(torch.autograd.Function):
    """An encoder MSDeformAttn layer's two input projections of the same tokens h
    (HF:m2f:919-1002): value = h Wv^T + bv and proj = (h + pos) Wp^T + bp (the fused
    sampling-offset / attention-weight projection).

    Backward: dh = [g_res] + dproj Wp + dvalue Wv as chained GEMMs with beta = 1 (g_res:
    the post-norm residual gradient of h handed over by ResidualSink), so autograd adds
    nothing at full size.  With `level_embed` (pos = a constant sine embedding + level
    embedding rows, the level sizes in `level_sizes`), pos gets no gradient: the level
    embedding's is (per-level column sums of dproj) Wp, exact by linearity, and the bias
    gradient of proj is the sum of the same per-level sums.  Weight gradients: split-K."""

    @staticmethod
    def forward(ctx, h, pos, wv, bv, wp, bp, level_embed=None, level_sizes=None, sink=None):
        q = h + pos
        ctx.save_for_backward(h, q, wv, wp)
        ctx.level = (level_embed is not None, tuple(level_sizes or ()),
                     level_embed.dtype if level_embed is not None else None)
        ctx.sink = sink
        if sink is not None:
            sink.arm()
        # proj (256 -> 288 at the C2 encoder) on the token GEMM by the forward rule: 36.9 vs 44.3
        # us per call; value (256 -> 256) ties (29.8 vs 28.9 us) and stays on the vendor GEMM
        # (tools/r6/enc_gemm_bench.py, profiles/r6_enc_gemm_bench.txt)
        return F.linear(h, wv, bv), _forward_gemm(q, wp, bp)

    @staticmethod
    def backward(ctx, gv, gp):
        h, q, wv, wp = ctx.saved_tensors
        Dh = h.shape[-1]
        has_level, sizes, ldt = ctx.level
        gv2 = gv.reshape(-1, gv.shape[-1]).contiguous()
        gp2 = gp.reshape(-1, gp.shape[-1]).contiguous()
        gres = ctx.sink.take() if ctx.sink is not None else None
        dq = None
        wp_, wv_ = wp.to(gp2.dtype), wv.to(gv2.dtype)
        if ctx.needs_input_grad[1]:                                   # d pos wanted on its own
            dq = gp2 @ wp_
            dh = torch.addmm(dq, gv2, wv_)
            if gres is not None:
                dh = dh + gres.reshape(dh.shape)
        else:
            dh = gp2 @ wp_ if gres is None else _addmm_into(gres.reshape(gp2.shape[0], Dh), gp2, wp_)
            dh.addmm_(gv2, wv_)                                       # + value's share, in the GEMM epilogue
        h2, q2 = h.reshape(-1, Dh), q.reshape(-1, Dh)
        gwv, gbv = weight_grad(gv2, h2.to(gv2.dtype), wv.dtype, bias=True)
        gwp = weight_grad(gp2, q2.to(gp2.dtype), wp.dtype)

        def bias_grad(g2, dt):
            if g2.shape[1] % 8 == 0 and g2.shape[1] <= ops.COLSUM_MAX_N:
                return ops.column_sum(g2).to(dt)
            return g2.sum(0, dtype=torch.float32).to(dt)

        glvl = None
        if has_level and gp2.shape[1] % 8 == 0 and gp2.shape[1] <= 2048:
            seg = ops.column_sum_segments(gp2.view(-1, sum(sizes), gp2.shape[1]), sizes)   # [levels, Np] f32
            gbp = seg.sum(0).to(wp.dtype)
            if ctx.needs_input_grad[6]:
                glvl = (seg @ wp.float()).to(ldt)
        else:
            gbp = bias_grad(gp2, wp.dtype)
            if has_level and ctx.needs_input_grad[6]:
                g3 = gp2.view(-1, sum(sizes), gp2.shape[1]).float()
                glvl = torch.stack([c.sum((0, 1)) for c in torch.split(g3, list(sizes), 1)]) @ wp.float()
                glvl = glvl.to(ldt)
        return (dh.view(h.shape), dq.view(h.shape) if dq is not None else None, gwv,
                gbv, gwp, gbp, glvl, None, None)


def value_query_projection(h, pos, wv, bv, wp, bp, level_embed=None, level_sizes=None, sink=None):
    """(h Wv^T + bv, (h + pos) Wp^T + bp) with the fused backward of _ValueQueryProjFn on
    token-heavy device tensors; the plain composition otherwise.  `level_embed` /
    `level_sizes`: pos already holds the level-embedding rows (detached) and the
    gradient goes to `level_embed` directly; `sink`: see ops.ResidualSink."""
    tokens = h.numel() // max(1, h.shape[-1])
    if (h.is_cuda and torch.is_grad_enabled() and wv.requires_grad and tokens >= MIN_TOKENS
            and not torch.is_autocast_enabled() and h.dtype == pos.dtype == wv.dtype == wp.dtype):
        return _ValueQueryProjFn.apply(h, pos, wv, bv, wp, bp, level_embed, level_sizes, sink)
    pos = reattach_level_embed(pos, level_embed, level_sizes)
    return linear_tokens(h, wv, bv), linear_tokens(h + pos, wp, bp)


def reattach_level_embed(pos, level_embed, sizes):
    """pos (holding detached level-embedding rows) with the level embedding's gradient
    path restored for the plain composition: pos + (rows - rows.detach()), exactly pos in
    value."""
    if level_embed is None or not (torch.is_grad_enabled() and level_embed.requires_grad):
        return pos
    rows = torch.cat([level_embed[i].view(1, 1, -1).expand(pos.shape[0], n, -1) for i, n in enumerate(sizes)], 1)
    rows = rows.to(pos.dtype)
    return pos + (rows - rows.detach())


def small_linear(x, w, b=None, relu=False, sink=None):
    """F.linear (+ ReLU when relu) on the small-token HIP kernels for bf16 device tokens
    (see _SmallLinearFn; sink: ops.ResidualSink, x's residual-path gradient added
    in-kernel); the plain composition otherwise."""
    tokens = x.numel() // max(1, x.shape[-1])
    O, I = w.shape
    if (_SMALL and x.is_cuda and torch.is_grad_enabled() and w.requires_grad and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and (b is None or b.dtype == torch.bfloat16)
            and tokens <= SMALL_MAX_TOKENS and O % 64 == 0 and I % 64 == 0 and not torch.is_autocast_enabled()):
        return _SmallLinearFn.apply(x, w, b, relu, None, sink)
    y = F.linear(x, w, b)
    return F.relu(y) if relu else y


def _ptrs3(ts):
    return (ctypes.c_void_p * 3)(*[L.ptr(t) for t in ts])


class _SelfAttnInProjFn(torch.autograd.Function):
    """q = (h + pos) Wq^T + bq, k = (h + pos) Wk^T + bk, v = h Wv^T + bv over the decoder's
    B x Q tokens (HF:m2f:1730-1745 with_pos_embed, Mask2FormerAttention q/k/v_proj) as one
    forward and one backward launch (csrc/small_linear.hip vs_self_attn_in_proj_*): the
    backward sums every use of h and of pos in-kernel (dpos = dq Wq + dk Wk, dh = dpos +
    dv Wv), where autograd ran an add, three Linear backwards and three gradient adds."""

    @staticmethod
    def forward(ctx, h, pos, wq, bq, wk, bk, wv, bv, sink=None, psink=None):
        B, Q, D = h.shape
        h2 = h.reshape(-1, D).contiguous()
        if pos.stride(0) == 0 and pos[0].is_contiguous():     # query_embed expanded over the batch
            p2, prows = pos[0], Q
        else:
            p2, prows = pos.reshape(-1, D).contiguous(), B * Q
        ws = [w.contiguous() for w in (wq, wk, wv)]
        outs = [torch.empty(h2.shape[0], D, device=h.device, dtype=torch.bfloat16) for _ in range(3)]
        L.check(L.lib().vs_self_attn_in_proj_forward(L.dtype_code(h2), L.ptr(h2), L.ptr(p2), prows, _ptrs3(ws),
                                                     _ptrs3([bq, bk, bv]), _ptrs3(outs), h2.shape[0], D,
                                                     L.stream(h2)), "self_attn_in_proj_forward")
        ctx.save_for_backward(h2, p2, *ws)
        ctx.shape, ctx.prows = h.shape, prows
        ctx.sink, ctx.psink = sink, psink
        if sink is not None:
            sink.arm()
        return tuple(o.view(B, Q, D) for o in outs)

    @staticmethod
    def backward(ctx, gq, gk, gv):
        h2, p2, wq, wk, wv = ctx.saved_tensors
        D = h2.shape[1]
        gs = [(g if g is not None else torch.zeros(ctx.shape, device=h2.device, dtype=torch.bfloat16))
              .reshape(-1, D).contiguous() for g in (gq, gk, gv)]
        T = h2.shape[0]
        gh = torch.empty_like(h2)
        gres = ctx.sink.take() if ctx.sink is not None else None
        if gres is not None:
            gres = gres.reshape(T, D).contiguous()
        gp, acc = _pos_grad_buffer(ctx.psink, T, D, h2) if ctx.needs_input_grad[1] else (None, False)
        gw = [torch.empty(D, D, device=h2.device, dtype=torch.bfloat16) for _ in range(3)]
        gb = [torch.empty(D, device=h2.device, dtype=torch.bfloat16) for _ in range(3)]
        L.check(L.lib().vs_self_attn_in_proj_backward(
            L.dtype_code(h2), L.ptr(h2), L.ptr(p2), ctx.prows, _ptrs3([wq, wk, wv]), _ptrs3(gs),
            L.ptr(gres) if gres is not None else None, L.ptr(gh), L.ptr(gp) if gp is not None else None, int(acc),
            _ptrs3(gw), _ptrs3(gb), T, D, L.stream(h2)), "self_attn_in_proj_backward")
        if ctx.psink is not None:
            gp = None
        return (gh.view(ctx.shape), gp.view(ctx.shape) if gp is not None else None,
                gw[0], gb[0], gw[1], gb[1], gw[2], gb[2], None, None)


def self_attn_in_proj(h, pos, q_proj, k_proj, v_proj, sink=None, psink=None):
    """(q, k, v) of the decoder self-attention: q = q_proj(h + pos), k = k_proj(h + pos),
    v = v_proj(h), each [B, Q, D] -- one launch each way on the bf16 device path (see
    _SelfAttnInProjFn), the plain composition otherwise.  sink: ops.ResidualSink (h's
    residual-path gradient added in-kernel); psink: ops.GradSink of pos (see
    _pos_grad_buffer)."""
    D = h.shape[-1]
    lins = (q_proj, k_proj, v_proj)
    tokens = h.numel() // max(1, D)
    if (_SMALL and _SMALL_FUSED and _QKV_FUSED and h.is_cuda and torch.is_grad_enabled() and h.dim() == 3
            and pos.shape == h.shape and not torch.is_autocast_enabled() and D % 64 == 0
            and tokens <= SMALL_MAX_TOKENS and h.dtype == pos.dtype == torch.bfloat16
            and all(m.weight.shape == (D, D) and m.bias is not None and m.weight.requires_grad
                    and m.weight.dtype == m.bias.dtype == torch.bfloat16 for m in lins)):
        return _SelfAttnInProjFn.apply(h, pos, q_proj.weight, q_proj.bias, k_proj.weight, k_proj.bias,
                                       v_proj.weight, v_proj.bias, sink, psink)
    hq = h + pos
    return q_proj(hq), k_proj(hq), v_proj(h)


class SmallLinear(nn.Linear):
    """nn.Linear for the decoder's B x Q tokens (see small_linear)."""

    def forward(self, x):
        return small_linear(x, self.weight, self.bias)


def _autocast_dtype(t):
    return torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled() else t.dtype


class TokenLayerNorm(nn.LayerNorm):
    """nn.LayerNorm on the HIP row kernel (csrc/norm.hip) for f32 / bf16 device tensors
    whose weight shares their dtype; anything else (autocast's f32 LayerNorm, CPU
    tensors, rows > 2048) is torch's own layer_norm."""

    def forward(self, x):
        if self.elementwise_affine and self.bias is not None and ops.layer_norm_supported(x, self.weight) \
                and not torch.is_autocast_enabled():
            return ops.layer_norm(x, self.weight, self.bias, self.eps)
        return F.layer_norm(x, self.normalized_shape, self.weight, self.bias, self.eps)

    def forward_windows(self, x, wrows, quant: bool = False):
        """LN(x) in the window layout of wrows (ops.WindowRows: the Swin partition folded
        into the kernel's stores) -> [wrows.total, C]; quant (bf16, C % 32 == 0): -> (y,
        (e4m3, e8m0 scales) of y) for an fp8 consumer, (y, None) where the copy cannot be made."""
        if self.elementwise_affine and self.bias is not None and ops.layer_norm_supported(x, self.weight) \
                and not torch.is_autocast_enabled():
            if quant and x.dtype == torch.bfloat16 and x.shape[-1] % (8 if quant == "rows" else 32) == 0:
                y, yq, ys = ops.layer_norm(x, self.weight, self.bias, self.eps, wrows=wrows,
                                           quant="rows" if quant == "rows" else True)
                return y, (yq, ys)
            y = ops.layer_norm(x, self.weight, self.bias, self.eps, wrows=wrows)
            return (y, None) if quant else y
        y = self(x)
        y = ops._to_windows(y.to(_autocast_dtype(y)), wrows)
        return (y, None) if quant else y

    def add_forward_windows(self, x, r, wrows, sink=None, quant: bool = False):
        """(x + r, LN(x + r) in the window layout of wrows) (+ the MX fp8 copy, see
        forward_windows)."""
        if self.elementwise_affine and self.bias is not None and ops.layer_norm_supported(x, self.weight) \
                and r.shape == x.shape and r.dtype == x.dtype and not torch.is_autocast_enabled():
            if quant and x.dtype == torch.bfloat16 and x.shape[-1] % (8 if quant == "rows" else 32) == 0:
                s, y, yq, ys = ops.add_layer_norm(x, r, self.weight, self.bias, self.eps, sink, wrows=wrows,
                                                  quant="rows" if quant == "rows" else True)
                return s, y, (yq, ys)
            s, y = ops.add_layer_norm(x, r, self.weight, self.bias, self.eps, sink, wrows=wrows)
            return (s, y, None) if quant else (s, y)
        s, y = self.add_forward(x, r, sink)
        y = ops._to_windows(y.to(_autocast_dtype(y)), wrows)
        return (s, y, None) if quant else (s, y)

    def add_forward(self, x, r, sink=None, quant: bool = False):
        """(x + r, LN(x + r)): the residual add fused into the norm on the HIP kernel
        (ops.add_layer_norm) where the plain norm would run there too.  `sink`: hand x's
        gradient to the armed consumer of x (ops.ResidualSink); `quant`: + the MX fp8 copy of
        LN(x + r) (see forward_windows)."""
        if self.elementwise_affine and self.bias is not None and ops.layer_norm_supported(x, self.weight) \
                and r.shape == x.shape and r.dtype == x.dtype and not torch.is_autocast_enabled():
            if quant == "rows" and x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0:
                s, y, yq, ys = ops.add_layer_norm(x, r, self.weight, self.bias, self.eps, sink, quant="rows")
                return s, y, (yq, ys)                  # [rows, C] e4m3, [rows, 1] f32
            if quant and x.dtype == torch.bfloat16 and x.shape[-1] % 32 == 0:
                s, y, yq, ys = ops.add_layer_norm(x, r, self.weight, self.bias, self.eps, sink, quant=True)
                return s, y, (yq.view(y.shape), ys.view(*y.shape[:-1], -1))
            s, y = ops.add_layer_norm(x, r, self.weight, self.bias, self.eps, sink)
            return (s, y, None) if quant else (s, y)
        s = x + r
        return (s, self(s), None) if quant else (s, self(s))


def linear_tokens(x, w, b=None, sink=None, gelu_sink=None):
    """F.linear with the split-K weight gradient when x carries many tokens (`sink`: see
    ops.ResidualSink; armed only on that path; `gelu_sink`: ops.ActBackwardSink when x is
    the GELU / ReLU output of an MLP feeding only this Linear)."""
    tokens = x.numel() // max(1, x.shape[-1])
    if not (x.is_cuda and torch.is_grad_enabled() and w.requires_grad and tokens >= MIN_TOKENS):
        return F.linear(x, w, b)
    if torch.is_autocast_enabled():
        dt = torch.get_autocast_dtype("cuda")
        with torch.autocast("cuda", enabled=False):
            return _LinearFn.apply(x.to(dt), w.to(dt), None if b is None else b.to(dt))
    return _LinearFn.apply(x, w, b, sink, gelu_sink)


class _LinearReluFn(torch.autograd.Function):
    """relu(x W^T + b) with the bias and the ReLU in the GEMM epilogue
    (torch._addmm_activation: hipBLASLt RELU_BIAS), so the pre-activation is never
    written and re-read by a separate ReLU pass (HF:m2f:1080-1082, the encoder FFN).
    Backward: ReLU's derivative from the OUTPUT (y > 0 exactly where x W^T + b > 0), one
    HIP pass for dY * [y > 0] and its column sums (= the bias gradient), then the dX GEMM
    (with the residual sink's gradient, beta = 1) and the split-K weight gradient."""

    @staticmethod
    def forward(ctx, x, weight, bias, sink=None, act_sink=None):
        x2 = x.reshape(-1, x.shape[-1])
        y = torch._addmm_activation(bias, x2, weight.t(), use_gelu=False)
        ctx.save_for_backward(x, weight, y)
        ctx.sink = sink
        if sink is not None:
            sink.arm()
        out = y.view(*x.shape[:-1], weight.shape[0])
        ctx.gs = act_sink if act_sink is not None and act_sink.kind == "relu" else None
        if ctx.gs is not None:            # fc2 reads y's sign in its dX epilogue (ops.ActBackwardSink)
            ctx.gs.pre = out
        return out

    @staticmethod
    def backward(ctx, gy):
        x, weight, y = ctx.saved_tensors
        N = y.shape[-1]
        M = y.shape[0]
        gy2 = gy.reshape(M, N).to(y.dtype).contiguous()
        if ctx.gs is not None and ctx.gs.done:
            # fc2's dX GEMM already applied the ReLU mask: gy IS the pre-activation's gradient
            ctx.gs.done = False
            gp, cs = gy2, None
        else:
            gp = torch.empty_like(y)
            cs = torch.empty(N, device=y.device, dtype=y.dtype)
            ws = torch.empty(int(L.lib().vs_column_sum_workspace_bytes(M, N)), device=y.device, dtype=torch.uint8)
            L.check(L.lib().vs_act_backward_colsum(L.dtype_code(y), 0, L.ptr(gy2), L.ptr(y), L.ptr(gp), L.ptr(cs),
                                                   L.ptr(ws), M, N, L.stream(y)), "act_backward_colsum")
        ctx.gs = None
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gres = ctx.sink.take() if ctx.sink is not None else None
            if gres is not None:
                gx = _addmm_into(gres.reshape(M, -1), gp, weight.to(gp.dtype)).view(x.shape)
            else:
                gx = _dgrad_gemm(gp, weight).view(x.shape)
        x2 = x.reshape(-1, x.shape[-1]).to(gp.dtype)
        if ctx.needs_input_grad[2] and cs is None:
            if ctx.needs_input_grad[1] and _token_wgrad_ok(gp, x2, weight.dtype):
                gw, gb = weight_grad(gp, x2, weight.dtype, bias=True)
            else:
                gb = ops.column_sum(gp).to(weight.dtype)
        elif ctx.needs_input_grad[2]:
            gb = cs.to(weight.dtype)
        if ctx.needs_input_grad[1] and gw is None:
            gw = weight_grad(gp, x2, weight.dtype)
        return gx, gw, gb, None, None


def linear_relu_tokens(x, w, b, sink=None, act_sink=None):
    """relu(F.linear(x, w, b)) -- fused on token-heavy device tensors (see _LinearReluFn);
    the unfused composition otherwise (`sink`: ops.ResidualSink, armed only when fused;
    `act_sink`: ops.ActBackwardSink("relu") when the output feeds only the FFN's fc2)."""
    from . import ops
    tokens = x.numel() // max(1, x.shape[-1])
    N = w.shape[0]
    if (x.is_cuda and torch.is_grad_enabled() and w.requires_grad and b is not None and tokens >= MIN_TOKENS
            and not torch.is_autocast_enabled() and x.dtype == w.dtype == b.dtype
            and x.dtype in (torch.float32, torch.bfloat16) and N % 8 == 0 and N <= ops.COLSUM_MAX_N and x.is_contiguous()):
        return _LinearReluFn.apply(x, w, b, sink, act_sink)
    return ops.activation(linear_tokens(x, w, b, sink), "relu")


class TokenLinear(nn.Linear):
    """nn.Linear whose backward splits the token axis of dW (see module docstring)."""

    def forward(self, x, sink=None):
        return linear_tokens(x, self.weight, self.bias, sink)


# ---------------------------------------------------------------------------------------
# Swin block Linears on the hand-written token GEMM (csrc/token_gemm.hip)
# ---------------------------------------------------------------------------------------
# bf16 fc1 + GELU: the vendor GEMM + the GELU pass (ops.activation) except on the streaming
# kernel (stage 1): the token GEMM's GELU epilogue measured slower than vendor + ATen GELU at
# the C2 shapes (e.g. stage-3 fc1 0.082 vs 0.075 ms, profiles/r4_tgemm_bench3.txt) and is used
# by the fp8 path only
# fp8 Linears only where the product is MFMA-bound: the K-deep ones (C5: stages 2-4 and
# every fc2); the stage-1 qkv / proj / fc1 of Swin-L (K = 192) are HBM-bound
FP8_MIN_K = int(os.environ.get("VS_FP8_MIN_K", "384"))


def fp8_operand_ok(K: int) -> bool:
    """Whether a Linear with K input features takes the MX fp8 path (linear_fp8_tokens):
    the producer of its input then makes the fp8 copy too."""
    return K % 128 == 0 and K >= FP8_MIN_K


def _tgemm_ok(x, w, b, tokens_min=MIN_TOKENS):
    tokens = x.numel() // max(1, x.shape[-1])
    K, N = w.shape[1], w.shape[0]
    return (x.is_cuda and torch.is_grad_enabled() and w.requires_grad and tokens >= tokens_min
            and not torch.is_autocast_enabled() and x.dtype == w.dtype == torch.bfloat16
            and (b is None or b.dtype == torch.bfloat16) and K % 8 == 0 and N % 8 == 0
            and N <= ops.COLSUM_MAX_N and x.is_contiguous())


# config C5 fp8 Linears: the input gradient dX = dY W on the MX fp8 token GEMM too (dY and W^T
# quantised per 32 along the output features) with VS_FP8_DGRAD=1.  Off by default: the C5
# step measured the same with it (131.05 vs 131.01 ms, profiles/r4_bench_c5_fp8_dgrad_ab.jsonl)
# -- the dY quantisation passes cost what the fp8 product saves -- and the bf16 dX carries
# no quantisation error
FP8_DGRAD = os.environ.get("VS_FP8_DGRAD", "0") == "1"


# config C5 fp8 GEMM backend.  "rows" (default): hipBLASLt's fp8 GEMM with one f32 scale per
# row of each operand (torch._scaled_mm rowwise: x per token, W per output feature; e4m3
# rows from ops.row_quantize_fp8).  "mx": the hand-written block-scaled MX token GEMM
# (csrc/token_gemm.hip), which reached 1.0-1.4 PF/s against the vendor kernel's 1.5-2.6
# (tools/r5/scaled_mm_probe.py, profiles/r5_scaled_mm_probe.txt).
FP8_GEMM = os.environ.get("VS_FP8_GEMM", "rows")


def _fp8_rows_ready(x, w, b) -> bool:
    """Operands the rowwise fp8 path takes: contiguous bf16 device tensors outside autocast
    (with or without grad: inference runs the same numerics as training)."""
    return (x.is_cuda and not torch.is_autocast_enabled() and x.dtype == w.dtype == torch.bfloat16
            and (b is None or b.dtype == torch.bfloat16) and x.is_contiguous())


def fp8_rows_ok(M: int, N: int, K: int) -> bool:
    """Static shape rule for the rowwise vendor fp8 GEMM (from the probe at the C5 Swin-L
    shapes, fp8 vs bf16 F.linear): K >= 768 ran 1.5-1.9x faster (qkv / fc1 / fc2 of stages
    3-4, stage-1 fc2); K = 384 pays only for fc1 (N = 4K: 1.3x; qkv 0.9x); K = 192 never
    (0.5x: the product is HBM-bound there)."""
    if (N, K) == (384, 1536):         # Swin-L stage-2 fc2: 0.218 vs 0.193 ms bf16 (measured exception)
        return False
    return M >= MIN_TOKENS and K % 16 == 0 and N % 16 == 0 and (K >= 768 or (K >= 384 and N >= 4 * K))


class _LinearFp8RowFn(torch.autograd.Function):
    """x W^T + b on hipBLASLt's rowwise-scaled fp8 GEMM (config C5): x and W quantised per
    row to e4m3 with power-of-two scales (ops.row_quantize_fp8; x's copy may come from its
    producer, e.g. the fused GELU of the MLP), f32 accumulation, bf16 out, the bias in the
    GEMM epilogue.  Straight-through: the backward is _LinearFn's on the bf16 operands."""

    @staticmethod
    def forward(ctx, x, weight, bias, xq=None, xs=None):
        K = x.shape[-1]
        N = weight.shape[0]
        if xq is None:
            xq, xs = ops.row_quantize_fp8(x.reshape(-1, K))
        wq, ws = ops.row_quantize_fp8(weight)
        with ops.timed("fp8_rows_gemm", x, flops=2.0 * xq.shape[0] * N * K):
            y = torch._scaled_mm(xq, wq.t(), scale_a=xs, scale_b=ws.view(1, N), bias=bias,
                                 out_dtype=torch.bfloat16)
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        ctx.sink = None
        return y.view(*x.shape[:-1], N)

    backward = _LinearFp8Fn_backward = None        # set below (shares _LinearFp8Fn's)


def _dgrad(gy2, weight):
    """dX = dY W for dY [M, N], W [N, K]: MX fp8 (FP8_DGRAD, N % 128 == 0) or the vendor GEMM."""
    N, K = weight.shape
    if FP8_DGRAD and N % 128 == 0 and K % 8 == 0 and gy2.dtype == torch.bfloat16:
        gq, gs = ops.mx_quantize(gy2.contiguous())
        wtq, wts = ops.mx_quantize(weight.t().contiguous())
        return ops.token_gemm(gq, wtq, None, x_scales=gs, w_scales=wts)
    return gy2 @ weight.to(gy2.dtype)


def _mx_pair(x2, weight):
    xq, xs = ops.mx_quantize(x2)
    wq, ws = ops.mx_quantize(weight)
    return xq, xs, wq, ws


class _LinearGeluFn(torch.autograd.Function):
    """gelu(x W^T + b), exact erf GELU (HF `gelu`, the Swin MLP HF:swin:511-536) in the
    token GEMM's epilogue: one kernel stores the pre-activation and the activation (the
    vendor GEMM + ATen GELU wrote the pre-activation, read it back and wrote the
    activation).  fp8: the GEMM on the block-scaled MX MFMA with the operands quantised
    per 32 elements along K (straight-through: the backward sees the bf16 operands).
    Backward: the GELU derivative at the saved pre-activation with the column sums (= the
    bias gradient) in one HIP pass, then the vendor dX GEMM and the split-K dW."""

    @staticmethod
    def forward(ctx, x, weight, bias, fp8=False, quant_out=False, xq=None, xs=None, gelu_sink=None):
        K = x.shape[-1]
        N = weight.shape[0]
        x2 = x.reshape(-1, K)
        q = None
        if fp8:
            if xq is None:
                xq, xs = ops.mx_quantize(x2)
            else:
                xq, xs = xq.reshape(-1, K), xs.reshape(-1, K // 32)
            wq, ws = ops.mx_quantize(weight)
            out = ops.token_gemm(xq, wq, bias, gelu=True, x_scales=xs, w_scales=ws, quant_out=quant_out)
        else:
            out = ops.token_gemm(x2, weight, bias, gelu=True, quant_out=quant_out)
        if quant_out:
            y, pre, q = out
        else:
            y, pre = out
        ctx.wt = _WT.request(weight) if not fp8 and _dgrad_on_token_gemm(x2.shape[0], weight, x.dtype) else None
        ctx.gs = gelu_sink if not quant_out else None          # ops.GeluBackwardSink: pre offered to fc2
        if ctx.gs is not None:
            ctx.gs.pre = pre.view(*x.shape[:-1], N)
        ctx.save_for_backward(x, weight, pre)
        ctx.has_bias = bias is not None
        ctx.fp8 = bool(fp8)
        y = y.view(*x.shape[:-1], N)
        if quant_out:        # the MX fp8 copy of y for the next GEMM: not differentiable
            ctx.mark_non_differentiable(q[0], q[1])
            return y, q[0], q[1]
        return y

    @staticmethod
    def backward(ctx, gy, *_):
        x, weight, pre = ctx.saved_tensors
        M, N = pre.shape
        gy2 = gy.reshape(M, N).to(pre.dtype).contiguous()
        if ctx.gs is not None and ctx.gs.done:
            # fc2's dX GEMM already applied the GELU derivative: gy IS the pre-activation's gradient
            ctx.gs.done = False
            gp, cs = gy2, None
        else:
            gp = torch.empty_like(pre)
            cs = torch.empty(N, device=pre.device, dtype=pre.dtype)
            ws = torch.empty(int(L.lib().vs_column_sum_workspace_bytes(M, N)), device=pre.device, dtype=torch.uint8)
            with ops.timed("act_bwd_colsum", pre, bytes_=3 * pre.numel() * pre.element_size()):
                L.check(L.lib().vs_act_backward_colsum(L.dtype_code(pre), 1, L.ptr(gy2), L.ptr(pre), L.ptr(gp),
                                                       L.ptr(cs), L.ptr(ws), M, N, L.stream(pre)), "act_backward_colsum")
        ctx.gs = None
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = (_dgrad(gp, weight) if ctx.fp8 else _dgrad_gemm(gp, weight, ctx.wt)).view(x.shape)
        ctx.wt = None
        want_b = ctx.has_bias and ctx.needs_input_grad[2]
        x2 = x.reshape(-1, x.shape[-1])
        if want_b and cs is None:
            if ctx.needs_input_grad[1] and _token_wgrad_ok(gp, x2, weight.dtype):
                gw, gb = weight_grad(gp, x2, weight.dtype, bias=True)
            else:
                gb = ops.column_sum(gp).to(weight.dtype)
        elif want_b:
            gb = cs.to(weight.dtype)
        if ctx.needs_input_grad[1] and gw is None:
            gw = weight_grad(gp, x2, weight.dtype)
        return gx, gw, gb, None, None, None, None, None


class _LinearFp8Fn(torch.autograd.Function):
    """x W^T + b with the product on the block-scaled MX MFMA (config C5's fp8 path): x and
    W quantised per 32 elements along K (vs_mx_quantize: e4m3 + e8m0), f32 accumulation,
    bf16 out.  Straight-through: the backward is _LinearFn's, on the bf16 operands."""

    @staticmethod
    def forward(ctx, x, weight, bias, xq=None, xs=None):
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        if xq is None:
            xq, xs = ops.mx_quantize(x2)
        wq, ws = ops.mx_quantize(weight)
        y = ops.token_gemm(xq.reshape(-1, K), wq, bias, x_scales=xs.reshape(-1, K // 32), w_scales=ws)
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        ctx.sink = None
        return y.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, gy):
        """_LinearFn's backward with dX on the MX fp8 GEMM (FP8_DGRAD)."""
        x, weight = ctx.saved_tensors
        gy2 = gy.reshape(-1, gy.shape[-1])
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = _dgrad(gy2, weight).view(x.shape)
        if ctx.needs_input_grad[1]:
            gw = weight_grad(gy2, x.reshape(-1, x.shape[-1]).to(gy2.dtype), weight.dtype)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            cs = ops.take_colsum(gy)
            if cs is not None:
                gb = cs.to(weight.dtype)
            elif gy2.shape[1] % 8 == 0 and gy2.shape[1] <= ops.COLSUM_MAX_N:
                gb = ops.column_sum(gy2).to(weight.dtype)
            else:
                gb = gy2.sum(0, dtype=torch.float32).to(weight.dtype)
        return gx, gw, gb, None, None


_LinearFp8RowFn.backward = _LinearFp8Fn.backward


# fc1 + GELU fused into the STREAMING token GEMM (K <= 128, >= 32768 tokens: Swin-T stage 1):
# one pass writes the pre-activation and the activation, 158 vs 203 us for the vendor GEMM +
# ATen GELU at C2 stage 1 (profiles/r5_tgemm_stream_ab.txt); at K = 192 (stage 2) the fused
# stream kernel's LDS leaves one workgroup per CU and the composition stays faster.
# VS_TGEMM_STREAM_GELU=0: the composition there too (A/B)
_STREAM_GELU = os.environ.get("VS_TGEMM_STREAM_GELU", "1") == "1"
STREAM_MIN_ROWS = int(os.environ.get("VS_TGEMM_STREAM_ROWS", "32768"))


def _stream_gelu_ok(x, w) -> bool:
    return (_STREAM_GELU and STREAM_MIN_ROWS > 0 and w.shape[1] <= 128
            and x.numel() // max(1, x.shape[-1]) >= STREAM_MIN_ROWS)


def linear_gelu_tokens(x, w, b, fp8: bool = False, gelu_sink=None):
    """gelu(F.linear(x, w, b)) with the exact erf GELU: fused into the token GEMM on
    token-heavy bf16 device tensors (_LinearGeluFn), the composition otherwise.  gelu_sink:
    ops.GeluBackwardSink when the output feeds only the MLP's fc2 (linear_tokens with the same
    sink), which then folds the GELU backward into its dX GEMM."""
    if (fp8 or _stream_gelu_ok(x, w)) and _tgemm_ok(x, w, b):
        return _LinearGeluFn.apply(x, w, b, bool(fp8 and w.shape[1] % 128 == 0 and w.shape[1] >= FP8_MIN_K), False,
                                   None, None, gelu_sink)
    return ops.activation(linear_tokens(x, w, b), "gelu", gelu_sink)


def linear_fp8_tokens(x, w, b, xq=None):
    """F.linear with the product in fp8 where it pays: FP8_GEMM "rows" -> the vendor rowwise
    fp8 GEMM (_LinearFp8RowFn) on the shapes of fp8_rows_ok; "mx" -> the MX token GEMM
    (_LinearFp8Fn: K % 128 == 0 and K >= FP8_MIN_K); linear_tokens otherwise.  xq: x's fp8
    copy (e4m3, scales) in the backend's format when its producer made one."""
    if FP8_GEMM == "rows":
        K, N = w.shape[1], w.shape[0]
        if _fp8_rows_ready(x, w, b) and fp8_rows_ok(x.numel() // K, N, K):
            return _LinearFp8RowFn.apply(x, w, b, *(xq if xq is not None else (None, None)))
        return linear_tokens(x, w, b)
    if _tgemm_ok(x, w, b) and w.shape[1] % 128 == 0 and w.shape[1] >= FP8_MIN_K:
        return _LinearFp8Fn.apply(x, w, b, *(xq if xq is not None else (None, None)))
    return linear_tokens(x, w, b)


def mlp_fp8(x, w1, b1, w2, b2, xq=None):
    """fc2(gelu(fc1(x))) on the MX fp8 token GEMM: fc1's epilogue writes the GELU output in
    bf16 (fc2's weight gradient) and as fc2's MX fp8 operand, so no quantisation pass runs
    between the two GEMMs (config C5).  xq: x's MX fp8 copy from its producer (the
    LayerNorm), if it made one."""
    K1, N1 = w1.shape[1], w1.shape[0]
    if FP8_GEMM == "rows":
        # fc1 on the rowwise fp8 GEMM where it pays (x's row-scaled copy from the LayerNorm
        # when it made one), then ONE pass for GELU + fc2's fp8 rows
        M = x.numel() // K1
        h = linear_fp8_tokens(x, w1, b1, xq)
        if _fp8_rows_ready(h, w2, b2) and fp8_rows_ok(M, w2.shape[0], N1) and h.is_contiguous():
            if torch.is_grad_enabled() and h.requires_grad:
                y, yq, ys = ops.gelu_row_quant(h)
            else:
                y, yq, ys = ops.row_quantize_fp8(h, gelu=True)
            return _LinearFp8RowFn.apply(y, w2, b2, yq, ys)
        return linear_tokens(ops.activation(h, "gelu"), w2, b2)
    fc1_fp8 = K1 % 128 == 0 and K1 >= FP8_MIN_K
    if _tgemm_ok(x, w1, b1) and N1 % 128 == 0 and N1 >= FP8_MIN_K and fc1_fp8:
        h, hq, hs = _LinearGeluFn.apply(x, w1, b1, True, True, *(xq if xq is not None else (None, None)))
        return linear_fp8_tokens(h, w2, b2, (hq, hs))
    # fc1 too shallow for fp8 (Swin-L stage 1, K = 192): the vendor GEMM + the GELU pass and
    # one quantisation of h for fc2 run faster than the bf16 token GEMM's GELU + MX-output
    # epilogue (C5: 0.95 vs 1.37 ms a launch, profiles/r4_c5_fp8_vs_bf16_kernel_diff.txt)
    return linear_fp8_tokens(ops.activation(linear_tokens(x, w1, b1), "gelu"), w2, b2)
