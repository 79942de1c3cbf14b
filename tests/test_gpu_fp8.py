"""fp8 (OCP e4m3) window attention, BASELINE config C5 (Swin-L, 1536^2, "fp8 MFMA
window-attention path"), through vs_window_attn_forward_fp8 / _backward_fp8: the
block-scaled MX MFMA v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 operands, one e8m0 scale per
32-element block: every q / k token; P = exp(S - max) <= 1 at one fixed scale, e4m3(256 P);
V, quantised once per workgroup while staged, with one scale per (window, head)).

Two yardsticks per case:
  * the kernel's own quantisation model, emulated in torch on the CPU (f32 math on
    torch.float8_e4m3fn-rounded operands, the same power-of-two scales): checks the MX fragment layout, the scales and the
    fused dequantisation up to f32 summation order and the occasional one-ulp e4m3 flip
    of P (the kernel's exp differs from torch's in the last f32 bit);
  * the exact fp32 oracle (oracle/ref_ops.window_attention_ref, pinned to HF): the fp8
    error budget, stated per test as a relative RMS / max bound.
The backward is the gradient of the quantised logits with straight-through operands
(dV, dP, dQ, dK formed in bf16 from the bf16 operands); its yardstick is that formula in
f32 and, loosely, the exact fp32 autograd gradient."""

import math

import pytest
import torch

from oracle import ref_ops as R

pytestmark = pytest.mark.gpu
DEV = "cuda"
E4M3 = torch.float8_e4m3fn


def _pow2_scale(amax):
    """2^floor(log2(448 / amax)) per block (1 for an all-zero block), as the kernel."""
    s = torch.where(amax > 0, torch.exp2(torch.floor(torch.log2(448.0 / amax.clamp_min(1e-30)))),
                    torch.ones_like(amax))
    return s


def _q8(x, s):
    return (x * s).to(E4M3).float() / s


P_SCALE = 256.0      # the kernel's fixed P scale (csrc/window_attn.hip mx_pfixed)


def _split(qkv, heads):
    Bw, N, C3 = qkv.shape
    q, k, v = qkv.float().view(Bw, N, 3, heads, 32).permute(2, 0, 3, 1, 4)   # [Bw, heads, N, 32]
    return q, k, v


def _bias_mask(table, ws, shift, nWh, nWw, Bw):
    N = ws * ws
    s = R.rel_bias(table.float(), ws).unsqueeze(0)                         # [1, heads, N, N]
    if shift:
        mask = torch.from_numpy(R.shift_attn_mask_np(nWh * ws, nWw * ws, ws, shift))
        nW = mask.shape[0]
        s = s + mask.unsqueeze(1).unsqueeze(0).expand(Bw // nW, -1, -1, -1, -1).reshape(Bw, 1, N, N)
    return s


def _fp8_logits(q, k, bm, scale):
    sq = _pow2_scale(q.abs().amax(dim=3, keepdim=True))          # one scale per token (32 channels)
    sk = _pow2_scale(k.abs().amax(dim=3, keepdim=True))
    return (_q8(q, sq) @ _q8(k, sk).transpose(2, 3)) * scale + bm


def emulate_fwd(qkv, table, heads, ws, shift, nWh, nWw, scale=32 ** -0.5):
    q, k, v = _split(qkv, heads)
    Bw = q.shape[0]
    s = _fp8_logits(q, k, _bias_mask(table, ws, shift, nWh, nWw, Bw), scale)
    m = s.amax(-1, keepdim=True)
    p = torch.exp(s - m)
    l = p.sum(-1, keepdim=True)
    sv = _pow2_scale(v.abs().amax(dim=(2, 3), keepdim=True))    # one scale per (window, head)
    o = (_q8(p, P_SCALE) @ _q8(v, sv)) / l
    return o.transpose(1, 2).reshape(Bw, -1, heads * 32), s


def emulate_bwd(qkv, table, out, go, heads, ws, shift, nWh, nWw, scale=32 ** -0.5):
    """The kernel's backward formula in f32: P from the fp8 logits, every product on the
    unquantised operands."""
    q, k, v = _split(qkv, heads)
    Bw, _, N, _ = q.shape
    s = _fp8_logits(q, k, _bias_mask(table, ws, shift, nWh, nWw, Bw), scale)
    p = torch.softmax(s, -1)
    dO = go.float().view(Bw, N, heads, 32).transpose(1, 2)
    O = out.float().view(Bw, N, heads, 32).transpose(1, 2)
    D = (dO * O).sum(-1, keepdim=True)
    dv = p.transpose(2, 3) @ dO
    ds = p * (dO @ v.transpose(2, 3) - D)
    dq = ds @ k * scale
    dk = ds.transpose(2, 3) @ q * scale
    dqkv = torch.stack([dq, dk, dv], 0).permute(1, 3, 0, 2, 4).reshape(Bw, N, 3 * heads * 32)
    idx = torch.from_numpy(R.rel_position_index_np(ws)).view(-1)
    T2 = (2 * ws - 1) ** 2
    gt = torch.zeros(T2, heads).index_add_(0, idx, ds.sum(0).reshape(heads, N * N).t())
    return dqkv, gt


def _exact(qkv, table, heads, ws, shift, nWh, nWw):
    q, k, v = _split(qkv, heads)
    mask = torch.from_numpy(R.shift_attn_mask_np(nWh * ws, nWw * ws, ws, shift)) if shift else None
    return R.window_attention_ref(q, k, v, table, ws, mask)


def _rel_rms(a, b):
    return float((a - b).pow(2).mean().sqrt() / b.pow(2).mean().sqrt())


CASES = [
    dict(B=1, nWh=3, nWw=2, heads=3, ws=12, shift=6),     # Swin-B/L ws 12 (N = 144, 5 query tiles)
    dict(B=2, nWh=2, nWw=2, heads=2, ws=12, shift=0),
    dict(B=1, nWh=2, nWw=3, heads=2, ws=10, shift=5),     # N = 100 (4 tiles)
    dict(B=1, nWh=3, nWw=3, heads=2, ws=9, shift=4),      # N = 81 (3 tiles)
    dict(B=2, nWh=2, nWw=3, heads=3, ws=7, shift=3),      # Swin-T ws 7 (N = 49, 2 tiles)
    dict(B=1, nWh=8, nWw=8, heads=6, ws=12, shift=6),     # Swin-L stage 1 @1536^2 tile (heads 6)
]


def _inputs(cfg, seed, qscale=1.0):
    Bw = cfg["B"] * cfg["nWh"] * cfg["nWw"]
    N, C = cfg["ws"] ** 2, cfg["heads"] * 32
    g = torch.Generator().manual_seed(seed)
    qkv = (qscale * torch.randn(Bw, N, 3 * C, generator=g)).to(torch.bfloat16)
    table = torch.randn((2 * cfg["ws"] - 1) ** 2, cfg["heads"], generator=g)
    go = torch.randn(Bw, N, C, generator=g).to(torch.bfloat16)
    return qkv, table, go


@pytest.mark.parametrize("cfg", CASES)
def test_fp8_window_attention_forward(cfg):
    from visionseg import ops
    qkv, table, _ = _inputs(cfg, 11)
    geo = (cfg["heads"], cfg["ws"], cfg["shift"], cfg["nWh"], cfg["nWw"])
    with torch.no_grad():
        out = ops.window_attention(qkv.to(DEV), table.to(DEV), *geo, fp8=True).float().cpu()
    emu, _ = emulate_fwd(qkv, table, *geo)
    exact = _exact(qkv, table, *geo)
    err_emu = (out - emu).abs()
    vmax = float(qkv.float().abs().max())
    rr = _rel_rms(out, exact)
    print(f"fp8 fwd ws{cfg['ws']}: vs emulation max {float(err_emu.max()):.2e} mean {float(err_emu.mean()):.2e}; "
          f"vs exact rel-RMS {rr:.3e} max {float((out - exact).abs().max()):.2e}")
    # emulation: bf16 output rounding + a rare one-ulp e4m3 flip of one P entry
    assert float(err_emu.mean()) <= 2e-3 * vmax
    assert float(err_emu.max()) <= 0.08 * vmax
    # fp8 budget vs the exact fp32 attention (e4m3: 3 mantissa bits on q, k, v and P);
    # measured round 2 on MI355X (per-window scales): rel-RMS 0.043-0.048 over these cases
    assert rr <= 0.08, rr


@pytest.mark.parametrize("cfg", CASES[:3] + CASES[4:5])
def test_fp8_window_attention_backward(cfg):
    from visionseg import ops
    qkv, table, go = _inputs(cfg, 12)
    geo = (cfg["heads"], cfg["ws"], cfg["shift"], cfg["nWh"], cfg["nWw"])
    qd = qkv.to(DEV).requires_grad_(True)
    td = table.to(DEV).requires_grad_(True)
    out = ops.window_attention(qd, td, *geo, fp8=True)
    out.backward(go.to(DEV))
    gq, gt = qd.grad.float().cpu(), td.grad.float().cpu()
    eq, et = emulate_bwd(qkv, table, out.detach().cpu(), go, *geo)
    # exact fp32 gradient of the unquantised attention
    qr = qkv.float().clone().requires_grad_(True)
    tr = table.clone().requires_grad_(True)
    _exact(qr, tr, *geo).backward(go.float())
    parts = []
    for i, name in enumerate("qkv"):
        sl = slice(i * cfg["heads"] * 32, (i + 1) * cfg["heads"] * 32)
        a = gq.view(gq.shape[0], gq.shape[1], -1)[..., sl]
        b = eq.view(eq.shape[0], eq.shape[1], -1)[..., sl]
        c = qr.grad.view(gq.shape[0], gq.shape[1], -1)[..., sl]
        m = float(b.abs().max())
        parts.append((name, float((a - b).abs().max()) / m, _rel_rms(a, c)))
        # the kernel's formula: bf16 P / dS / operand rounding (as the bf16 MFMA path)
        assert float((a - b).abs().max()) <= 3e-2 * m, (name, parts[-1])
        # vs the exact gradient: fp8 logits move P by a few %
        assert _rel_rms(a, c) <= 0.15, (name, parts[-1])
    tmax = float(et.abs().max())
    terr = float((gt - et).abs().max()) / tmax
    print(f"fp8 bwd ws{cfg['ws']}: " + ", ".join(f"d{n} {e:.2e} (exact rel-RMS {r:.2e})" for n, e, r in parts)
          + f"; dtable {terr:.2e} (exact rel-RMS {_rel_rms(gt, tr.grad):.2e})")
    assert terr <= 3e-2
    assert _rel_rms(gt, tr.grad) <= 0.15


def test_fp8_scales_cover_large_and_small_magnitudes():
    """Per-block scales: activations at 1e-3 and at 1e2 scale (where a fixed e4m3
    scale would underflow / overflow) keep the same relative error."""
    from visionseg import ops
    cfg = CASES[0]
    geo = (cfg["heads"], cfg["ws"], cfg["shift"], cfg["nWh"], cfg["nWw"])
    errs = []
    for sc in (1e-3, 1.0, 30.0):
        qkv, table, _ = _inputs(cfg, 13, qscale=sc)
        with torch.no_grad():
            out = ops.window_attention(qkv.to(DEV), table.to(DEV), *geo, fp8=True).float().cpu()
        emu, _ = emulate_fwd(qkv, table, *geo)
        assert bool(torch.isfinite(out).all())
        errs.append(_rel_rms(out, emu))
    print("fp8 rel-RMS vs emulation at activation scales 1e-3 / 1 / 30:", errs)
    assert max(errs) <= 2e-2


def test_fp8_rejects_unsupported():
    from visionseg import ops
    qkv = torch.zeros(4, 49, 3 * 64, device=DEV)
    table = torch.zeros(169, 2, device=DEV)
    with pytest.raises(ValueError):
        ops.window_attention(qkv, table, 2, 7, 0, 2, 2, fp8=True)          # f32 storage
    qkv = torch.zeros(1, 196, 3 * 64, device=DEV, dtype=torch.bfloat16)
    table = torch.zeros(729, 2, device=DEV)
    with pytest.raises(ValueError):
        ops.window_attention(qkv, table, 2, 14, 0, 1, 1, fp8=True)         # N > 160


def test_swin_l_fp8_model_vs_oracle():
    """Config C5's model (Swin-L + Mask2Former, ws 12) with fp8 window attention in every
    Swin block, bf16 everywhere else, vs the fp32 oracle on the same bf16-rounded weights,
    at 384^2 (the C5 arithmetic per window is resolution-independent; 1536^2 is the bench
    shape).  Yardstick: the same model with the bf16 window-attention kernels; the fp8
    mode may add error but must stay within 2.5x of it and within the absolute caps
    (max 0.08 / mean 0.01 of the step's max |logit|).  Measured round 2: bf16 attention
    1.42e-2 / 2.04e-3, fp8 attention 1.41e-2 / 2.02e-3 (the logits' error is dominated by
    the bf16 activations elsewhere)."""
    from visionseg.model import M2FConfig, Mask2Former
    from oracle.ref_model import RefConfig, RefMask2Former
    cfg = M2FConfig.preset("swin_l", num_queries=100)
    m = Mask2Former(cfg).init_weights(0)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "rel_table" in n or "attention_weights" in n or "level_embed" in n:
                p.add_(0.3 * torch.randn(p.shape, generator=g))
        for p in m.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    ref = RefMask2Former(RefConfig.from_dict(cfg.to_dict()))
    ref.load_state_dict({k: v.clone() for k, v in m.state_dict().items()})
    ref.eval()
    px = torch.randn(1, 3, 384, 384, generator=torch.Generator().manual_seed(5)).to(torch.bfloat16).float()
    with torch.no_grad():
        ref.decoder.record = True
        rmasks, _ = ref(px)
        forced = [rb for rb, _ in ref.decoder.trace]
        m = m.to(DEV).to(torch.bfloat16).eval()
        m.decoder.mask_override = forced
        res = {}
        for fp8 in (False, True):
            for st in m.backbone.stages:
                for blk in st.blocks:
                    blk.attn_fp8 = fp8
            masks, _ = m(px.to(DEV).to(torch.bfloat16))
            wmax = max(float((a.float().cpu() - b).abs().max()) / float(b.abs().max()) for a, b in zip(masks, rmasks))
            wmean = max(float((a.float().cpu() - b).abs().mean()) / float(b.abs().max()) for a, b in zip(masks, rmasks))
            res[fp8] = (wmax, wmean)
    print(f"swin_l@384 mask logits vs fp32 oracle: bf16 attention max {res[False][0]:.2e} mean {res[False][1]:.2e}; "
          f"fp8 attention max {res[True][0]:.2e} mean {res[True][1]:.2e}")
    assert res[True][0] <= max(2.5 * res[False][0], 0.02) and res[True][1] <= max(2.5 * res[False][1], 3e-3)
    assert res[True][0] <= 0.08 and res[True][1] <= 0.01


def test_swin_l_fp8_linears_model_vs_oracle_and_step():
    """Config C5's fp8 Linears (M2FConfig.linear_fp8: qkv / proj / fc1 / fc2 on the MX fp8
    token GEMM where K >= 384, the norms and fc1's GELU epilogue handing over e4m3 + scales,
    straight-through bf16 weight gradients), alone and with fp8 window attention, vs the
    fp32 oracle at 384^2 with the oracle's attention masks forced in (Swin-L's stage 1 is
    192 wide: its block stays bf16 except the 768-deep fc2).  Yardstick: the all-bf16 model.
    Caps: max 0.15 / mean 0.02 of the step's max |logit| (twice the fp8-attention caps:
    e4m3 operands in every K-deep product of the backbone; the per-GEMM error budget is
    tests/test_gpu_tgemm.py's).  Then one training step with fp8 Linears through the
    Trainer: finite loss and gradients, weights move."""
    from visionseg.criterion import SetCriterion
    from visionseg.data import synthetic_batch
    from visionseg.model import M2FConfig, Mask2Former
    from visionseg.train import SolverConfig, Trainer
    from oracle.ref_model import RefConfig, RefMask2Former
    cfg = M2FConfig.preset("swin_l", num_queries=100)
    m = Mask2Former(cfg).init_weights(0)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "rel_table" in n or "attention_weights" in n or "level_embed" in n:
                p.add_(0.3 * torch.randn(p.shape, generator=g))
        for p in m.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    ref = RefMask2Former(RefConfig.from_dict(cfg.to_dict()))
    ref.load_state_dict({k: v.clone() for k, v in m.state_dict().items()})
    ref.eval()
    px = torch.randn(1, 3, 384, 384, generator=torch.Generator().manual_seed(5)).to(torch.bfloat16).float()
    with torch.no_grad():
        ref.decoder.record = True
        rmasks, _ = ref(px)
        forced = [rb for rb, _ in ref.decoder.trace]
        m = m.to(DEV).to(torch.bfloat16).eval()
        m.decoder.mask_override = forced
        res = {}
        for mode in ("bf16", "linear_fp8", "all_fp8"):
            for st in m.backbone.stages:
                for blk in st.blocks:
                    blk.linear_fp8 = blk.mlp.fp8 = mode != "bf16"
                    blk.attn_fp8 = mode == "all_fp8"
            masks, _ = m(px.to(DEV).to(torch.bfloat16))
            wmax = max(float((a.float().cpu() - b).abs().max()) / float(b.abs().max()) for a, b in zip(masks, rmasks))
            wmean = max(float((a.float().cpu() - b).abs().mean()) / float(b.abs().max()) for a, b in zip(masks, rmasks))
            res[mode] = (wmax, wmean)
    print("swin_l@384 mask logits vs fp32 oracle (max, mean of max|logit|): "
          + ", ".join(f"{k} {v[0]:.2e} / {v[1]:.2e}" for k, v in res.items()))
    for mode in ("linear_fp8", "all_fp8"):
        assert res[mode][0] <= 0.15 and res[mode][1] <= 0.02, (mode, res)
    del m
    torch.cuda.empty_cache()
    cfg8 = M2FConfig.preset("swin_l", linear_fp8=True)
    tr = Trainer(Mask2Former(cfg8).init_weights(0), SetCriterion(cfg8), SolverConfig(warmup_iters=0), device=DEV)
    assert any(b.linear_fp8 and b.mlp.fp8 for st in tr.model.backbone.stages for b in st.blocks)
    batch = synthetic_batch(2, 384, seed=42, device=DEV)
    w0 = tr.opt.master.clone()
    losses = [float(tr.step(*batch)) for _ in range(2)]
    torch.cuda.synchronize()
    print("swin_l@384 fp8-Linear training losses", losses)
    assert all(math.isfinite(v) for v in losses)
    assert bool(torch.isfinite(tr.opt.master).all()) and float((tr.opt.master - w0).abs().max()) > 0
