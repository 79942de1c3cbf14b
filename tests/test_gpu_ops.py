"""GPU parity of the hand-written kernels against the oracle (through the C ABI).

Index ops: bit-exact.  f32 kernels vs the fp32 oracle: <= 1e-5 abs (op level).  bf16
kernels: compared with the oracle evaluated on the same bf16-rounded inputs in f32;
tolerance stated per test (bf16 output rounding, 2^-8 relative).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import ref_ops as R

pytestmark = pytest.mark.gpu

DEV = "cuda"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ops():
    from visionseg import ops
    return ops


# ------------------------------------------------------------------ window ops
WINDOW_CASES = [
    (2, 10, 13, 8, 7, 3), (1, 9, 9, 4, 4, 2), (1, 14, 7, 5, 7, 0), (3, 4, 4, 6, 7, 3), (1, 24, 24, 3, 12, 6),
    (2, 64, 64, 96, 7, 3),            # Swin-T stage-1 tile, bf16-friendly 16-B rows
    (1, 256, 256, 96, 7, 3),          # Swin-T stage 1 at 1024^2 (pad 256 -> 259)
    (1, 32, 32, 768, 7, 3),           # Swin-T stage 4 at 1024^2 (pad 32 -> 35)
    (1, 64, 64, 512, 12, 6),          # Swin-B stage 3, ws 12
]


@pytest.mark.parametrize("case", WINDOW_CASES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_window_partition_reverse_bit_exact(case, dtype):
    ops = _ops()
    B, H, W, C, ws, shift = case
    g = torch.Generator().manual_seed(hash(case) % 1000)
    x = torch.randn(B, H, W, C, generator=g).to(dtype)
    xd = x.to(DEV)
    win = ops.window_partition(xd, ws, shift)
    x_np = x.view(torch.int16).numpy() if dtype == torch.bfloat16 else x.numpy()
    exp = R.window_partition_np(x_np, ws, shift)
    got = win.cpu()
    got = got.view(torch.int16).numpy() if dtype == torch.bfloat16 else got.numpy()
    assert np.array_equal(got, exp)
    back = ops.window_reverse(win, B, H, W, ws, shift)
    assert torch.equal(back.cpu().view(torch.int16) if dtype == torch.bfloat16 else back.cpu(),
                       x.view(torch.int16) if dtype == torch.bfloat16 else x)


def test_window_ops_autograd_roundtrip():
    ops = _ops()
    B, H, W, C, ws, shift = 2, 10, 13, 8, 7, 3
    x = torch.randn(B, H, W, C, device=DEV, requires_grad=True)
    win = ops.window_partition(x, ws, shift)
    gw = torch.randn_like(win)
    (win * gw).sum().backward()
    exp = R.window_reverse_np(gw.cpu().numpy(), B, H, W, ws, shift)
    assert np.array_equal(x.grad.cpu().numpy(), exp)
    w2 = torch.randn_like(win).requires_grad_(True)
    y = ops.window_reverse(w2, B, H, W, ws, shift)
    gy = torch.randn_like(y)
    (y * gy).sum().backward()
    exp2 = R.window_partition_np(gy.cpu().numpy(), ws, shift)
    assert np.array_equal(w2.grad.cpu().numpy(), exp2)


# ------------------------------------------------------------------ MSDA
def _msda_inputs(B, shapes, H, Q, P, seed, spread=1.4):
    g = torch.Generator().manual_seed(seed)
    S = sum(h * w for h, w in shapes)
    L = len(shapes)
    value = torch.randn(B, S, H, 32, generator=g)
    loc = torch.rand(B, Q, H, L, P, 2, generator=g) * spread - (spread - 1) / 2
    w = torch.softmax(torch.randn(B, Q, H, L * P, generator=g), -1).view(B, Q, H, L, P)
    return value, loc, w


def test_msda_golden_fixture(golden):
    """Kernel vs the HF-generated fixture (borders, pixel centres, outside points)."""
    ops = _ops()
    d = golden("msda.npz")
    shapes = [tuple(x) for x in d["shapes"].tolist()]
    v = torch.from_numpy(d["value"]).to(DEV).requires_grad_(True)
    loc = torch.from_numpy(d["loc"]).to(DEV).requires_grad_(True)
    w = torch.from_numpy(d["weights"]).to(DEV).requires_grad_(True)
    o = ops.ms_deform_attn(v, shapes, loc, w)
    np.testing.assert_allclose(o.detach().cpu().numpy(), d["out"], atol=1e-5, rtol=0)
    o.backward(torch.from_numpy(d["grad_out"]).to(DEV))
    np.testing.assert_allclose(v.grad.cpu().numpy(), d["grad_value"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(w.grad.cpu().numpy(), d["grad_weights"], atol=1e-5, rtol=0)


@pytest.mark.parametrize("cfg", [
    dict(B=2, shapes=[(6, 7), (3, 4), (2, 2)], H=2, Q=11, P=4),
    dict(B=1, shapes=[(32, 32), (64, 64), (128, 128)], H=8, Q=21504, P=4),   # 1024^2, one image
    dict(B=2, shapes=[(16, 16), (32, 32), (64, 64), (8, 8)], H=8, Q=300, P=4),  # 4 levels (MaskDINO)
])
def test_msda_fp32_vs_oracle(cfg):
    ops = _ops()
    value, loc, w = _msda_inputs(cfg["B"], cfg["shapes"], cfg["H"], cfg["Q"], cfg["P"], seed=5)
    vr, lr, wr = (t.clone().requires_grad_(True) for t in (value, loc, w))
    ref = R.msda_ref(vr, cfg["shapes"], lr, wr)
    go = torch.randn(ref.shape, generator=torch.Generator().manual_seed(9))
    ref.backward(go)
    vd, ld, wd = (t.to(DEV).requires_grad_(True) for t in (value, loc, w))
    out = ops.ms_deform_attn(vd, cfg["shapes"], ld, wd)
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), atol=1e-5, rtol=0)
    out.backward(go.to(DEV))
    np.testing.assert_allclose(vd.grad.cpu().numpy(), vr.grad.numpy(), atol=2e-5, rtol=0)
    np.testing.assert_allclose(wd.grad.cpu().numpy(), wr.grad.numpy(), atol=2e-5, rtol=0)
    gl = lr.grad.numpy()
    np.testing.assert_allclose(ld.grad.cpu().numpy(), gl, atol=2e-5 * max(1.0, np.abs(gl).max()), rtol=0)


def test_msda_bf16_vs_oracle():
    ops = _ops()
    shapes = [(32, 32), (64, 64), (128, 128)]
    value, loc, w = _msda_inputs(1, shapes, 8, 4096, 4, seed=6)
    vb = value.to(torch.bfloat16)
    ref = R.msda_ref(vb.float(), shapes, loc, w)
    out = ops.ms_deform_attn(vb.to(DEV), shapes, loc.to(DEV), w.to(DEV))
    assert out.dtype == torch.bfloat16
    err = (out.float().cpu() - ref).abs()
    # output rounded once to bf16: |err| <= 2^-8 * |ref| + tiny accumulation slack
    assert bool((err <= ref.abs() * 2 ** -8 + 1e-3).all()), float(err.max())


def test_msda_rejects_bad_shapes():
    ops = _ops()
    v = torch.zeros(1, 10, 1, 32, device=DEV)
    loc = torch.zeros(1, 2, 1, 1, 1, 2, device=DEV)
    w = torch.zeros(1, 2, 1, 1, 1, device=DEV)
    with pytest.raises(ValueError):
        ops.ms_deform_attn(v, [(3, 3)], loc, w)


# ------------------------------------------------------------------ window attention
def _win_attn_ref(qkv, table, heads, ws, shift, nWh, nWw):
    Bw, N, C3 = qkv.shape
    q, k, v = qkv.view(Bw, N, 3, heads, 32).permute(2, 0, 3, 1, 4)
    mask = torch.from_numpy(R.shift_attn_mask_np(nWh * ws, nWw * ws, ws, shift)) if shift else None
    return R.window_attention_ref(q, k, v, table, ws, mask)


@pytest.mark.parametrize("cfg", [
    dict(B=2, nWh=2, nWw=3, heads=2, ws=7, shift=3),
    dict(B=1, nWh=2, nWw=2, heads=1, ws=7, shift=0),
    dict(B=1, nWh=3, nWw=2, heads=3, ws=12, shift=6),
    dict(B=1, nWh=37, nWw=37, heads=3, ws=7, shift=3),    # Swin-T stage 1 @ 1024^2, one image
])
def test_window_attention_fp32_vs_oracle(cfg):
    ops = _ops()
    Bw = cfg["B"] * cfg["nWh"] * cfg["nWw"]
    N, C = cfg["ws"] ** 2, cfg["heads"] * 32
    g = torch.Generator().manual_seed(3)
    qkv = torch.randn(Bw, N, 3 * C, generator=g)
    table = torch.randn((2 * cfg["ws"] - 1) ** 2, cfg["heads"], generator=g)
    qr, tr = qkv.clone().requires_grad_(True), table.clone().requires_grad_(True)
    ref = _win_attn_ref(qr, tr, cfg["heads"], cfg["ws"], cfg["shift"], cfg["nWh"], cfg["nWw"])
    go = torch.randn(ref.shape, generator=g)
    ref.backward(go)
    qd, td = qkv.to(DEV).requires_grad_(True), table.to(DEV).requires_grad_(True)
    out = ops.window_attention(qd, td, cfg["heads"], cfg["ws"], cfg["shift"], cfg["nWh"], cfg["nWw"])
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), atol=1e-5, rtol=0)
    out.backward(go.to(DEV))
    np.testing.assert_allclose(qd.grad.cpu().numpy(), qr.grad.numpy(), atol=5e-5, rtol=0)
    gt = tr.grad.numpy()
    np.testing.assert_allclose(td.grad.cpu().numpy(), gt, atol=1e-4 * max(1.0, np.abs(gt).max()), rtol=1e-5)


def test_window_attention_bf16_vs_oracle():
    ops = _ops()
    B, nWh, nWw, heads, ws, shift = 2, 4, 4, 3, 7, 3
    Bw, N, C = B * nWh * nWw, ws * ws, heads * 32
    g = torch.Generator().manual_seed(4)
    qkv = torch.randn(Bw, N, 3 * C, generator=g).to(torch.bfloat16)
    table = torch.randn((2 * ws - 1) ** 2, heads, generator=g)
    ref = _win_attn_ref(qkv.float(), table, heads, ws, shift, nWh, nWw)
    out = ops.window_attention(qkv.to(DEV), table.to(DEV), heads, ws, shift, nWh, nWw)
    err = (out.float().cpu() - ref).abs()
    # the MFMA path rounds P to bf16 for the P.V product (flash-attention practice)
    assert bool((err <= ref.abs() * 2 ** -7 + 4e-3).all()), float(err.max())


# ------------------------------------------------------------------ mask head + bitmask
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_mask_head_grad_sink_sums_calls(dtype):
    """Several mask-head calls sharing one pixel embedding through ops.GradSink: the
    embedding gradient (accumulated in place by the backward kernel) equals autograd's sum
    of the per-call gradients; the mask-embedding gradients are unchanged."""
    ops = _ops()
    g = torch.Generator(device=DEV).manual_seed(0)
    B, Q, C, H, W, calls = 2, 100, 256, 32, 48, 4
    P = (torch.randn(B, H * W, C, device=DEV, generator=g)).to(dtype)
    Es = [torch.randn(B, Q, C, device=DEV, generator=g).to(dtype) for _ in range(calls)]
    gls = [torch.randn(B, Q, H, W, device=DEV, generator=g) for _ in range(calls)]
    outs = []
    for use_sink in (False, True):
        p = P.clone().requires_grad_(True)
        es = [e.clone().requires_grad_(True) for e in Es]
        sink = ops.GradSink() if use_sink else None
        src = sink.source(p) if use_sink else p
        loss = sum((ops.mask_head(e, src, H, W, sink=sink) * gl).sum() for e, gl in zip(es, gls))
        loss.backward()
        outs.append((p.grad.float(), [e.grad.float() for e in es]))
    (pa, ea), (pb, eb) = outs
    tol = 1e-5 if dtype == torch.float32 else 2 ** -6
    assert float((pa - pb).abs().max()) <= tol * float(pa.abs().max())
    for x, y in zip(ea, eb):
        assert torch.equal(x, y)


def test_mask_head_golden(golden):
    """MLP on host-side torch, einsum + mask on the kernels vs the HF predictor fixture."""
    ops = _ops()
    d = golden("mask_head.npz")
    h = torch.from_numpy(d["h"]).transpose(0, 1)
    pix = torch.from_numpy(d["pix"])
    lin = [(torch.from_numpy(d[f"w_mask_embedder.{i}.0.weight"]), torch.from_numpy(d[f"w_mask_embedder.{i}.0.bias"]))
           for i in range(3)]
    e = torch.relu(torch.nn.functional.linear(h, *lin[0]))
    e = torch.relu(torch.nn.functional.linear(e, *lin[1]))
    e = torch.nn.functional.linear(e, *lin[2])
    B, C, H, W = pix.shape
    nhwc = pix.permute(0, 2, 3, 1).reshape(B, H * W, C)
    lo = ops.mask_head(e.to(DEV), nhwc.to(DEV), H, W)
    for ti in range(4):
        tgt = tuple(d[f"t{ti}_size"].tolist())
        np.testing.assert_allclose(lo.cpu().numpy(), d[f"t{ti}_logits"], atol=1e-5, rtol=0)
        words = ops.attn_bitmask(lo, tgt)
        blocked = ops.unpack_bitmask(words, tgt[0] * tgt[1]).cpu()
        exp = R.unblock_full_rows(torch.from_numpy(d[f"t{ti}_mask"]).view(B, 2, -1, tgt[0] * tgt[1])[:, 0])
        assert torch.equal(blocked, exp), ti


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 100, 256, 64, 64), (1, 300, 256, 32, 48), (4, 100, 256, 256, 256)])
def test_mask_head_vs_oracle(dtype, shape):
    ops = _ops()
    B, Q, C, H, W = shape
    g = torch.Generator().manual_seed(12)
    E = (torch.randn(B, Q, C, generator=g) / 8).to(dtype)
    P = torch.randn(B, H * W, C, generator=g).to(dtype)
    Ed, Pd = E.to(DEV), P.to(DEV)
    lo = ops.mask_head(Ed, Pd, H, W)
    # oracle on the same (rounded) inputs in f32; bf16 products are exact in f32
    for b in range(B):
        ref = torch.einsum("qc,nc->qn", E[b].float(), P[b].float()).view(Q, H, W)
        np.testing.assert_allclose(lo[b].cpu().numpy(), ref.numpy(), atol=2e-5 if dtype == torch.float32 else 1e-4,
                                   rtol=1e-5)
        if B * H * W > 65536 and b > 0:
            break


def test_attn_bitmask_vs_oracle():
    ops = _ops()
    g = torch.Generator().manual_seed(13)
    lo = torch.randn(2, 7, 64, 64, generator=g) * 3
    lo[0, 2] = -5.0          # fully blocked row -> un-blocked by the fix
    for tgt in [(8, 8), (16, 16), (32, 32), (64, 64), (5, 7), (37, 61), (128, 128), (1, 1)]:
        words = ops.attn_bitmask(lo.to(DEV), tgt)
        am = torch.nn.functional.interpolate(lo, size=tgt, mode="bilinear", align_corners=False)
        exp = R.unblock_full_rows(am.sigmoid().flatten(2) < 0.5)
        got = ops.unpack_bitmask(words, tgt[0] * tgt[1]).cpu()
        assert torch.equal(got, exp), tgt
        assert not got[0, 2].any()


# ------------------------------------------------------------------ masked cross-attention
def _xattn_case(B, Q, S, heads, seed, dtype=torch.float32, p_block=0.7):
    g = torch.Generator().manual_seed(seed)
    C = heads * 32
    q = torch.randn(B, Q, C, generator=g).to(dtype)
    k = torch.randn(B, S, C, generator=g).to(dtype)
    v = torch.randn(B, S, C, generator=g).to(dtype)
    blocked = torch.rand(B, Q, S, generator=g) < p_block
    blocked[0, 0] = True                  # fully blocked -> fixed
    blocked = R.unblock_full_rows(blocked)
    nw = (S + 31) // 32
    pad = torch.zeros(B, Q, nw * 32, dtype=torch.bool)
    pad[..., :S] = blocked
    bits = (pad.view(B, Q, nw, 32).to(torch.int64) << torch.arange(32)).sum(-1)
    words = torch.where(bits >= 2 ** 31, bits - 2 ** 32, bits).to(torch.int32)
    return q, k, v, blocked, words


@pytest.mark.parametrize("cfg", [dict(B=2, Q=7, S=40, heads=2), dict(B=2, Q=100, S=1024, heads=8),
                                 dict(B=1, Q=100, S=16384, heads=8), dict(B=1, Q=300, S=4096, heads=8)])
def test_masked_attention_fp32_vs_oracle(cfg):
    ops = _ops()
    q, k, v, blocked, words = _xattn_case(cfg["B"], cfg["Q"], cfg["S"], cfg["heads"], seed=21)
    assert torch.equal(ops.unpack_bitmask(words, cfg["S"]), blocked)
    H = cfg["heads"]
    qr, kr, vr = (t.clone().requires_grad_(True) for t in (q, k, v))
    B, Q, C = q.shape
    S = k.shape[1]
    ref = R.masked_attention_ref(qr.view(B, Q, H, 32).transpose(1, 2), kr.view(B, S, H, 32).transpose(1, 2),
                                 vr.view(B, S, H, 32).transpose(1, 2), blocked)
    go = torch.randn(ref.shape, generator=torch.Generator().manual_seed(22))
    ref.backward(go)
    qd, kd, vd = (t.to(DEV).requires_grad_(True) for t in (q, k, v))
    out = ops.masked_attention(qd, kd, vd, words.to(DEV), H)
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), atol=1e-5, rtol=0)
    out.backward(go.to(DEV))
    for a, r_ in ((qd, qr), (kd, kr), (vd, vr)):
        np.testing.assert_allclose(a.grad.cpu().numpy(), r_.grad.numpy(), atol=5e-5, rtol=0)


def test_masked_attention_golden(golden):
    ops = _ops()
    d = golden("masked_attn.npz")
    D, heads = 64, 2
    W = torch.from_numpy(d["w_in_proj_weight"])
    b = torch.from_numpy(d["w_in_proj_bias"])
    q = torch.nn.functional.linear(torch.from_numpy(d["q"]).transpose(0, 1), W[:D], b[:D])
    k = torch.nn.functional.linear(torch.from_numpy(d["k"]).transpose(0, 1), W[D:2 * D], b[D:2 * D])
    v = torch.nn.functional.linear(torch.from_numpy(d["v"]).transpose(0, 1), W[2 * D:], b[2 * D:])
    B, Q, S = q.shape[0], q.shape[1], k.shape[1]
    blocked = torch.from_numpy(d["blocked_fixed"]).view(B, heads, Q, S)[:, 0]
    nw = (S + 31) // 32
    pad = torch.zeros(B, Q, nw * 32, dtype=torch.bool)
    pad[..., :S] = blocked
    bits = (pad.view(B, Q, nw, 32).to(torch.int64) << torch.arange(32)).sum(-1)
    words = torch.where(bits >= 2 ** 31, bits - 2 ** 32, bits).to(torch.int32)
    o = ops.masked_attention(q.to(DEV), k.to(DEV), v.to(DEV), words.to(DEV), heads).cpu()
    o = torch.nn.functional.linear(o, torch.from_numpy(d["w_out_proj.weight"]), torch.from_numpy(d["w_out_proj.bias"]))
    np.testing.assert_allclose(o.transpose(0, 1).numpy(), d["out"], atol=1e-5, rtol=0)


def test_masked_attention_bf16_vs_oracle():
    ops = _ops()
    q, k, v, blocked, words = _xattn_case(2, 100, 4096, 8, seed=23, dtype=torch.bfloat16)
    B, Q, C = q.shape
    S = k.shape[1]
    ref = R.masked_attention_ref(q.float().view(B, Q, 8, 32).transpose(1, 2), k.float().view(B, S, 8, 32).transpose(1, 2),
                                 v.float().view(B, S, 8, 32).transpose(1, 2), blocked)
    out = ops.masked_attention(q.to(DEV), k.to(DEV), v.to(DEV), words.to(DEV), 8)
    err = (out.float().cpu() - ref).abs()
    assert bool((err <= ref.abs() * 2 ** -8 + 1e-3).all()), float(err.max())


@pytest.mark.parametrize("shape", [(2, 100, 256, 64, 64), (4, 100, 256, 256, 256), (1, 37, 128, 20, 30)])
def test_mask_head_backward_bf16_vs_oracle(shape):
    """Fused bf16 backward vs f32 GEMMs on the same bf16-rounded operands (dL rounded to
    bf16 as the MFMA consumes it): accumulation-order differences only."""
    ops = _ops()
    B, Q, C, H, W = shape
    g = torch.Generator().manual_seed(14)
    E = (torch.randn(B, Q, C, generator=g) / 8).to(torch.bfloat16)
    P = torch.randn(B, H * W, C, generator=g).to(torch.bfloat16)
    gl = torch.randn(B, Q, H, W, generator=g)
    Ed, Pd = E.to(DEV).requires_grad_(True), P.to(DEV).requires_grad_(True)
    lo = ops.mask_head(Ed, Pd, H, W)
    lo.backward(gl.to(DEV))
    glb = gl.to(torch.bfloat16).float().view(B, Q, H * W)
    for b in range(min(B, 2)):
        refE = glb[b] @ P[b].float()
        refP = glb[b].t() @ E[b].float()
        gE = Ed.grad[b].float().cpu()
        gP = Pd.grad[b].float().cpu()
        assert float((gE - refE).abs().max()) <= 2 ** -7 * float(refE.abs().max()) + 1e-3
        assert float((gP - refP).abs().max()) <= 2 ** -7 * float(refP.abs().max()) + 1e-3


@pytest.mark.parametrize("cfg", [
    dict(B=2, shapes=[(6, 7), (3, 4), (2, 2)], H=2, spread=2.0),
    dict(B=1, shapes=[(32, 32), (64, 64), (128, 128)], H=8, spread=4.0),     # 1024^2 pixel decoder, init-like
    dict(B=1, shapes=[(16, 16), (32, 32), (64, 64)], H=8, spread=12.0),      # many far taps (atomic path)
    dict(B=2, shapes=[(12, 20), (24, 40), (48, 80)], H=8, spread=3.0),       # non-square (tiny fixture 'b' like)
    dict(B=2, shapes=[(48, 80), (24, 40), (12, 20), (6, 10)], H=4, spread=3.0),  # 4 levels, finest first
])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_msda_encoder_shapes_backward_vs_oracle(cfg, dtype):
    """The default backward (geom gather + query-tile LDS-window scatter) on pixel-decoder
    encoder problems (queries = value grid) vs the oracle: the 1024^2 level shapes with
    init-like offsets, many far taps (clipped windows: direct atomics), non-square
    levels, and 4 levels stored finest first."""
    ops = _ops()
    shapes, B, H, L, P = cfg["shapes"], cfg["B"], cfg["H"], len(cfg["shapes"]), 4
    S = sum(h * w for h, w in shapes)
    g = torch.Generator().manual_seed(31)
    ref = R.reference_points(shapes, B)                                          # [B,S,L,2]
    off = (torch.rand(B, S, H, L, P, 2, generator=g) * 2 - 1) * cfg["spread"]
    norm = torch.tensor([[w, h] for h, w in shapes], dtype=torch.float32)[None, None, None, :, None, :]
    loc = ref[:, :, None, :, None, :] + off / norm
    value = torch.randn(B, S, H, 32, generator=g).to(dtype)
    w = torch.softmax(torch.randn(B, S, H, L * P, generator=g), -1).view(B, S, H, L, P)
    vr, lr, wr = value.float().clone().requires_grad_(True), loc.clone().requires_grad_(True), w.clone().requires_grad_(True)
    out_r = R.msda_ref(vr, shapes, lr, wr)
    go = torch.randn(out_r.shape, generator=g)
    go_q = go.to(dtype).float()
    out_r.backward(go_q)
    vd, ld, wd = value.to(DEV).requires_grad_(True), loc.to(DEV).requires_grad_(True), w.to(DEV).requires_grad_(True)
    out = ops.ms_deform_attn(vd, shapes, ld, wd)
    out.backward(go.to(dtype).to(DEV))
    if dtype == torch.float32:
        # f32: the coordinate x*W-0.5 carries ~|xW|*2^-24 rounding (fma vs mul+sub), scaled
        # by the channel sums -> tolerance relative to the gradient magnitude
        for got, exp in ((vd.grad, vr.grad), (wd.grad, wr.grad)):
            e = exp.numpy()
            np.testing.assert_allclose(got.cpu().numpy(), e, atol=2e-5 * max(1.0, float(np.abs(e).max())), rtol=0)
    else:
        gvr = vr.grad
        err = (vd.grad.float().cpu() - gvr).abs()
        assert bool((err <= gvr.abs() * 2 ** -8 + 1e-4).all()), float(err.max())
        # grad_loc / grad_attn of the production bf16 kernel vs the oracle (bf16 value and
        # grad_out are exact in f32; f32 sums in another order + fma'd coordinates)
        _check_geo_vs_oracle(ld.grad.cpu(), lr.grad, wd.grad.cpu(), wr.grad)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C", [96, 256, 768])
def test_add_layer_norm_colsum_feeds_linear_bias(monkeypatch, dtype, C):
    """The LayerNorm backward's fused column sums of dx (vs_layer_norm_backward_ex) become
    the bias gradient of the TokenLinear whose output is the residual branch r (no
    column_sum launch), and equal autograd's sum of dL/dr (f64 reference); an in-place
    update of the gradient afterwards invalidates them (version check)."""
    from visionseg.linear import TokenLinear
    ops = _ops()
    calls = []
    real = ops.column_sum
    monkeypatch.setattr(ops, "column_sum", lambda t: calls.append(t.shape) or real(t))
    g = torch.Generator(device="cuda").manual_seed(C)
    M, Ci = 20000, 64
    lin = TokenLinear(Ci, C).to(DEV, dtype)
    w = (1 + 0.1 * torch.randn(C, device=DEV, generator=g)).to(dtype).requires_grad_(True)
    b = (0.1 * torch.randn(C, device=DEV, generator=g)).to(dtype).requires_grad_(True)
    x = torch.randn(M, C, device=DEV, generator=g).to(dtype).requires_grad_(True)
    h = torch.randn(M, Ci, device=DEV, generator=g).to(dtype)
    gy = torch.randn(M, C, device=DEV, generator=g).to(dtype)
    gs = torch.randn(M, C, device=DEV, generator=g).to(dtype)
    r = lin(h)
    s, y = ops.add_layer_norm(x, r, w, b)
    torch.autograd.backward([y, s], [gy, gs])
    assert not calls, calls                                   # bias gradient came from the LN pass
    # reference: dL/dr = dL/d(x + r) from an f64 torch LayerNorm
    xs = (x.detach().double() + r.detach().double()).requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xs, (C,), w.detach().double(), b.detach().double(), 1e-5)
    torch.autograd.backward([yr, xs], [gy.double(), gs.double()])
    exp = xs.grad.sum(0)
    tol = 1e-4 if dtype == torch.float32 else 2 ** -6
    rel = float((lin.bias.grad.double() - exp).abs().max() / exp.abs().max())
    assert rel <= tol, rel
    # a modified gradient must not reuse the recorded sums
    gx = torch.randn(M, C, device=DEV, generator=g).to(dtype)
    ops.attach_colsum(gx, torch.zeros(C, device=DEV, dtype=dtype))
    assert ops.take_colsum(gx) is not None
    gx.add_(1)
    assert ops.take_colsum(gx) is None


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("K", [40000, 70756])
def test_token_linear_split_k_grads(dtype, K):
    """Split-K weight gradient (visionseg.linear) vs an f64 reference of dY^T X; the
    K remainder (K not a multiple of the chunk) is covered by 70756 = 69*1025 + 1031."""
    from visionseg.linear import TokenLinear, split_count
    g = torch.Generator(device="cuda").manual_seed(0)
    lin = TokenLinear(192, 576).to(DEV, dtype)
    x = torch.randn(2, K // 2, 192, device=DEV, generator=g).to(dtype).requires_grad_(True)
    gy = torch.randn(2, K // 2, 576, device=DEV, generator=g).to(dtype)
    assert split_count(K, 576, 192) > 1
    y = lin(x)
    np.testing.assert_array_equal(y.detach().float().cpu(), torch.nn.functional.linear(x, lin.weight, lin.bias).detach().float().cpu())
    y.backward(gy)
    x2, gy2 = x.detach().double().reshape(-1, 192), gy.double().reshape(-1, 576)
    ew, eb, ex = gy2.t() @ x2, gy2.sum(0), gy2 @ lin.weight.detach().double()
    tol = 1e-5 if dtype == torch.float32 else 8e-3
    for got, exp in ((lin.weight.grad, ew), (lin.bias.grad, eb), (x.grad.reshape(-1, 192), ex)):
        rel = float((got.double() - exp).abs().max() / exp.abs().max())
        assert rel <= tol, rel


# grad_loc / grad_attn of the bf16 MSDA backward vs the oracle.  value and grad_out are
# bf16 (exact in f32), so the products are the oracle's; what differs is the f32
# summation order over 32 channels x 4 corners and the coordinate x*W-0.5 (one fma on the
# GPU, mul + sub in grid_sample), which can put a tap that sits within an ulp of a cell
# edge into the neighbouring cell: grad_loc jumps there (d bilinear / d loc is
# discontinuous at cell edges).  Bound: every element within 1e-4 of the tensor's max
# |value| + 2^-8 relative, except at most 1e-4 of the grad_loc entries (edge taps)
# which must still be within 5e-2 of the max.
GEO_ATOL, GEO_RTOL, EDGE_FRAC, EDGE_ATOL = 1e-4, 2 ** -8, 1e-4, 5e-2


def _check_geo_vs_oracle(gl, gl_ref, gw, gw_ref):
    out = []
    for name, got, exp, edges in (("grad_loc", gl, gl_ref, True), ("grad_attn", gw, gw_ref, False)):
        sc = max(float(exp.abs().max()), 1e-12)
        err = (got.float() - exp).abs()
        bad = err > GEO_ATOL * sc + GEO_RTOL * exp.abs()
        nbad = int(bad.sum())
        out.append(f"{name} max|err|/max {float(err.max()) / sc:.2e} ({nbad} of {err.numel()} beyond tol)")
        if edges:
            assert nbad <= EDGE_FRAC * err.numel(), out[-1]
            assert float(err.max()) <= EDGE_ATOL * sc, out[-1]
        else:
            assert nbad == 0, out[-1]
    print("; ".join(out))


def _encoder_like_inputs(B, shapes, H, P, seed, jitter):
    """Queries = every pixel of every level (encoder self-attention), sampling points =
    reference point + a smooth per-head offset field + `jitter` (pixels) of noise."""
    g = torch.Generator().manual_seed(seed)
    S = sum(h * w for h, w in shapes)
    L = len(shapes)
    ref = R.reference_points(shapes, B)                                 # [B,S,L,2]
    base = torch.randn(1, 1, H, L, P, 2, generator=g) * 2.0             # pixels, shared by all queries
    ramp = torch.linspace(0, 1.5, S)[None, :, None, None, None, None]   # slow drift along the query order
    off = base + ramp * torch.randn(1, 1, H, L, P, 2, generator=g) + jitter * torch.randn(B, S, H, L, P, 2, generator=g)
    norm = torch.tensor([[w, h] for h, w in shapes], dtype=torch.float32)[None, None, None, :, None, :]
    loc = ref[:, :, None, :, None, :] + off / norm
    value = torch.randn(B, S, H, 32, generator=g)
    w = torch.softmax(torch.randn(B, S, H, L * P, generator=g), -1).view(B, S, H, L, P)
    return value, loc, w


@pytest.mark.parametrize("run,win", [("16", "tile"), ("0", "0"), ("16", "sub"), ("16", "tile-1024"),
                                     ("16", "tile-odd")])
@pytest.mark.parametrize("jitter", [0.0, 0.3, 3.0])
def test_msda_carry_backward_vs_oracle(monkeypatch, run, win, jitter):
    """Atomic-scatter grad_value on encoder-shaped queries vs the oracle, f32: the binned
    query-tile kernel (csrc/msda.hip msda_bwd_binned_kernel; 4x4 grid tiles "tile", also
    at the 1024^2 level shapes and on odd level sizes with partial tiles, or runs of 16
    queries for a query subset "sub") and the single fused kernel (VS_MSDA_RUN=0)."""
    monkeypatch.setenv("VS_MSDA_RUN", run)
    ops = _ops()
    monkeypatch.setattr(ops, "_MSDA_BWD", "carry")
    shapes, B, H = [(8, 8), (16, 16), (32, 32)], 2, 4
    if win == "tile-1024":
        shapes, B, H = [(32, 32), (64, 64), (128, 128)], 1, 8
    elif win.endswith("-odd"):
        shapes = [(9, 13), (18, 26), (35, 51)]
    value, loc, w = _encoder_like_inputs(B, shapes, H, 4, seed=11, jitter=jitter)
    if win == "sub":                                   # Q != S: windows over runs of 16 queries
        idx = torch.randperm(loc.shape[1], generator=torch.Generator().manual_seed(5))[:700].sort().values
        loc, w = loc[:, idx].contiguous(), w[:, idx].contiguous()
    vr, lr, wr = (t.clone().requires_grad_(True) for t in (value, loc, w))
    ref = R.msda_ref(vr, shapes, lr, wr)
    go = torch.randn(ref.shape, generator=torch.Generator().manual_seed(3))
    ref.backward(go)
    vd, ld, wd = (t.to(DEV).requires_grad_(True) for t in (value, loc, w))
    out = ops.ms_deform_attn(vd, shapes, ld, wd)
    out.backward(go.to(DEV))
    np.testing.assert_allclose(vd.grad.cpu().numpy(), vr.grad.numpy(), atol=2e-5, rtol=0)
    # grad_attn / grad_loc: fp32 dots of 32 channels whose interpolation weights differ by
    # an ulp of the unnormalised coordinate (fma on the GPU) -- relative to their scale
    gw = wr.grad.numpy()
    np.testing.assert_allclose(wd.grad.cpu().numpy(), gw, atol=2e-5 * max(1.0, np.abs(gw).max()), rtol=0)
    gl = lr.grad.numpy()
    np.testing.assert_allclose(ld.grad.cpu().numpy(), gl, atol=2e-5 * max(1.0, np.abs(gl).max()), rtol=0)


@pytest.mark.parametrize("win", ["tile", "tile-1024", "tile-odd", "sub", "4lvl", "ragged", "wide"])
@pytest.mark.parametrize("jitter", [0.0, 0.3, 3.0, 12.0])
def test_msda_mfma_backward_vs_binned_and_oracle(monkeypatch, win, jitter):
    """bf16 grad_value + grad_loc / grad_attn of the MFMA backward kernels vs (a) the binned
    kernel on the same inputs (VS_MSDA_MFMA=0; all sum in f32: within two bf16 ulps) and (b)
    the oracle (bf16 output rounding: 2^-8 relative + 1e-4):
      * "col": msda_bwd_col_kernel, pyramid columns of 8 x 16 finest-level queries
        (3 chunks of 64), one flush per (band, cell) per column; "col16": 16 x 16 (6 chunks);
      * "tile" / "tile_s": msda_bwd_mfma_wg_kernel (VS_MSDA_COL=0), 8 x 8 query tiles, on its
        two band skeletons (VS_MSDA_SKEL 0 / 2), and "tile_sep" with the separate grad_loc
        gather kernel (VS_MSDA_GEOM=0).
    jitter 12 px drives boxes past the 128-cell band cap; "sub" runs 16 consecutive queries
    of a query subset (Q != S: the column kernel does not apply), "4lvl" four levels stored
    finest first, "ragged" a 2x pyramid whose finest level is not a multiple of the blocks,
    "wide" a finest level 150 cells wide with far taps (boxes wider than the band cap: bands
    split along x too)."""
    ops = _ops()
    monkeypatch.setattr(ops, "_MSDA_BWD", "carry")
    monkeypatch.setenv("VS_MSDA_RUN", "16")            # the split kernels at every size
    shapes, B, H = [(8, 8), (16, 16), (32, 32)], 2, 4
    if win == "tile-1024":
        shapes, B, H = [(32, 32), (64, 64), (128, 128)], 1, 8
    elif win == "tile-odd":
        shapes = [(9, 13), (18, 26), (35, 51)]
    elif win == "4lvl":
        shapes = [(48, 80), (24, 40), (12, 20), (6, 10)]
    elif win == "ragged":                              # partial border tiles
        shapes = [(5, 3), (10, 6), (20, 12)]
    elif win == "wide":
        shapes, jitter = [(10, 38), (20, 75), (40, 150)], jitter * 4 + 20
    value, loc, w = _encoder_like_inputs(B, shapes, H, 4, seed=13, jitter=jitter)
    if win == "sub":
        idx = torch.randperm(loc.shape[1], generator=torch.Generator().manual_seed(5))[:700].sort().values
        loc, w = loc[:, idx].contiguous(), w[:, idx].contiguous()
    value = value.to(torch.bfloat16)
    vr, lr, wr = value.float().clone().requires_grad_(True), loc.clone().requires_grad_(True), w.clone().requires_grad_(True)
    ref = R.msda_ref(vr, shapes, lr, wr)
    go = torch.randn(ref.shape, generator=torch.Generator().manual_seed(3)).to(torch.bfloat16)
    ref.backward(go.float())
    grads, geo = {}, {}
    variants = {
        "tile_sep": dict(VS_MSDA_MFMA="1", VS_MSDA_GEOM="0", VS_MSDA_SKEL="0", VS_MSDA_COL="0"),
        "binned": dict(VS_MSDA_MFMA="0", VS_MSDA_GEOM="0", VS_MSDA_SKEL="0", VS_MSDA_COL="0"),
        "tile": dict(VS_MSDA_MFMA="1", VS_MSDA_GEOM="1", VS_MSDA_SKEL="0", VS_MSDA_COL="0"),
        "tile_s": dict(VS_MSDA_MFMA="1", VS_MSDA_GEOM="1", VS_MSDA_SKEL="2", VS_MSDA_COL="0"),
        "col": dict(VS_MSDA_MFMA="1", VS_MSDA_GEOM="1", VS_MSDA_SKEL="2", VS_MSDA_COL="8x16"),
        "col16": dict(VS_MSDA_MFMA="1", VS_MSDA_GEOM="1", VS_MSDA_SKEL="2", VS_MSDA_COL="16x16"),
    }
    for name, env in variants.items():
        for k, v in env.items():
            if v is None:
                monkeypatch.delenv(k, raising=False)
            else:
                monkeypatch.setenv(k, v)
        vd = value.to(DEV).requires_grad_(True)
        ld, wd = loc.to(DEV).requires_grad_(True), w.to(DEV).requires_grad_(True)
        out = ops.ms_deform_attn(vd, shapes, ld, wd)
        out.backward(go.to(DEV))
        grads[name] = vd.grad.float().cpu()
        geo[name] = (ld.grad.cpu(), wd.grad.cpu())
    # grad_loc / grad_attn fused into the band walk vs the separate gather kernel: the same
    # bf16 x bf16 products summed in f32 in another order
    for name in ("tile", "col", "col16"):
        for a, b in zip(geo[name], geo["tile_sep"]):
            sc = float(b.abs().max())
            assert float((a - b).abs().max()) <= 1e-4 * sc, (name, float((a - b).abs().max()) / sc)
        # and vs the oracle (f32 value, bf16-rounded inputs)
        _check_geo_vs_oracle(geo[name][0], lr.grad, geo[name][1], wr.grad)
    # the two band skeletons of the tile kernel walk the same bands in the same order:
    # grad_loc / grad_attn bit-identical; grad_value differs only by the order of its atomics
    for a, b in zip(geo["tile_s"], geo["tile"]):
        assert torch.equal(a, b), float((a - b).abs().max())
    scale = float(vr.grad.abs().max())
    for name, gv in grads.items():
        err = (gv - vr.grad).abs()
        bad = err > vr.grad.abs() * 2 ** -8 + 1e-4
        assert not bool(bad.any()), (name, float(err.max()), int(bad.sum()), float(vr.grad[bad][0]),
                                     float(gv[bad][0]))
    for name in ("tile", "tile_s", "col", "col16"):
        d = (grads[name] - grads["binned"]).abs()
        # all f32 sums, rounded to bf16 once: within two bf16 ulps, plus f32 summation-order
        # noise (~1e-7 of the summed magnitudes) where contributions cancel to ~0
        assert bool((d <= grads["binned"].abs() * 2 ** -6 + 3e-5 * scale).all()), (name, float(d.max()))


@pytest.mark.parametrize("shapes", [[(32, 32), (64, 64), (128, 128)], [(9, 13), (18, 26), (35, 51)],
                                    [(5, 3), (10, 6), (20, 12)], [(48, 80), (24, 40), (12, 20), (6, 10)],
                                    [(64, 64), (32, 32)]])
def test_msda_forward_column_order_equals_query_order(monkeypatch, shapes):
    """The bf16 forward visits encoder queries (Q == S) in pyramid-column order (msda_fwd4_kernel
    COL): every query is computed exactly as in query order (VS_MSDA_FWD_COL=0) -- bit-equal
    outputs, so no query is skipped or computed twice -- on 2x pyramids, odd and ragged level
    sizes (border columns with padding slots), 4 levels stored finest first, and 2 levels."""
    ops = _ops()
    B, H = 2, 8
    value, loc, w = _encoder_like_inputs(B, shapes, H, 4, seed=7, jitter=1.5)
    value = value.to(torch.bfloat16).to(DEV)
    loc, w = loc.to(DEV), w.to(DEV)
    res = {}
    for col in ("1", "0"):
        monkeypatch.setenv("VS_MSDA_FWD_COL", col)
        with torch.no_grad():
            res[col] = ops.ms_deform_attn(value, shapes, loc, w).float().cpu()
    assert torch.equal(res["1"], res["0"])
    ref = R.msda_ref(value.float().cpu(), shapes, loc.cpu(), w.cpu())
    err = (res["1"] - ref).abs()
    assert bool((err <= ref.abs() * 2 ** -8 + 1e-4).all()), float(err.max())


@pytest.mark.parametrize("wscale", [1.0, 3.0, 40.0])
def test_msda_col_backward_unnormalised_weights(monkeypatch, wscale):
    """The column kernel's fixed-point W build with attention weights that are NOT
    softmax-normalised (the op, like upstream MSDeformAttnFunction, accepts any): per query
    and level sum_p |aw_p| up to ~wscale * 2.  The quantum follows that bound (2^-30 while it
    is <= 1, coarser beyond), so grad_value stays within bf16 rounding of the oracle and of
    the f32 W build (VS_MSDA_WINT=0); a fixed 2^-30 wrapped int32 from a bound of 2 on
    (round-5 ADVICE)."""
    ops = _ops()
    monkeypatch.setattr(ops, "_MSDA_BWD", "carry")
    monkeypatch.setenv("VS_MSDA_RUN", "16")
    monkeypatch.setenv("VS_MSDA_COL", "8x16")
    shapes, B, H = [(16, 16), (32, 32), (64, 64)], 1, 4
    value, loc, w = _encoder_like_inputs(B, shapes, H, 4, seed=21, jitter=0.3)
    g = torch.Generator().manual_seed(4)
    w = (torch.rand(w.shape, generator=g) * 2 - 0.5) * wscale                  # signed, unnormalised
    value = value.to(torch.bfloat16)
    vr, lr, wr = value.float().clone().requires_grad_(True), loc.clone().requires_grad_(True), w.clone().requires_grad_(True)
    ref = R.msda_ref(vr, shapes, lr, wr)
    go = torch.randn(ref.shape, generator=torch.Generator().manual_seed(3)).to(torch.bfloat16)
    ref.backward(go.float())
    res = {}
    for wint in ("1", "0"):
        monkeypatch.setenv("VS_MSDA_WINT", wint)
        vd = value.to(DEV).requires_grad_(True)
        ld, wd = loc.to(DEV).requires_grad_(True), w.to(DEV).requires_grad_(True)
        out = ops.ms_deform_attn(vd, shapes, ld, wd)
        out.backward(go.to(DEV))
        res[wint] = vd.grad.float().cpu()
        assert bool(torch.isfinite(res[wint]).all())
    scale = float(vr.grad.abs().max())
    for wint, gv in res.items():
        err = (gv - vr.grad).abs()
        assert bool((err <= vr.grad.abs() * 2 ** -7 + 1e-4 * scale).all()), (wint, float(err.max()), scale)
    d = (res["1"] - res["0"]).abs()
    assert bool((d <= res["0"].abs() * 2 ** -6 + 3e-5 * scale).all()), float(d.max())


@pytest.mark.parametrize("case", [
    dict(B=2, shapes=[(8, 8), (16, 16), (32, 32)], H=4, jitter=0.0, Q=None),
    dict(B=2, shapes=[(8, 8), (16, 16), (32, 32)], H=4, jitter=3.0, Q=None),
    dict(B=1, shapes=[(32, 32), (64, 64), (128, 128)], H=8, jitter=0.3, Q=None),     # 1024^2 encoder, one image
    dict(B=1, shapes=[(16, 16), (32, 32), (64, 64)], H=8, jitter=12.0, Q=None),      # far taps, many off-grid
    dict(B=2, shapes=[(12, 20), (24, 40), (48, 80), (6, 10)], H=8, jitter=1.0, Q=300),  # decoder-like, 4 levels
    dict(B=1, shapes=[(5, 7)], H=2, jitter=1.0, Q=0),                                  # no queries
])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("mode", ["tiled"])
def test_msda_destination_backward_vs_oracle(monkeypatch, case, dtype, mode):
    """Deterministic backward: grad_value by destination tiles owned by one wave
    (vs_msda_backward_tiled, VS_MSDA_BWD=tiled; no float atomics) vs the oracle; bf16:
    grad_value is produced in bf16 from f32 sums."""
    ops = _ops()
    monkeypatch.setattr(ops, "_MSDA_BWD", mode)
    shapes, B, H = case["shapes"], case["B"], case["H"]
    value, loc, w = _encoder_like_inputs(B, shapes, H, 4, seed=21, jitter=case["jitter"])
    if case["Q"] is not None:
        g = torch.Generator().manual_seed(4)
        idx = torch.randint(0, loc.shape[1], (case["Q"],), generator=g)
        loc, w = loc[:, idx].contiguous(), w[:, idx].contiguous()
    value = value.to(dtype)
    vr, lr, wr = value.float().clone().requires_grad_(True), loc.clone().requires_grad_(True), w.clone().requires_grad_(True)
    ref = R.msda_ref(vr, shapes, lr, wr)
    go = torch.randn(ref.shape, generator=torch.Generator().manual_seed(8)).to(dtype)
    ref.backward(go.float())
    vd, ld, wd = value.to(DEV).requires_grad_(True), loc.to(DEV).requires_grad_(True), w.to(DEV).requires_grad_(True)
    out = ops.ms_deform_attn(vd, shapes, ld, wd)
    out.backward(go.to(DEV))
    assert vd.grad.dtype == dtype
    if dtype == torch.float32:
        np.testing.assert_allclose(vd.grad.cpu().numpy(), vr.grad.numpy(), atol=2e-5, rtol=0)
    else:
        err = (vd.grad.float().cpu() - vr.grad).abs()
        assert bool((err <= vr.grad.abs() * 2 ** -8 + 1e-4).all()), float(err.max())
    if loc.shape[1] and dtype == torch.float32:
        e = wr.grad.numpy()
        np.testing.assert_allclose(wd.grad.cpu().numpy(), e, atol=2e-5 * max(1.0, np.abs(e).max()), rtol=0)
        gl = lr.grad.numpy()
        np.testing.assert_allclose(ld.grad.cpu().numpy(), gl, atol=2e-5 * max(1.0, np.abs(gl).max()), rtol=0)
    elif loc.shape[1]:
        _check_geo_vs_oracle(ld.grad.cpu(), lr.grad, wd.grad.cpu(), wr.grad)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,C", [(1, 96), (1000, 96), (4099, 192), (777, 256), (2048, 384), (513, 768), (65, 1536),
                                 (33, 2048), (0, 96)])
def test_layer_norm_vs_torch(dtype, M, C):
    """HIP LayerNorm (csrc/norm.hip) forward + backward vs torch f64 on the same inputs."""
    ops = _ops()
    g = torch.Generator().manual_seed(M * 7 + C)
    x = (torch.randn(M, C, generator=g) * 3 + 0.5).to(dtype)
    w = (1 + 0.1 * torch.randn(C, generator=g)).to(dtype)
    b = (0.1 * torch.randn(C, generator=g)).to(dtype)
    gy = torch.randn(M, C, generator=g).to(dtype)
    xr, wr, br = (t.double().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (C,), wr, br, 1e-5)
    yr.backward(gy.double())
    xd, wd, bd = (t.to(DEV).requires_grad_(True) for t in (x, w, b))
    y = ops.layer_norm(xd, wd, bd, 1e-5)
    assert y.dtype == dtype
    y.backward(gy.to(DEV))
    tol = 2e-5 if dtype == torch.float32 else 2 ** -7
    for got, exp in ((y, yr), (xd.grad, xr.grad)):
        err = (got.detach().double().cpu() - exp.detach()).abs()
        assert float(err.max() if err.numel() else 0) <= tol * max(1.0, float(exp.detach().abs().max() if exp.numel() else 1))
    for got, exp in ((wd.grad, wr.grad), (bd.grad, br.grad)):
        err = float((got.double().cpu() - exp).abs().max())
        assert err <= (1e-4 if dtype == torch.float32 else 2 ** -7) * max(1.0, float(exp.abs().max())), err


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,C", [(1000, 96), (4099, 192), (2048, 384), (65, 768), (0, 96)])
@pytest.mark.parametrize("use_s", [True, False])
def test_add_layer_norm_vs_torch(dtype, M, C, use_s):
    """Fused residual add + LayerNorm (ops.add_layer_norm, csrc/norm.hip RES / ADD
    variants): s = x + r (rounded to dtype) and y = LN(s) vs torch f64 on the rounded s;
    gradients of x and r = LN backward + the gradient of s (when s is used downstream)."""
    ops = _ops()
    g = torch.Generator().manual_seed(M * 11 + C)
    x = (torch.randn(M, C, generator=g) * 3 + 0.5).to(dtype)
    r = torch.randn(M, C, generator=g).to(dtype)
    w = (1 + 0.1 * torch.randn(C, generator=g)).to(dtype)
    b = (0.1 * torch.randn(C, generator=g)).to(dtype)
    gy = torch.randn(M, C, generator=g).to(dtype)
    gs = torch.randn(M, C, generator=g).to(dtype)
    s_ref = (x.float() + r.float()).to(dtype)
    sr, wr, br = (t.double().requires_grad_(True) for t in (s_ref, w, b))
    yr = torch.nn.functional.layer_norm(sr, (C,), wr, br, 1e-5)
    yr.backward(gy.double())
    gx_exp = sr.grad + (gs.double() if use_s else 0)
    xd, rd, wd, bd = (t.to(DEV).requires_grad_(True) for t in (x, r, w, b))
    s, y = ops.add_layer_norm(xd, rd, wd, bd, 1e-5)
    assert torch.equal(s.detach().cpu(), s_ref)
    loss = (y * gy.to(DEV)).sum() + ((s * gs.to(DEV)).sum() if use_s else 0)
    loss.backward()
    tol = 2e-5 if dtype == torch.float32 else 2 ** -7
    for got, exp in ((y, yr), (xd.grad, gx_exp), (rd.grad, gx_exp)):
        err = (got.detach().double().cpu() - exp.detach()).abs()
        assert float(err.max() if err.numel() else 0) <= tol * max(1.0, float(exp.detach().abs().max() if exp.numel() else 1))
    for got, exp in ((wd.grad, wr.grad), (bd.grad, br.grad)):
        err = float((got.double().cpu() - exp).abs().max())
        assert err <= (1e-4 if dtype == torch.float32 else 2 ** -7) * max(1.0, float(exp.abs().max())), err


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N", [(262144, 96), (86016, 256), (5, 384), (0, 64), (1023, 2048), (4099, 3072),
                                 (1500, 6144), (77, 2056)])
def test_column_sum_vs_torch(dtype, M, N):
    ops = _ops()
    x = torch.randn(M, N, generator=torch.Generator().manual_seed(N)).to(dtype)
    exp = x.double().sum(0)
    got = ops.column_sum(x.to(DEV)).double().cpu()
    tol = 1e-5 if dtype == torch.float32 else 2 ** -8
    assert float((got - exp).abs().max()) <= tol * max(1.0, float(exp.abs().max())) + 1e-3 * (M ** 0.5) * (dtype != torch.float32)


@pytest.mark.parametrize("shift", [0, 3])
@pytest.mark.parametrize("heads,nWh,nWw", [(3, 4, 4), (6, 3, 5), (12, 2, 2)])
@pytest.mark.parametrize("kernel", ["mfma", "scalar"])
def test_window_attention_bf16_fwd_bwd_vs_oracle(monkeypatch, shift, heads, nWh, nWw, kernel):
    """bf16 window attention forward + backward (MFMA path for ws=7, and the scalar path
    via VS_WIN_ATTN_SCALAR=1) vs the f32 oracle on the same bf16-rounded inputs."""
    if kernel == "scalar":
        monkeypatch.setenv("VS_WIN_ATTN_SCALAR", "1")
    ops = _ops()
    B, ws = 2, 7
    Bw, N, C = B * nWh * nWw, ws * ws, heads * 32
    g = torch.Generator().manual_seed(heads * 10 + shift)
    qkv = torch.randn(Bw, N, 3 * C, generator=g).to(torch.bfloat16)
    table = torch.randn((2 * ws - 1) ** 2, heads, generator=g)
    qr, tr = qkv.float().requires_grad_(True), table.clone().requires_grad_(True)
    ref = _win_attn_ref(qr, tr, heads, ws, shift, nWh, nWw)
    go = torch.randn(ref.shape, generator=g).to(torch.bfloat16)
    ref.backward(go.float())
    qd, td = qkv.to(DEV).requires_grad_(True), table.to(DEV).requires_grad_(True)
    out = ops.window_attention(qd, td, heads, ws, shift, nWh, nWw)
    err = (out.float().cpu() - ref.detach()).abs()
    assert bool((err <= ref.detach().abs() * 2 ** -7 + 4e-3).all()), float(err.max())
    out.backward(go.to(DEV))
    for got, exp in ((qd.grad, qr.grad), (td.grad, tr.grad)):
        e = float((got.float().cpu() - exp).abs().max())
        assert e <= 2e-2 * float(exp.abs().max()), (e, float(exp.abs().max()))


@pytest.mark.parametrize("ws,shift,heads,nWh,nWw", [(12, 0, 4, 2, 3), (12, 6, 4, 3, 3), (12, 6, 8, 2, 2),
                                                    (9, 4, 2, 2, 2), (10, 5, 3, 3, 2), (11, 0, 1, 2, 2)])
def test_window_attention_bf16_large_windows_vs_oracle(ws, shift, heads, nWh, nWw):
    """bf16 MFMA window attention for 64 < N <= 160 (Swin-B/L ws 12: N = 144; one wave per
    32-query tile, csrc/window_attn.hip win_attn_*_mfma_big) vs the f32 oracle on the same
    bf16-rounded inputs; tolerances as the N <= 64 path."""
    ops = _ops()
    B = 2
    Bw, N, C = B * nWh * nWw, ws * ws, heads * 32
    g = torch.Generator().manual_seed(ws * 100 + shift * 10 + heads)
    qkv = torch.randn(Bw, N, 3 * C, generator=g).to(torch.bfloat16)
    table = torch.randn((2 * ws - 1) ** 2, heads, generator=g)
    qr, tr = qkv.float().requires_grad_(True), table.clone().requires_grad_(True)
    ref = _win_attn_ref(qr, tr, heads, ws, shift, nWh, nWw)
    go = torch.randn(ref.shape, generator=g).to(torch.bfloat16)
    ref.backward(go.float())
    qd, td = qkv.to(DEV).requires_grad_(True), table.to(DEV).requires_grad_(True)
    out = ops.window_attention(qd, td, heads, ws, shift, nWh, nWw)
    err = (out.float().cpu() - ref.detach()).abs()
    assert bool((err <= ref.detach().abs() * 2 ** -7 + 4e-3).all()), float(err.max())
    out.backward(go.to(DEV))
    gq, gr = qd.grad.float().cpu().view(Bw, N, 3, C), qr.grad.view(Bw, N, 3, C)
    for part in range(3):      # q, k, v gradients separately (each scaled to its own range)
        e = float((gq[:, :, part] - gr[:, :, part]).abs().max())
        assert e <= 2e-2 * float(gr[:, :, part].abs().max()), (part, e)
    e = float((td.grad.cpu() - tr.grad).abs().max())
    assert e <= 2e-2 * float(tr.grad.abs().max()), e


@pytest.mark.parametrize("P,H,T", [(5476, 3, 169), (400, 12, 169), (1444, 6, 169), (7, 3, 169), (13, 4, 529),
                                   (64, 8, 529), (100, 48, 529), (9, 2, 8)])
def test_window_table_grad_partial_sum(P, H, T):
    """The relative-position-table gradient: per-window f32 partials summed by the column-sum
    kernel (8 partial rows folded into one when heads * T % 8 != 0, remainder rows added)
    against an f64 sum of the same partials; one f32 rounding per partial bounds the error."""
    ops = _ops()
    g = torch.Generator().manual_seed(P * 7 + H)
    part = torch.randn(P, H, T, generator=g)
    ref = part.double().sum(0)
    got = ops.table_grad_from_partials(part.to(DEV)).double().cpu()
    assert got.shape == (H, T)
    bound = P * 2.0 ** -23 * part.double().abs().sum(0) + 1e-30
    assert bool(((got - ref).abs() <= bound).all()), float((got - ref).abs().max())


@pytest.mark.parametrize("P,H,T", [(5476, 3, 169), (400, 12, 169), (1444, 6, 169), (100, 24, 169), (7, 3, 169),
                                   (13, 4, 529), (64, 8, 529), (100, 48, 529), (9, 2, 8), (12, 1, 3)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_rel_table_grad_fold(P, H, T, dtype):
    """ops.rel_table_grad: the partials folded to a multiple-of-8 width, column-summed, folded
    back, transposed to the table's [T, heads] layout and cast (vs_rel_table_grad; the 4-5
    launch composition where P does not fold) vs an f64 sum: one f32 rounding per partial,
    then the output dtype's rounding."""
    ops = _ops()
    g = torch.Generator().manual_seed(P * 5 + H)
    part = torch.randn(P, H, T, generator=g)
    ref = part.double().sum(0).t()
    got = ops.rel_table_grad(part.to(DEV), dtype)
    assert got.shape == (T, H) and got.dtype == dtype
    got = got.double().cpu()
    bound = P * 2.0 ** -23 * part.double().abs().sum(0).t() + (2.0 ** -8 * ref.abs() if dtype == torch.bfloat16 else 0)
    assert bool(((got - ref).abs() <= bound + 1e-30).all()), float((got - ref).abs().max())


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("ws,shift,heads,nWh,nWw,amp", [(12, 6, 4, 3, 3, 1.0), (7, 3, 3, 4, 4, 1.0), (12, 0, 2, 2, 2, 12.0),
                                                        (10, 5, 3, 3, 2, 1.0), (12, 6, 6, 4, 4, 0.0)])
def test_window_attention_bwd_fixed_point_bins_equal_f32_bins(monkeypatch, fp8, ws, shift, heads, nWh, nWw, amp):
    """The round-5 backward (win_attn_bwd_fb: natural-layout staging + transposed LDS reads,
    the bias gradient in fixed-point integer bins) against the round-4 one (f32 bins): the
    q / k / v gradients are the same products in the same order (bit-equal), the table
    gradient agrees to the fixed-point quantum.  amp scales q / k (peaked softmax, large dS)
    and 0 makes V and the gradient all-zero rows (the bound is 0)."""
    ops = _ops()
    if fp8 and ws * ws > 160:
        pytest.skip("fp8 path: N <= 160")
    B = 2
    Bw, N, C = B * nWh * nWw, ws * ws, heads * 32
    g = torch.Generator().manual_seed(ws * 7 + heads)
    qkv = torch.randn(Bw, N, 3, C, generator=g)
    qkv[:, :, :2] *= max(amp, 1.0)
    if amp == 0.0:
        qkv[:, :, 2] = 0
    qkv = qkv.view(Bw, N, 3 * C).to(torch.bfloat16)
    table = torch.randn((2 * ws - 1) ** 2, heads, generator=g)
    go = torch.randn(Bw, N, C, generator=g).to(torch.bfloat16)
    if amp == 0.0:
        go.zero_()
    res = []
    for fb in ("0", "2"):                     # 2: the round-5 kernel for every N and fp8 too
        monkeypatch.setenv("VS_WIN_BWD_FB", fb)
        qd, td = qkv.to(DEV).requires_grad_(True), table.to(DEV).requires_grad_(True)
        out = ops.window_attention(qd, td, heads, ws, shift, nWh, nWw, fp8=fp8)
        out.backward(go.to(DEV))
        torch.cuda.synchronize()
        res.append((qd.grad.float().cpu(), td.grad.double().cpu()))
    (gq0, gt0), (gq1, gt1) = res
    assert torch.equal(gq0, gq1), float((gq0 - gq1).abs().max())
    assert bool(torch.isfinite(gt1).all())
    e = float((gt0 - gt1).abs().max())
    assert e <= 1e-5 * max(float(gt0.abs().max()), 1e-30), (e, float(gt0.abs().max()))


@pytest.mark.parametrize("kernel", ["mfma", "mfma-4blk", "scalar"])
@pytest.mark.parametrize("B,Q,S", [(2, 100, 4096), (1, 100, 1000), (2, 7, 300), (1, 128, 16384), (1, 130, 512)])
def test_masked_attention_bf16_fwd_bwd_vs_oracle(monkeypatch, kernel, B, Q, S):
    """bf16 masked cross-attention forward + backward (MFMA kernels, and the scalar ones
    via VS_XATTN_SCALAR=1) vs the f32 oracle on the same bf16-rounded inputs: ragged key
    counts, fully blocked rows (unblocked by the producer's rule), Q > 128 (scalar bwd);
    "mfma-4blk": four 128-key blocks per backward workgroup (dQ partial accumulated over
    the blocks, chunks that end past S), as the C2 decoder's 128^2 level runs."""
    if kernel == "scalar":
        monkeypatch.setenv("VS_XATTN_SCALAR", "1")
    elif kernel == "mfma-4blk":
        monkeypatch.setenv("VS_XATTN_BLOCKS", "4")
    ops = _ops()
    heads = 8
    q, k, v, blocked, words = _xattn_case(B, Q, S, heads, seed=Q + S, dtype=torch.bfloat16)
    C = heads * 32
    qr, kr, vr = (t.float().requires_grad_(True) for t in (q, k, v))
    ref = R.masked_attention_ref(qr.view(B, Q, heads, 32).transpose(1, 2), kr.view(B, S, heads, 32).transpose(1, 2),
                                 vr.view(B, S, heads, 32).transpose(1, 2), blocked)
    go = torch.randn(ref.shape, generator=torch.Generator().manual_seed(5)).to(torch.bfloat16)
    ref.backward(go.float())
    qd, kd, vd = (t.to(DEV).requires_grad_(True) for t in (q, k, v))
    out = ops.masked_attention(qd, kd, vd, words.to(DEV), heads)
    err = (out.float().cpu() - ref.detach()).abs()
    assert bool((err <= ref.detach().abs() * 2 ** -7 + 4e-3).all()), float(err.max())
    out.backward(go.to(DEV))
    for got, exp in ((qd.grad, qr.grad), (kd.grad, kr.grad), (vd.grad, vr.grad)):
        e = float((got.float().cpu() - exp).abs().max())
        assert e <= 2e-2 * float(exp.abs().max()) + 1e-4, (e, float(exp.abs().max()))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("shape,groups,cl", [((2, 256, 64, 64), 32, True), ((2, 256, 17, 23), 32, True),
                                             ((1, 64, 5, 7), 8, False), ((1, 256, 256, 256), 32, True),
                                             ((4, 256, 128, 128), 32, True), ((9, 512, 33, 31), 64, True),
                                             ((3, 16, 9, 11), 2, True), ((8, 256, 128, 128), 32, True)])
def test_group_norm_nhwc_vs_torch(dtype, relu, shape, groups, cl):
    """Channels-last GroupNorm (+ReLU) forward/backward (csrc/groupnorm.hip) vs torch f64.
    Shapes cover 1..256 row chunks per image and 1..64 dw/db slices (B = 8 at 128^2:
    2048 channel partials), a column count below one 64-lane block (C = 16).
    With the ReLU, a pre-activation within rounding of 0 may be masked differently by
    the kernel (f32 statistics) and the f64 reference: every such disagreement must sit at
    |pre-activation| < 1e-4, and the gradients are compared against the reference using
    the kernel's own mask (decisions separated from arithmetic)."""
    _check_group_norm(_ops().group_norm_nhwc, dtype, relu, shape, groups, cl)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("shape,groups", [((2, 256, 64, 64), 32), ((2, 96, 17, 23), 32), ((1, 64, 5, 7), 8),
                                          ((3, 48, 9, 8), 16), ((1, 256, 256, 256), 32)])
def test_group_norm_nchw_vs_torch(dtype, relu, shape, groups):
    """NCHW GroupNorm (+ReLU) kernels, incl. groups of 3 channels and HW % 8 != 0 (scalar
    path), same checks as the channels-last test."""
    _check_group_norm(_ops().group_norm_nchw, dtype, relu, shape, groups, False)


def _check_group_norm(fn, dtype, relu, shape, groups, cl):
    B, C, H, W = shape
    g = torch.Generator().manual_seed(C + H)
    x = (torch.randn(shape, generator=g) * 2 + 0.3).to(dtype)
    w = (1 + 0.2 * torch.randn(C, generator=g)).to(dtype)
    b = (0.2 * torch.randn(C, generator=g)).to(dtype)
    gy = torch.randn(shape, generator=g).to(dtype)
    xd = x.to(DEV)
    if cl:
        xd = xd.contiguous(memory_format=torch.channels_last)
    xd, wd, bd = xd.requires_grad_(True), w.to(DEV).requires_grad_(True), b.to(DEV).requires_grad_(True)
    y = fn(xd, wd, bd, groups, 1e-5, relu)
    y.backward(gy.to(DEV))
    xr, wr, br = (t.double().requires_grad_(True) for t in (x, w, b))
    pre = torch.nn.functional.group_norm(xr, groups, wr, br, 1e-5)
    yr = pre
    if relu:
        mask = (y.detach().cpu() > 0)
        ref_mask = pre.detach() > 0
        flips = mask != ref_mask
        if flips.any():
            assert float(pre.detach()[flips].abs().max()) < 1e-4
        yr = pre * mask.double()
    yr.backward(gy.double())
    tol = 3e-5 if dtype == torch.float32 else 2 ** -7
    e = (y.detach().double().cpu() - (torch.relu(pre) if relu else pre).detach()).abs().max()
    assert float(e) <= tol * max(1.0, float(pre.detach().abs().max()))
    for name, got, exp in (("dx", xd.grad, xr.grad), ("dw", wd.grad, wr.grad), ("db", bd.grad, br.grad)):
        e = float((got.detach().double().cpu() - exp.detach()).abs().max())
        assert e <= tol * max(1.0, float(exp.detach().abs().max())), (name, e, float(exp.detach().abs().max()))


# ------------------------------------------------------------------ small-token Linear
@pytest.mark.parametrize("T,I,O,bias", [(400, 256, 256, True), (400, 256, 2048, True), (400, 2048, 256, True),
                                        (1, 64, 128, True), (1000, 128, 64, False), (64, 256, 256, True),
                                        (0, 64, 64, True), (130, 64, 64, True), (257, 128, 192, True),
                                        (2000, 64, 128, True)])
def test_small_linear_grads_vs_torch(T, I, O, bias):
    """csrc/small_linear.hip forward Y, dX and dW / db (one backward launch) vs torch f64 on
    the same bf16 operands (T > 64: the token-split dW, chunks spread over the four waves,
    ragged last chunk; T % 32 != 0: ragged token tiles of the forward / dX)."""
    from visionseg.linear import small_linear
    g = torch.Generator().manual_seed(T + I + O)
    x = torch.randn(T, I, generator=g).to(torch.bfloat16)
    w = (torch.randn(O, I, generator=g) / I ** 0.5).to(torch.bfloat16)
    b = torch.randn(O, generator=g).to(torch.bfloat16) if bias else None
    gy = torch.randn(T, O, generator=g).to(torch.bfloat16)
    xd = x.to(DEV).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    bd = b.to(DEV).requires_grad_(True) if bias else None
    y = small_linear(xd, wd, bd)
    y.backward(gy.to(DEV))
    xr, wr = x.double().requires_grad_(True), w.double().requires_grad_(True)
    br = b.double().requires_grad_(True) if bias else None
    yr = torch.nn.functional.linear(xr, wr, br)
    yr.backward(gy.double())
    pairs = [("y", y.detach(), yr.detach()), ("dx", xd.grad, xr.grad), ("dw", wd.grad, wr.grad)] + \
        ([("db", bd.grad, br.grad)] if bias else [])
    for name, got, exp in pairs:
        e = float((got.double().cpu() - exp).abs().max()) if exp.numel() else 0.0
        scale = float(exp.abs().max()) if exp.numel() else 0.0
        assert e <= 2 ** -7 * max(1.0, scale) + 1e-3, (name, e, scale)


@pytest.mark.parametrize("need", ["x", "w"])
def test_small_linear_partial_backward(need):
    """Only dX (frozen weight) or only dW / db (input without grad) requested: the fused
    backward launches just that half; the result equals the full backward's."""
    from visionseg.linear import _SmallLinearFn
    small_linear = _SmallLinearFn.apply
    g = torch.Generator().manual_seed(11)
    x = torch.randn(4, 100, 256, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(512, 256, generator=g) / 16).to(torch.bfloat16).to(DEV)
    b = torch.randn(512, generator=g).to(torch.bfloat16).to(DEV)
    gy = torch.randn(4, 100, 512, generator=g).to(torch.bfloat16).to(DEV)
    xf, wf, bf = (t.clone().requires_grad_(True) for t in (x, w, b))
    small_linear(xf, wf, bf).backward(gy)
    xp = x.clone().requires_grad_(need == "x")
    wp = w.clone().requires_grad_(need == "w")
    bp = b.clone().requires_grad_(need == "w")
    small_linear(xp, wp, bp).backward(gy)
    if need == "x":
        assert wp.grad is None and bp.grad is None and torch.equal(xp.grad, xf.grad)
    else:
        assert xp.grad is None and torch.equal(wp.grad, wf.grad) and torch.equal(bp.grad, bf.grad)


@pytest.mark.parametrize("B,Q,D,expand", [(4, 100, 256, True), (4, 100, 256, False), (2, 37, 128, True),
                                         (1, 300, 64, False)])
def test_self_attn_in_proj_vs_torch(B, Q, D, expand):
    """linear.self_attn_in_proj (one forward, one backward launch: q, k from h + pos, v from
    h, every gradient use summed in-kernel) vs torch f64 on the same bf16 operands: q / k /
    v, dh, dpos (through the batch expand of the query-position table when expand=True),
    dW / db of the three projections.  h + pos is rounded to bf16 first, as torch's add."""
    from visionseg.linear import SmallLinear, self_attn_in_proj
    g = torch.Generator().manual_seed(B * Q + D)
    h = torch.randn(B, Q, D, generator=g).to(torch.bfloat16)
    table = torch.randn(Q, D, generator=g).to(torch.bfloat16)
    full = torch.randn(B, Q, D, generator=g).to(torch.bfloat16)
    lins = [SmallLinear(D, D).to(torch.bfloat16) for _ in range(3)]
    for m in lins:
        with torch.no_grad():
            m.weight.copy_((torch.randn(D, D, generator=g) / D ** 0.5).to(torch.bfloat16))
            m.bias.copy_(torch.randn(D, generator=g).to(torch.bfloat16))
    gys = [torch.randn(B, Q, D, generator=g).to(torch.bfloat16) for _ in range(3)]
    dl = [SmallLinear(D, D).to(torch.bfloat16).to(DEV) for _ in range(3)]
    for a, m in zip(dl, lins):
        a.load_state_dict(m.state_dict())
    hd = h.to(DEV).requires_grad_(True)
    src = (table if expand else full).to(DEV).requires_grad_(True)
    pd = src.unsqueeze(0).expand(B, -1, -1) if expand else src
    outs = self_attn_in_proj(hd, pd, *dl)
    torch.autograd.backward(outs, [t.to(DEV) for t in gys])
    hr = h.double().requires_grad_(True)
    sr = (table if expand else full).double().requires_grad_(True)
    pr = sr.unsqueeze(0).expand(B, -1, -1) if expand else sr
    wr = [(m.weight.detach().double().requires_grad_(True), m.bias.detach().double().requires_grad_(True))
          for m in lins]
    hq = (h.float() + (table.float() if expand else full.float())).to(torch.bfloat16).double()  # bf16 add
    hq = hq + (hr + pr - (hr + pr).detach())                       # value of the rounded add, grads of h + pos
    F_ = torch.nn.functional
    ref = [F_.linear(hq, *wr[0]), F_.linear(hq, *wr[1]), F_.linear(hr, *wr[2])]
    torch.autograd.backward(ref, [t.double() for t in gys])
    pairs = [("q", outs[0], ref[0]), ("k", outs[1], ref[1]), ("v", outs[2], ref[2]), ("dh", hd.grad, hr.grad),
             ("dpos", src.grad, sr.grad)]
    for i, (a, (w_, b_)) in enumerate(zip(dl, wr)):
        pairs += [(f"dw{i}", a.weight.grad, w_.grad), (f"db{i}", a.bias.grad, b_.grad)]
    for name, got, exp in pairs:
        e = float((got.detach().double().cpu() - exp.detach()).abs().max())
        scale = float(exp.detach().abs().max())
        assert e <= 2 ** -7 * max(1.0, scale) + 1e-3, (name, e, scale)


@pytest.mark.parametrize("relu,pos", [(True, None), (False, "expand"), (True, "full"), (False, "full")])
def test_small_linear_relu_pos_vs_torch(relu, pos):
    """_SmallLinearFn with the fused ReLU (forward epilogue; backward: gY masked by the
    ReLU output in both the dX and the dW / db loads) and the position rows added to X in
    the operand loads (pos expanded over the batch or per token; pos gets X's gradient)
    vs torch f64 on the same bf16 operands, x + pos rounded to bf16 first."""
    from visionseg.linear import _SmallLinearFn
    B, Q, I, O = 4, 100, 256, 512
    g = torch.Generator().manual_seed(17)
    x = torch.randn(B, Q, I, generator=g).to(torch.bfloat16)
    w = (torch.randn(O, I, generator=g) / I ** 0.5).to(torch.bfloat16)
    b = torch.randn(O, generator=g).to(torch.bfloat16)
    src = None if pos is None else torch.randn(*((Q, I) if pos == "expand" else (B, Q, I)), generator=g).to(torch.bfloat16)
    gy = torch.randn(B, Q, O, generator=g).to(torch.bfloat16)
    xd, wd, bd = (t.to(DEV).requires_grad_(True) for t in (x, w, b))
    sd = src.to(DEV).requires_grad_(True) if src is not None else None
    pd = None if sd is None else (sd.unsqueeze(0).expand(B, -1, -1) if pos == "expand" else sd)
    y = _SmallLinearFn.apply(xd, wd, bd, relu, pd)
    y.backward(gy.to(DEV))
    xr, wr, br = (t.double().requires_grad_(True) for t in (x, w, b))
    sr = src.double().requires_grad_(True) if src is not None else None
    xin = xr
    if sr is not None:
        pr = sr.unsqueeze(0).expand(B, -1, -1) if pos == "expand" else sr
        rounded = (x.float() + (src.float() if pos == "full" else src.float()[None])).to(torch.bfloat16).double()
        xin = rounded + (xr + pr - (xr + pr).detach())
    yr = torch.nn.functional.linear(xin, wr, br)
    yr = torch.relu(yr) if relu else yr
    yr.backward(gy.double())
    pairs = [("y", y.detach(), yr.detach()), ("dx", xd.grad, xr.grad), ("dw", wd.grad, wr.grad), ("db", bd.grad, br.grad)]
    if sr is not None:
        pairs.append(("dpos", sd.grad, sr.grad))
    for name, got, exp in pairs:
        e = float((got.double().cpu() - exp).abs().max())
        scale = float(exp.abs().max())
        assert e <= 2 ** -7 * max(1.0, scale) + 1e-3, (name, e, scale)


def test_decoder_layer_small_kernels_vs_library():
    """One masked-attention decoder layer (B = 2, Q = 100, a 32 x 32 memory level) in bf16
    on the small-token kernels (fused Linears, q / k / v in one launch, residual gradients
    handed to the projections through ops.ResidualSink, the query-position gradient summed
    in one ops.GradSink buffer) and on the library path: each against the same layer in
    fp32; every output / gradient error of the fused path <= 1.25 x the library path's
    (+ 1e-3): the fusions add no error beyond bf16 rounding (tools/decoder_layer_ab.py)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("dl_ab", os.path.join(ROOT, "tools", "decoder_layer_ab.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    from visionseg import linear
    saved = (linear._SMALL_FUSED, linear._QKV_FUSED)
    try:
        errs = mod.compare()
    finally:
        linear._SMALL_FUSED, linear._QKV_FUSED = saved
    bad = {k: v for k, v in errs.items() if k != "self_attn.k_proj.bias" and v[0] > 1.25 * v[1] + 1e-3}
    assert not bad, bad
    assert errs["out"][0] < 1e-2 and errs["dh"][0] < 5e-2 and errs["dpos"][0] < 5e-2


def test_small_linear_weight_slice():
    """A weight slice (the decoder's cross-attention q rows of in_proj_weight) gets its
    gradient rows back through autograd's slice."""
    from visionseg.linear import small_linear
    g = torch.Generator().manual_seed(5)
    W = (torch.randn(768, 256, generator=g) / 16).to(torch.bfloat16).to(DEV).requires_grad_(True)
    bb = torch.randn(768, generator=g).to(torch.bfloat16).to(DEV).requires_grad_(True)
    x = torch.randn(4, 100, 256, generator=g).to(torch.bfloat16).to(DEV)
    small_linear(x, W[:256], bb[:256]).float().sum().backward()
    assert float(W.grad[256:].abs().max()) == 0.0 and float(bb.grad[256:].abs().max()) == 0.0
    ref = x.double().reshape(-1, 256).sum(0)
    assert torch.allclose(W.grad[0].double().cpu(), ref.cpu(), rtol=2 ** -7, atol=1e-2)
    assert abs(float(bb.grad[0]) - 400.0) <= 2.0


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,C,Hs,Ws,H,W", [(2, 256, 16, 16, 32, 32), (1, 64, 128, 128, 256, 256), (1, 64, 21, 36, 42, 72),
                                           (2, 32, 13, 21, 25, 42), (1, 32, 7, 9, 7, 9), (1, 96, 40, 70, 64, 100)])
def test_upsample_add_vs_torch(dtype, B, C, Hs, Ws, H, W):
    """FPN merge (csrc/upsample.hip): cur + bilinear upsample of a token-major level vs
    F.interpolate(align_corners=False) + add (up rounded to dtype first, as the unfused
    graph), and the source gradient vs autograd of F.interpolate."""
    ops = _ops()
    g = torch.Generator().manual_seed(C + H)
    cur = torch.randn(B, C, H, W, generator=g).to(dtype)
    big = torch.randn(B, Hs * Ws + 37, C, generator=g).to(dtype)    # the level is a slice of a longer sequence
    go = torch.randn(B, C, H, W, generator=g).to(dtype)
    src = big[:, 5:5 + Hs * Ws]
    sr = src.double().clone().requires_grad_(True)
    up = F.interpolate(sr.transpose(1, 2).reshape(B, C, Hs, Ws), size=(H, W), mode="bilinear", align_corners=False)
    exp = (cur.double() + up.to(dtype).double()).to(dtype)
    up.backward(go.double())
    bd = big.to(DEV).requires_grad_(True)
    out = ops.upsample_add(cur.to(DEV), bd[:, 5:5 + Hs * Ws], Hs, Ws)
    err = (out.double().cpu() - exp.double()).abs().max()
    tol = 1e-5 if dtype == torch.float32 else 2 ** -7
    assert float(err) <= tol * max(1.0, float(exp.double().abs().max())), float(err)
    out.backward(go.to(DEV))
    gsrc = bd.grad[:, 5:5 + Hs * Ws].double().cpu()
    e2 = float((gsrc - sr.grad).abs().max())
    assert e2 <= (1e-5 if dtype == torch.float32 else 2 ** -7) * max(1.0, float(sr.grad.abs().max())), e2
    assert float(bd.grad[:, :5].abs().max()) == 0.0 and float(bd.grad[:, 5 + Hs * Ws:].abs().max()) == 0.0


# ------------------------------------------------------------------ MSDA prologue
def _prep_ref(off, lg, ref, shapes, H, P):
    """The oracle's composition (oracle/ref_model.py:234-238, HF:m2f:994-1002) in f32 on
    the CPU, from the same (dtype-rounded) projections."""
    B, Q, nl = off.shape[0], off.shape[1], len(shapes)
    norm = torch.tensor([[w, h] for h, w in shapes], dtype=torch.float32)
    o = off.float().cpu().reshape(B, Q, H, nl, P, 2)
    a = F.softmax(lg.float().cpu().reshape(B, Q, H, nl * P), -1).view(B, Q, H, nl, P)
    loc = ref.float().cpu()[:, :, None, :, None, :] + o / norm[None, None, None, :, None, :]
    return loc, a


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", [(2, 37, 8, [(4, 5), (2, 3), (1, 1)], 4, "fused"), (1, 300, 8, [(10, 30)] * 4, 4, "plain"),
                                  (3, 5, 2, [(7, 3)], 1, "plain"), (2, 0, 8, [(2, 2)] * 3, 4, "plain"),
                                  (1, 64, 3, [(8, 8), (4, 4)], 8, "fused"),
                                  (2, 37, 8, [(4, 5), (2, 3), (1, 1)], 4, "packed"),
                                  (4, 300, 8, [(10, 20), (5, 10), (3, 5)], 4, "packed")])
def test_msda_prep_vs_torch(case, dtype):
    """csrc/msda_prep.hip (sampling locations + softmax weights and their adjoint) vs the
    f32 torch composition: loc / weights <= 1e-6 abs (f32 math on identical inputs), input
    grads within one output-dtype rounding (f32 1e-6, bf16 2^-8 relative); batch-shared
    reference points (batch stride 0), projections as views of one fused row (row stride
    > row), ragged Q, one level, Q = 0."""
    ops = _ops()
    B, Q, H, shapes, P, layout = case
    nl = len(shapes)
    g = torch.Generator().manual_seed(Q + H)
    if layout in ("fused", "packed"):   # packed: the production row (offsets then logits, P = 4: vector kernels)
        proj = (torch.randn(B, Q, H * nl * P * 3 + (5 if layout == "fused" else 0), generator=g) * 3).to(dtype).to(DEV)
        off, lg = proj[..., :H * nl * P * 2], proj[..., H * nl * P * 2:H * nl * P * 3]
    else:
        off = (torch.randn(B, Q, H * nl * P * 2, generator=g) * 3).to(dtype).to(DEV)
        lg = (torch.randn(B, Q, H * nl * P, generator=g) * 3).to(dtype).to(DEV)
    ref = torch.rand(1, Q, nl, 2, generator=g).expand(B, -1, -1, -1).to(DEV)
    offr, lgr = off.detach().clone().requires_grad_(True), lg.detach().clone().requires_grad_(True)
    loc, aw = ops.msda_prep(offr, lgr, ref, shapes, H, P)
    eloc, eaw = _prep_ref(off, lg, ref, shapes, H, P)
    assert loc.dtype == torch.float32 and aw.dtype == torch.float32
    assert loc.shape == eloc.shape and aw.shape == eaw.shape
    torch.testing.assert_close(loc.cpu(), eloc, atol=1e-6, rtol=1e-6)
    torch.testing.assert_close(aw.cpu(), eaw, atol=1e-6, rtol=1e-5)
    if Q == 0:
        return
    gl = torch.randn(loc.shape, generator=g)
    ga = torch.randn(aw.shape, generator=g)
    torch.autograd.backward((loc, aw), (gl.to(DEV), ga.to(DEV)))
    o32 = off.float().cpu().requires_grad_(True)
    l32 = lg.float().cpu().requires_grad_(True)
    e1, e2 = _prep_ref(o32, l32, ref, shapes, H, P)
    torch.autograd.backward((e1, e2), (gl, ga))
    tol = dict(atol=1e-6, rtol=1e-5) if dtype == torch.float32 else dict(atol=1e-6, rtol=2 ** -8)
    assert offr.grad.dtype == dtype and lgr.grad.dtype == dtype
    torch.testing.assert_close(offr.grad.float().cpu(), o32.grad, **tol)
    torch.testing.assert_close(lgr.grad.float().cpu(), l32.grad, **tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("kind,N", [("gelu", 384), ("gelu", 96), ("relu", 1024), ("relu", 256), ("gelu", 3072),
                                    ("gelu", 6144), ("relu", 2056)])
def test_activation_backward_colsum(dtype, kind, N):
    """ops.activation: torch's forward; the HIP backward (vs_act_backward_colsum) vs
    autograd of F.gelu / F.relu (f64), and its recorded column sums as the bias gradient of
    the TokenLinear feeding it (no column_sum launch for that bias)."""
    from visionseg.linear import TokenLinear
    ops = _ops()
    g = torch.Generator(device="cuda").manual_seed(N)
    M, Ci = 20000, 64
    lin = TokenLinear(Ci, N).to(DEV, dtype)
    h = torch.randn(M, Ci, device=DEV, generator=g).to(dtype)
    gy = torch.randn(M, N, device=DEV, generator=g).to(dtype)
    pre = lin(h)
    y = ops.activation(pre, kind)
    ref_f = torch.nn.functional.gelu if kind == "gelu" else torch.nn.functional.relu
    assert torch.equal(y, ref_f(pre))
    pre.retain_grad()
    y.backward(gy)
    xr = pre.detach().double().requires_grad_(True)
    ref_f(xr).backward(gy.double())
    tol = 1e-5 if dtype == torch.float32 else 2 ** -7
    err = float((pre.grad.double() - xr.grad).abs().max() / xr.grad.abs().max())
    assert err <= tol, err
    exp_b = xr.grad.sum(0)
    rel = float((lin.bias.grad.double() - exp_b).abs().max() / exp_b.abs().max())
    assert rel <= (1e-4 if dtype == torch.float32 else 2 ** -6), rel


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,sizes,N", [(4, [1024, 4096, 16384], 288), (2, [0, 37, 1000, 5], 256), (1, [7], 8),
                                       (3, [16384, 4096, 1024, 256], 64)])
def test_column_sum_segments(dtype, B, sizes, N):
    """Per-segment column sums of [B, S, N] (the level-embedding gradient's reduction)
    vs f64 torch sums over each level's rows of every image; empty segments give 0."""
    ops = _ops()
    g = torch.Generator(device="cuda").manual_seed(N + B)
    x = torch.randn(B, sum(sizes), N, device=DEV, generator=g).to(dtype)
    got = ops.column_sum_segments(x, sizes)
    exp = torch.stack([c.double().sum((0, 1)) for c in torch.split(x, sizes, 1)])
    assert got.shape == exp.shape and got.dtype == torch.float32
    err = float((got.double() - exp).abs().max())
    assert err <= 1e-5 * max(1.0, float(exp.abs().max())) + 1e-4, err
    with pytest.raises(ValueError):
        ops.column_sum_segments(x, sizes + [1])


def _encoder_grads(monkeypatch, fused, dtype, seed=0):
    """Parameter + input gradients of a 2-layer MSDeformAttn encoder stack (PixelDecoder's
    encoder loop, 3 levels at 1024^2 strides, B = 1) with the fused paths
    (value_query_projection with level-embedding routing and residual sinks, TokenLinear
    fc1 with a sink) or, fused=False, every Linear as F.linear (MIN_TOKENS above S)."""
    from visionseg import linear as LN
    from visionseg.model import EncoderLayer, reference_points
    if not fused:
        monkeypatch.setattr(LN, "MIN_TOKENS", 1 << 30)
    torch.manual_seed(seed)
    d, shapes = 256, [(32, 32), (64, 64), (128, 128)]
    layers = torch.nn.ModuleList([EncoderLayer(d, 1024, 8, 3, 4) for _ in range(2)]).to(DEV, dtype)
    for m in layers.modules():
        if isinstance(m, torch.nn.Linear):
            torch.nn.init.normal_(m.weight, std=0.05)
            torch.nn.init.normal_(m.bias, std=0.05)
    lvl = torch.nn.Parameter(torch.randn(3, d, device=DEV).to(dtype))
    S = sum(h * w for h, w in shapes)
    g = torch.Generator(device="cuda").manual_seed(seed + 1)
    h0 = torch.randn(1, S, d, device=DEV, generator=g).to(dtype).requires_grad_(True)
    sine = torch.randn(1, S, d, device=DEV, generator=g).to(dtype)
    sizes = [h * w for h, w in shapes]
    p = sine + torch.cat([lvl.detach()[i].view(1, 1, -1).expand(1, n, -1) for i, n in enumerate(sizes)], 1)
    ref = reference_points(shapes, 1, DEV)
    norm = torch.tensor([[w, hh] for hh, w in shapes], device=DEV, dtype=torch.float32)[None, None, None, :, None, :]
    h = h0
    for layer in layers:
        h = layer(h, p, ref, shapes, norm, (lvl, sizes))
    gy = torch.randn(h.shape, device=DEV, generator=g).to(dtype)
    h.backward(gy)
    out = {n: q.grad.detach().float().clone() for n, q in layers.named_parameters()}
    out["level_embed"] = lvl.grad.detach().float().clone()
    out["h0"] = h0.grad.detach().float().clone()
    return out


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_encoder_fused_gradients_match_plain_composition(monkeypatch, dtype):
    """The encoder's fused backward -- residual gradients added by the dX GEMMs
    (ops.ResidualSink), the level embedding's gradient from per-level column sums x Wp,
    one packed offset/weight projection gradient -- equals the plain autograd composition
    (every Linear as F.linear, pos carrying the level rows with their gradient).  f32:
    2e-4 of each gradient's max (summation order, f32 MSDA atomics); bf16: 3e-2."""
    a = _encoder_grads(monkeypatch, True, dtype)
    monkeypatch.undo()
    b = _encoder_grads(monkeypatch, False, dtype)
    tol = 2e-4 if dtype == torch.float32 else 3e-2
    for k in b:
        scale = float(b[k].abs().max())
        err = float((a[k] - b[k]).abs().max())
        assert err <= tol * scale + 1e-6, (k, err, scale)


def test_residual_sink_plain_paths_keep_gradients():
    """A sink that no consumer armed leaves the LayerNorm's x gradient with autograd; an
    armed sink hands it to the consumer's dX GEMM and x's gradient still equals the sum
    of both paths."""
    from visionseg.linear import TokenLinear
    ops = _ops()
    g = torch.Generator(device="cuda").manual_seed(3)
    M, C = 20000, 64
    lin = TokenLinear(C, C).to(DEV)
    w = torch.ones(C, device=DEV)
    b = torch.zeros(C, device=DEV)
    x = torch.randn(M, C, device=DEV, generator=g)
    gy = torch.randn(M, C, device=DEV, generator=g)
    res = []
    for arm in (False, True):
        xx = x.clone().requires_grad_(True)
        sink = ops.ResidualSink()
        r = lin(xx, sink) if arm else lin(xx)
        _, y = ops.add_layer_norm(xx, r, w, b, 1e-5, sink)
        assert sink.armed == arm
        y.backward(gy)
        assert sink.g is None
        res.append(xx.grad.clone())
        lin.zero_grad()
    err = float((res[0] - res[1]).abs().max())
    assert err <= 1e-4 * float(res[0].abs().max()), err


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_linear_relu_fused_vs_torch(dtype):
    """Encoder-FFN fc1 + ReLU with bias and ReLU in the GEMM epilogue
    (linear._LinearReluFn: torch._addmm_activation, backward masked by the OUTPUT and fused
    with the bias column sums) vs F.relu(F.linear) in f64 on the same rounded inputs:
    output, dX, dW, db.  Tolerances: f32 1e-4 of the scale; bf16 2^-7 relative + a
    bf16-rounding term of the scale."""
    from visionseg.linear import linear_relu_tokens
    g = torch.Generator().manual_seed(7)
    T, Ci, Co = 2 * 8192 + 24, 256, 1024
    x = (torch.randn(1, T, Ci, generator=g)).to(dtype)
    w = (torch.randn(Co, Ci, generator=g) / 16).to(dtype)
    b = (torch.randn(Co, generator=g) / 4).to(dtype)
    go = torch.randn(1, T, Co, generator=g).to(dtype)
    xr, wr, br = (t.double().requires_grad_(True) for t in (x, w, b))
    ref = F.relu(F.linear(xr, wr, br))
    ref.backward(go.double())
    xd, wd, bd = (t.to(DEV).requires_grad_(True) for t in (x, w, b))
    out = linear_relu_tokens(xd, wd, bd)
    assert out.grad_fn is not None and "LinearRelu" in type(out.grad_fn).__name__
    out.backward(go.to(DEV))
    tol = 1e-4 if dtype == torch.float32 else 2 ** -7
    for got, exp in ((out, ref), (xd.grad, xr.grad), (wd.grad, wr.grad), (bd.grad, br.grad)):
        e = (got.detach().double().cpu() - exp.detach()).abs()
        scale = float(exp.detach().abs().max())
        assert float(e.max()) <= tol * scale + (1e-6 if dtype == torch.float32 else 2 ** -8 * scale), \
            (float(e.max()), scale)


@pytest.mark.parametrize("S,n", [(3, 36864), (16, 65536), (33, 4100), (256, 36864)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_splitk_sum_vs_torch(monkeypatch, S, n, dtype):
    """Split-K epilogue (csrc/norm.hip vs_splitk_sum): out = sum_s part[s] + extra, f32
    sums rounded once -- the phased kernel (S >= 16: 8 partial phases per element quad,
    combined in phase order) and the one-thread-per-quad kernel (VS_SPLITK_PHASED=0) vs
    torch's f64 sum: f32 summation-order error only (<= 1e-6 of the summed magnitudes),
    then one rounding to the output dtype."""
    from visionseg import _lib as L
    g = torch.Generator(device=DEV).manual_seed(S)
    part = torch.randn(S, n, device=DEV, generator=g)
    extra = torch.randn(n, device=DEV, generator=g)
    exp = part.double().sum(0) + extra.double()
    mag = part.double().abs().sum(0) + extra.double().abs()
    outs = []
    for phased in ("1", "0"):
        monkeypatch.setenv("VS_SPLITK_PHASED", phased)
        out = torch.empty(n, device=DEV, dtype=dtype)
        L.check(L.lib().vs_splitk_sum(L.dtype_code(out), L.ptr(part), S, n, L.ptr(extra), L.ptr(out), L.stream(out)),
                "splitk_sum")
        torch.cuda.synchronize()
        outs.append(out)
        ulp = 2.0 ** -8 if dtype == torch.bfloat16 else 0.0
        err = (out.double() - exp).abs()
        assert bool((err <= 1e-6 * mag + ulp * exp.abs()).all()), (phased, float(err.max()))


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("ws,shift,heads,B,H,W", [(7, 3, 3, 2, 20, 26), (7, 0, 6, 1, 14, 14), (12, 6, 4, 2, 26, 30),
                                                  (12, 0, 8, 1, 24, 36), (7, 3, 2, 1, 8, 6)])
def test_window_attention_image_layout_equals_reverse(fp8, ws, shift, heads, B, H, W):
    """ops.window_attention_image (the window reverse folded into the bf16 / fp8 kernels:
    output and output gradient in the image layout, padding cropped) == window_attention +
    window_reverse, bit for bit: same kernels, only the rows they read / write move.  The
    backward gets the same image-layout gradient both ways; grad_qkv and the table gradient
    are identical too (padded tokens carry a zero output gradient either way)."""
    ops = _ops()
    if fp8 and ws * ws > 160:
        pytest.skip("fp8 needs window^2 <= 160")
    g = torch.Generator(device="cuda").manual_seed(ws * 100 + H + W + shift)
    nwh, nww = -(-H // ws), -(-W // ws)
    C = heads * 32
    qkv = torch.randn(B * nwh * nww, ws * ws, 3 * C, device=DEV, generator=g).to(torch.bfloat16)
    table = 0.3 * torch.randn((2 * ws - 1) ** 2, heads, device=DEV, generator=g)
    gy = torch.randn(B, H, W, C, device=DEV, generator=g).to(torch.bfloat16)
    res = []
    for image in (True, False):
        q = qkv.clone().requires_grad_(True)
        t = table.clone().requires_grad_(True)
        if image:
            o = ops.window_attention_image(q, t, heads, ws, shift, B, H, W, fp8=fp8)
        else:
            o = ops.window_reverse(ops.window_attention(q, t, heads, ws, shift, nwh, nww, fp8=fp8), B, H, W, ws, shift)
        o.backward(gy)
        res.append((o.detach(), q.grad, t.grad))
    torch.cuda.synchronize()
    (oi, gqi, gti), (ow, gqw, gtw) = res
    assert oi.shape == (B, H, W, C)
    assert torch.equal(oi, ow)
    assert torch.equal(gqi, gqw)
    assert torch.equal(gti, gtw)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,H,W,C,ws,shift", [(2, 20, 26, 96, 7, 3), (1, 14, 14, 192, 7, 0), (2, 26, 30, 128, 12, 6),
                                              (1, 24, 36, 384, 12, 0), (1, 8, 6, 64, 7, 3)])
def test_layer_norm_window_rows_equals_partition(dtype, B, H, W, C, ws, shift):
    """The Swin window partition folded into the LayerNorm before it (ops.WindowRows,
    vs_*layer_norm*_rows): LN(x) / add-LN(x, r) written straight into the window layout ==
    window_partition of the image-layout result, bit for bit (the same row kernel, only the
    row it stores moves; padding rows zero); the backward reading grad_y through the same
    row map gives the same input / weight / bias gradients."""
    ops = _ops()
    g = torch.Generator(device="cuda").manual_seed(H * 100 + W + C + shift)
    x = torch.randn(B, H * W, C, device=DEV, generator=g).to(dtype)
    r = torch.randn(B, H * W, C, device=DEV, generator=g).to(dtype)
    w = (1 + 0.1 * torch.randn(C, device=DEV, generator=g)).to(dtype)
    b = (0.1 * torch.randn(C, device=DEV, generator=g)).to(dtype)
    wr = ops.window_rows(B, H, W, ws, shift, torch.device(DEV))
    nw = -(-H // ws) * -(-W // ws)
    gy = torch.randn(B * nw * ws * ws, C, device=DEV, generator=g).to(dtype)
    gs = torch.randn(B, H * W, C, device=DEV, generator=g).to(dtype)
    for add in (False, True):
        res = []
        for rows in (True, False):
            xx, rr, ww, bb = (t.clone().requires_grad_(True) for t in (x, r, w, b))
            if add:
                s, y = ops.add_layer_norm(xx, rr, ww, bb, wrows=wr if rows else None)
            else:
                s, y = None, ops.layer_norm(xx, ww, bb, wrows=wr if rows else None)
            if not rows:
                y = ops.window_partition(y.view(B, H, W, C), ws, shift).view(-1, C)
            outs = [y] + ([s] if add else [])
            torch.autograd.backward(outs, [gy] + ([gs] if add else []))
            res.append([y.detach(), xx.grad, ww.grad, bb.grad] + ([rr.grad, s.detach()] if add else []))
        torch.cuda.synchronize()
        for a, c in zip(*res):
            assert a.shape == c.shape and torch.equal(a, c)
