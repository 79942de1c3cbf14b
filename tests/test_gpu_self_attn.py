"""GPU parity of the decoder self-attention core (csrc/self_attn.hip, ops.self_attention)
against an f64 restatement of HF:m2f:1659-1664 (Mask2FormerAttention over the queries: softmax
(q k^T d^-1/2) v, no mask) and of MaskDINO's DN-masked self-attention (True = blocked, shared
by the batch and the heads).

The kernel keeps the softmax, lse and dS in f32 and feeds P / dS to the MFMAs as exact bf16
hi + lo pairs, so its only rounding of note is the bf16 output store: outputs and gradients
are gated at 2^-8 relative + 2e-3 of the tensor's max, and against the oracle composition run
in bf16 (the training-step parity test's yardstick) the kernel's error must be at most half
the yardstick's.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ops():
    from visionseg import ops
    return ops


def _case(B, Q, heads, mask, seed):
    g = torch.Generator().manual_seed(seed)
    C = heads * 32
    q, k, v = (torch.randn(B, Q, C, generator=g).mul(1.5).to(torch.bfloat16) for _ in range(3))
    go = torch.randn(B, Q, C, generator=g).to(torch.bfloat16)
    blocked = None
    if mask == "dn":
        # MaskDINO-shaped: `pad` denoising queries in groups of 23 that see only their own
        # group, then matching queries that see each other but no DN query
        pad, grp = Q - 300, 23
        i = torch.arange(Q)
        dn = i < pad
        gid = torch.where(dn, i // grp, torch.full_like(i, -1))
        blocked = (dn[:, None] & dn[None, :] & (gid[:, None] != gid[None, :])) | (~dn[:, None] & dn[None, :])
    elif mask == "batch":
        blocked = torch.rand(B, Q, Q, generator=g) < 0.6
        blocked[0, 3] = True                     # a row blocked at every key
    return q, k, v, go, blocked


def _reference(q, k, v, go, blocked, heads, dtype):
    """softmax((q k^T) * 32^-1/2 + (-inf where blocked)) v with its autograd gradients, in
    `dtype` (f64: the exact reference; bf16: the yardstick); a row blocked at every key
    gives a zero output (the kernel's rule; SDPA would give NaN)."""
    B, Q, C = q.shape
    qs, ks, vs = (t.to(dtype).view(B, Q, heads, 32).transpose(1, 2).requires_grad_(True) for t in (q, k, v))
    s = torch.matmul(qs, ks.transpose(-1, -2)) * (32 ** -0.5)
    full = None
    if blocked is not None:
        bm = blocked if blocked.dim() == 3 else blocked[None]
        full = bm.all(-1)                                             # [B|1, Q]
        bm = bm & ~full[..., None]
        s = s.masked_fill(bm[:, None], float("-inf"))
    p = torch.softmax(s, -1)
    if full is not None:
        p = p.masked_fill(full[:, None, :, None], 0.0)
    o = torch.matmul(p, vs).transpose(1, 2).reshape(B, Q, C)
    o.backward(go.to(dtype))
    return [t.detach().double() for t in (o, qs.grad.transpose(1, 2).reshape(B, Q, C),
                                          ks.grad.transpose(1, 2).reshape(B, Q, C),
                                          vs.grad.transpose(1, 2).reshape(B, Q, C))]


@pytest.mark.parametrize("B,Q,heads,mask", [(4, 100, 8, None), (2, 37, 4, None), (1, 130, 8, None),
                                            (2, 460, 8, "dn"), (3, 200, 8, "batch"), (1, 300, 8, None)])
def test_self_attention_bf16_vs_f64(B, Q, heads, mask):
    ops = _ops()
    q, k, v, go, blocked = _case(B, Q, heads, mask, seed=Q + B)
    exact = _reference(q, k, v, go, blocked, heads, torch.float64)
    yard = _reference(q, k, v, go, blocked, heads, torch.bfloat16)
    words = None
    if blocked is not None:
        bm = blocked.clone()
        words = ops.pack_blocked(bm.to(DEV))
        assert torch.equal(ops.unpack_bitmask(words, Q).cpu(), bm)
    qd, kd, vd = (t.to(DEV).requires_grad_(True) for t in (q, k, v))
    out = ops.self_attention(qd, kd, vd, heads, words=words)
    out.backward(go.to(DEV))
    torch.cuda.synchronize()
    got = [out.detach(), qd.grad, kd.grad, vd.grad]
    rows = []
    for name, a, e, y in zip(("out", "dq", "dk", "dv"), got, exact, yard):
        a = a.double().cpu()
        assert bool(torch.isfinite(a).all()), name
        err = (a - e).abs()
        bound = 2.0 ** -8 * e.abs() + 2e-3 * float(e.abs().max())
        rows.append((name, float(err.max()), float((y - e).abs().max()), float(e.abs().max()),
                     bool((err <= bound).all())))
    print("self_attn", (B, Q, heads, mask), [(n, f"{m:.2e}", f"{ye:.2e}", f"{mx:.2f}", ok) for n, m, ye, mx, ok in rows])
    for name, m, ye, mx, ok in rows:
        assert ok, (name, m, mx)
        assert m <= 0.5 * ye, (name, m, ye)


def test_self_attention_fully_blocked_rows_are_zero():
    """A row blocked at every key: zero output, zero dQ, and no NaN reaching dK / dV."""
    ops = _ops()
    B, Q, heads = 2, 64, 8
    q, k, v, go, _ = _case(B, Q, heads, None, seed=3)
    blocked = torch.zeros(Q, Q, dtype=torch.bool)
    blocked[5] = True
    blocked[40, :33] = True
    words = ops.pack_blocked(blocked.to(DEV))
    qd, kd, vd = (t.to(DEV).requires_grad_(True) for t in (q, k, v))
    out = ops.self_attention(qd, kd, vd, heads, words=words)
    out.backward(go.to(DEV))
    assert float(out[:, 5].abs().max()) == 0.0
    assert float(qd.grad[:, 5].abs().max()) == 0.0
    for t in (out, qd.grad, kd.grad, vd.grad):
        assert bool(torch.isfinite(t).all())
    exact = _reference(q, k, v, go, blocked, heads, torch.float64)
    for a, e in zip((out.detach(), qd.grad, kd.grad, vd.grad), exact):
        err = (a.double().cpu() - e).abs()
        assert bool((err <= 2.0 ** -8 * e.abs() + 2e-3 * float(e.abs().max())).all()), float(err.max())


@pytest.mark.parametrize("mask", [None, "dn"])
def test_self_attention_f32_path_vs_f64(mask):
    """f32 inputs (the parity kernel mode) run the scalar masked-attention kernels with
    explicit words: <= 1e-5 of the f64 reference."""
    ops = _ops()
    B, Q, heads = 2, (320 if mask else 100), 8
    q, k, v, go, blocked = _case(B, Q, heads, mask, seed=11)
    q, k, v = (t.float() for t in (q, k, v))
    exact = _reference(q, k, v, go.float(), blocked, heads, torch.float64)
    words = ops.pack_blocked(blocked.to(DEV)) if blocked is not None else None
    qd, kd, vd = (t.to(DEV).requires_grad_(True) for t in (q, k, v))
    out = ops.self_attention(qd, kd, vd, heads, words=words)
    out.backward(go.float().to(DEV))
    for a, e in zip((out.detach(), qd.grad, kd.grad, vd.grad), exact):
        err = float((a.double().cpu() - e).abs().max())
        assert err <= 1e-5 * max(1.0, float(e.abs().max())), err


def test_decoder_self_attention_never_calls_sdpa(monkeypatch):
    """The decoders' self-attention runs on the hand-written kernels: no module of the package
    names SDPA (AOTriton on ROCm), and the shared core (model.self_attention_core, used by the
    M2F DecoderLayer and the MaskDINO DINODecoderLayer) runs with SDPA patched to raise."""
    import glob
    import os
    from visionseg import model as M
    from visionseg import maskdino as MD

    pkg = os.path.dirname(M.__file__)
    for f in glob.glob(os.path.join(pkg, "*.py")):
        assert "scaled_dot_product_attention" not in open(f).read(), f

    def _boom(*a, **k):
        raise AssertionError("F.scaled_dot_product_attention reached")

    monkeypatch.setattr(F, "scaled_dot_product_attention", _boom)
    ops = _ops()
    B = 2
    for Q, blocked in ((100, None), (330, torch.zeros(330, 330, dtype=torch.bool))):
        if blocked is not None:
            blocked[30:, :30] = True                       # matching queries do not see the DN ones
        x = torch.randn(B, Q, 256, device=DEV, dtype=torch.bfloat16, requires_grad=True)
        words = ops.pack_blocked(blocked.to(DEV)) if blocked is not None else None
        att = M.self_attention_core(x, x, x, 8, 32 ** -0.5, words)
        att.float().sum().backward()
        assert bool(torch.isfinite(x.grad).all())
    assert MD.self_attention_core is M.self_attention_core
