"""GPU parity of the hand-written kernels against the oracle (through the C ABI).

Index ops: bit-exact.  f32 kernels vs the fp32 oracle: <= 1e-5 abs (op level).  bf16
kernels: compared with the oracle evaluated on the same bf16-rounded inputs in f32;
tolerance stated per test (bf16 output rounding, 2^-8 relative).
"""
import numpy as np
import pytest
import torch

from oracle import ref_ops as R

pytestmark = pytest.mark.gpu

DEV = "cuda"


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
