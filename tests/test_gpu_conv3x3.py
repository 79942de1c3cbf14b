"""The pixel decoder's channels-last tail: the hand-written 3 x 3 conv
(csrc/conv3x3.hip) and the NHWC FPN merge (csrc/upsample.hip NHWC forms) against torch
fp32 references of the same arithmetic, and the whole NHWC tail against the NCHW path.

* conv forward / input gradient / weight gradient vs F.conv2d and its autograd in f64 on
  the same bf16 operands: the kernels accumulate in f32 and round the output to bf16 once,
  so |err| <= 2^-8 |ref| + 2^-12 max|ref| per element (the f32 summation-order term is
  ~sqrt(K) 2^-24, far below);
* shapes: ragged row segments (W = 70: a 64-pixel segment + 6), image borders (every
  padding tap), a partial pixel tile (B H W not a multiple of 256), Ci / Co = 64 / 24 for
  the forward entry point alone (the input gradient needs Co % 64, the weight gradient
  Ci, Co % 128), the C2 shape (4 x 256 x 256 x 256) against MIOpen's bf16 conv (relative
  RMS 1e-2: both round to bf16, in different orders);
* upsample NHWC forward bit-exact vs the NCHW kernel at exact 2x / 1x (same formula, same order;
  one bf16 rounding apart at other factors, where the compiler contracts differently), backward
  vs torch's F.interpolate adjoint in f32 (1e-5 relative)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ops():
    from visionseg import ops
    return ops


def _bf(shape, g, scale=1.0):
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(DEV)


def _check(out, ref, what):
    out, ref = out.double(), ref.double()
    tol = 2.0 ** -8 * ref.abs() + 2.0 ** -12 * ref.abs().max()
    bad = (out - ref).abs() > tol
    assert not bool(bad.any()), f"{what}: {int(bad.sum())} elements off, max err {float((out - ref).abs().max()):.3g}"


@pytest.mark.parametrize("B,Ci,H,W,Co", [(2, 128, 12, 70, 128), (1, 256, 9, 33, 256), (3, 128, 5, 7, 256)])
@pytest.mark.parametrize("bias", [False, True])
def test_conv3x3_vs_conv2d(B, Ci, H, W, Co, bias):
    ops = _ops()
    g = torch.Generator().manual_seed(B * 1000 + Ci + H + W + int(bias))
    x = _bf((B, Ci, H, W), g).contiguous(memory_format=torch.channels_last)
    w = _bf((Co, Ci, 3, 3), g, (9 * Ci) ** -0.5)
    b = _bf((Co,), g) if bias else None
    gy = _bf((B, Co, H, W), g).contiguous(memory_format=torch.channels_last)
    xs, ws = x.clone().requires_grad_(), w.clone().requires_grad_()
    bs = b.clone().requires_grad_() if bias else None
    y = ops.conv3x3_nhwc(xs, ws, bs)
    assert y.shape == (B, Co, H, W) and y.is_contiguous(memory_format=torch.channels_last)
    y.backward(gy)
    xr, wr = x.double().requires_grad_(), w.double().requires_grad_()
    br = b.double().requires_grad_() if bias else None
    yr = F.conv2d(xr, wr, br, padding=1)
    yr.backward(gy.double())
    _check(y, yr, "forward")
    _check(xs.grad, xr.grad, "input gradient")
    _check(ws.grad, wr.grad, "weight gradient")
    if bias:
        _check(bs.grad, br.grad, "bias gradient")


def test_conv3x3_forward_entry_small_channels():
    """vs_conv3x3_forward alone at Ci = 64, Co = 24 (the 128-tile path, a ragged N tile)."""
    ops = _ops()
    g = torch.Generator().manual_seed(7)
    B, Ci, H, W, Co = 2, 64, 6, 11, 24
    x = _bf((B, H, W, Ci), g)
    w = _bf((Co, Ci, 3, 3), g, (9 * Ci) ** -0.5)
    wf, wb = ops.conv3x3_layouts(w, fwd=True, bwd=True)
    assert torch.equal(wf, w.permute(0, 2, 3, 1)) and torch.equal(wb, w.flip(2, 3).permute(1, 2, 3, 0))
    y = ops.conv3x3_raw(x, wf)
    yr = F.conv2d(x.permute(0, 3, 1, 2).double(), w.double(), padding=1).permute(0, 2, 3, 1)
    _check(y, yr, "forward")


def test_conv3x3_c2_shape_vs_miopen():
    ops = _ops()
    g = torch.Generator(device=DEV).manual_seed(3)
    B, C, H, W = 4, 256, 256, 256
    x = torch.randn(B, C, H, W, device=DEV, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(C, C, 3, 3, device=DEV, generator=g) * (9 * C) ** -0.5).to(torch.bfloat16)
    gy = torch.randn(B, C, H, W, device=DEV, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xs, ws = x.clone().requires_grad_(), w.clone().requires_grad_()
    y = ops.conv3x3_nhwc(xs, ws)
    y.backward(gy)
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    yr = F.conv2d(xr, wr, padding=1)
    yr.backward(gy)

    def rel(a, b):
        return float((a.float() - b.float()).norm() / b.float().norm())

    assert rel(y, yr) < 1e-2 and rel(xs.grad, xr.grad) < 1e-2 and rel(ws.grad, wr.grad) < 1e-2


@pytest.mark.parametrize("H,W,Hs,Ws", [(32, 48, 16, 24), (20, 14, 13, 9), (8, 8, 8, 8)])
def test_upsample_nhwc_vs_nchw_and_torch(H, W, Hs, Ws):
    ops = _ops()
    g = torch.Generator().manual_seed(H * W + Hs)
    B, C = 2, 64
    cur = _bf((B, C, H, W), g)
    src = _bf((B, Hs * Ws, C), g)
    out_nchw = ops.upsample_add(cur, src, Hs, Ws)
    out_nhwc = ops.upsample_add_nhwc(cur.contiguous(memory_format=torch.channels_last), src, Hs, Ws)
    assert out_nhwc.is_contiguous(memory_format=torch.channels_last)
    if 2 * Hs == H and 2 * Ws == W or (Hs, Ws) == (H, W):
        assert torch.equal(out_nhwc, out_nchw)
    else:   # the compiler may contract the bilinear sums differently: the rounded upsample and
        # the rounded sum can each land one bf16 step apart (2^-8 relative at most, each)
        d = (out_nhwc.float() - out_nchw.float()).abs()
        bound = 2.0 ** -7 * (out_nchw.float().abs() + cur.float().abs()) + 1e-6
        assert bool((d <= bound).all()), float(d.max())
    # backward in f32 vs torch's adjoint
    cur32 = cur.float().contiguous(memory_format=torch.channels_last).requires_grad_()
    src32 = src.float().requires_grad_()
    gout = torch.randn(B, C, H, W, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
    ops.upsample_add_nhwc(cur32, src32, Hs, Ws).backward(gout)
    cr, sr = cur.float().requires_grad_(), src.float().requires_grad_()
    up = F.interpolate(sr.transpose(1, 2).reshape(B, C, Hs, Ws), size=(H, W), mode="bilinear", align_corners=False)
    (cr + up).backward(gout)
    assert torch.equal(cur32.grad, cr.grad)
    assert float((src32.grad - sr.grad).norm() / sr.grad.norm()) < 1e-5


def test_pixel_decoder_nhwc_tail_vs_nchw(monkeypatch):
    """The whole channels-last tail (lateral token GEMM, GroupNorm NHWC, upsample NHWC, the
    3x3 conv, GroupNorm + ReLU, mask projection token GEMM) vs the NCHW path on the same
    module and inputs: mask features and every parameter gradient of the tail (bf16: both
    paths round intermediates to bf16 in different orders; relative 3e-2)."""
    from visionseg import model as model_mod
    torch.manual_seed(0)
    cfg = model_mod.M2FConfig(enc_layers=1)
    chans = [96, 192, 384, 768]
    pd = model_mod.PixelDecoder(cfg, chans).to(DEV).to(torch.bfloat16)
    g = torch.Generator().manual_seed(1)
    B, S = 2, 128
    feats = [(torch.randn(B, c, S // 2 ** i, S // 2 ** i, generator=g)).to(DEV, torch.bfloat16)
             .contiguous(memory_format=torch.channels_last) for i, c in enumerate(chans)]
    gm = torch.randn(B, 256, S, S, generator=g).to(DEV, torch.bfloat16)
    tail = [pd.lateral.conv.weight, pd.lateral.gn.weight, pd.output.conv.weight, pd.output.gn.weight,
            pd.output.gn.bias, pd.mask_proj.weight, pd.mask_proj.bias]

    def run(nhwc):
        monkeypatch.setattr(model_mod, "_PIXDEC_NHWC", nhwc)
        pd.zero_grad(set_to_none=True)
        fs = [f.clone().requires_grad_() for f in feats]
        m, _ = pd(fs)
        (m.float() * gm.float()).sum().backward()
        return m.detach().float(), [p.grad.float() for p in tail], fs[0].grad.float()

    m1, g1, f1 = run(True)
    m0, g0, f0 = run(False)

    def rel(a, b):
        return float((a - b).norm() / b.norm().clamp_min(1e-12))

    assert rel(m1, m0) < 3e-2
    assert rel(f1, f0) < 3e-2
    for a, b, p in zip(g1, g0, tail):
        assert rel(a, b) < 3e-2, tuple(p.shape)
