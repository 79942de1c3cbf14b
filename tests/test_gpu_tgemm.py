"""Token GEMM (csrc/token_gemm.hip, vs_token_gemm) and the MX quantiser (vs_mx_quantize)
against torch references of the same arithmetic:

* bf16: y = x w^T + b vs the f64 product of the same bf16 operands (f32 accumulation in
  another order, one bf16 rounding of the output: bound 2^-7 relative + a small absolute
  term); ragged M / N tiles, K tails (K = 96: a partial 128-byte K-step), no bias;
* GELU epilogue: the pre-activation as above, the activation vs HF `gelu` (exact erf) of
  the kernel's own rounded pre-activation in f64 (one bf16 rounding);
* MX quantiser: bit-exact vs the rule in torch -- per 32 elements k = floor(log2(448 /
  amax)) (0 for an all-zero block), e4m3 = float8_e4m3fn(x 2^k), scale byte 127 - k;
* fp8 GEMM: vs the f64 product of the DEQUANTISED operands (e4m3 value x 2^-k): the
  fused dequantisation and the MX fragment layout up to f32 summation order (1e-5 of the
  largest |y| + the bf16 output rounding), and vs the bf16 product as the fp8 error budget
  (relative RMS <= 0.06: e4m3 has 3 mantissa bits, errors of the two operands add).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ops():
    from visionseg import ops
    return ops


def _rand(shape, g, scale=1.0):
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16)


def _ref(x, w, b):
    y = x.double() @ w.double().t()
    return y + b.double() if b is not None else y


# the last two take the 256 x 256 tile (>= 256 tiles, N >= 512, K >= 256), one with ragged edges
SHAPES = [(300, 96, 96), (1000, 384, 96), (513, 200, 192), (4096, 576, 192), (777, 3072, 768), (256, 768, 3072),
          (130, 132, 136), (4096, 4096, 512), (4000, 4100, 264)]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("with_bias", [True, False])
def test_token_gemm_bf16_vs_f64(M, N, K, with_bias):
    ops = _ops()
    g = torch.Generator().manual_seed(M + N + K)
    x, w = _rand((M, K), g), _rand((N, K), g, 1 / math.sqrt(K))
    b = _rand((N,), g) if with_bias else None
    y = ops.token_gemm(x.to(DEV), w.to(DEV), b.to(DEV) if b is not None else None).cpu().double()
    ref = _ref(x, w, b)
    err = (y - ref).abs()
    assert bool((err <= ref.abs() * 2 ** -7 + 1e-3 * float(ref.abs().max())).all()), float(err.max())


@pytest.mark.parametrize("M,N,K", [(1000, 384, 96), (777, 3072, 768), (4096, 1536, 384), (4000, 4100, 384)])
def test_token_gemm_gelu_epilogue(M, N, K):
    ops = _ops()
    g = torch.Generator().manual_seed(7 * M + K)
    x, w, b = _rand((M, K), g), _rand((N, K), g, 1 / math.sqrt(K)), _rand((N,), g)
    y, pre = ops.token_gemm(x.to(DEV), w.to(DEV), b.to(DEV), gelu=True)
    y, pre = y.cpu().double(), pre.cpu().double()
    ref = _ref(x, w, b)
    err = (pre - ref).abs()
    assert bool((err <= ref.abs() * 2 ** -7 + 1e-3 * float(ref.abs().max())).all()), float(err.max())
    gel = 0.5 * pre * (1 + torch.erf(pre / math.sqrt(2)))          # HF gelu of the kernel's pre-activation
    e2 = (y - gel).abs()
    assert bool((e2 <= gel.abs() * 2 ** -8 + 1e-6).all()), float(e2.max())


@pytest.mark.parametrize("M,N,K,bias,gelu", [(40000, 288, 96, True, False), (33000, 96, 96, False, False),
                                             (65555, 384, 96, True, True), (40000, 576, 192, True, False),
                                             (32768, 200, 136, True, False), (50000, 192, 192, True, True),
                                             (1000, 384, 96, True, False), (70, 128, 64, False, True)])
def test_token_gemm_stream_equals_tile_kernel(monkeypatch, M, N, K, bias, gelu):
    """The streaming kernel for short rows (K <= 192, many tokens; W slice resident, token
    tiles streamed) against the tile kernel on the same operands -- the same products in
    the same K order, so bit-equal outputs -- and against the f64 product.  Ragged token
    tiles, N not a multiple of the 128-feature slice, K tails inside a 128-byte step; the
    last two shapes force the streaming kernel below its row threshold."""
    ops = _ops()
    g = torch.Generator().manual_seed(M + N + K)
    x, w = _rand((M, K), g), _rand((N, K), g, 1 / math.sqrt(K))
    b = _rand((N,), g) if bias else None
    xd, wd, bd = x.to(DEV), w.to(DEV), (b.to(DEV) if b is not None else None)
    res = []
    for rows in ("0", "1"):                  # 0: the tile kernel; 1: streaming for any M
        monkeypatch.setenv("VS_TGEMM_STREAM_ROWS", rows)
        out = ops.token_gemm(xd, wd, bd, gelu=gelu)
        torch.cuda.synchronize()
        res.append([t.cpu() for t in (out if gelu else (out,))])
    for a, s in zip(*res):
        assert torch.equal(a, s), float((a.double() - s.double()).abs().max())
    y = res[1][-1 if gelu else 0].double()   # the pre-activation (gelu) or the output
    ref = _ref(x, w, b)
    err = (y - ref).abs()
    assert bool((err <= ref.abs() * 2 ** -7 + 1e-3 * float(ref.abs().max())).all()), float(err.max())


def _mx_emulate(x):
    """The quantiser's rule in torch: (e4m3 bytes, scale bytes, dequantised f64)."""
    rows, K = x.shape
    xb = x.float().view(rows, K // 32, 32)
    amax = xb.abs().amax(-1, keepdim=True)
    k = torch.where(amax > 0, torch.floor(torch.log2(448.0 / amax.clamp_min(1e-38))), torch.zeros_like(amax))
    k = k.clamp(-126, 126)
    q = (xb * torch.exp2(k)).to(torch.float8_e4m3fn)
    deq = q.double() * torch.exp2(-k.double())
    return q.view(torch.uint8).view(rows, K), (127 - k).to(torch.uint8).view(rows, K // 32), deq.view(rows, K)


@pytest.mark.parametrize("rows,K,scale", [(64, 128, 1.0), (333, 768, 1e-3), (100, 3072, 30.0)])
def test_mx_quantize_bit_exact(rows, K, scale):
    ops = _ops()
    g = torch.Generator().manual_seed(rows + K)
    x = _rand((rows, K), g, scale)
    x[0, :32] = 0                                   # an all-zero block
    x[1, 5] = 0.0
    q, s = ops.mx_quantize(x.to(DEV))
    eq, es, _ = _mx_emulate(x)
    assert torch.equal(s.cpu(), es)
    assert torch.equal(q.cpu(), eq)


@pytest.mark.parametrize("M,N,K", [(300, 384, 384), (777, 3072, 768), (256, 768, 3072), (4096, 576, 256),
                                   (4000, 4100, 512)])
@pytest.mark.parametrize("gelu", [False, True])
def test_token_gemm_fp8_vs_dequantised(M, N, K, gelu):
    ops = _ops()
    g = torch.Generator().manual_seed(3 * M + N)
    x, w, b = _rand((M, K), g), _rand((N, K), g, 1 / math.sqrt(K)), _rand((N,), g)
    xq, xs = ops.mx_quantize(x.to(DEV))
    wq, ws = ops.mx_quantize(w.to(DEV))
    out = ops.token_gemm(xq, wq, b.to(DEV), gelu=gelu, x_scales=xs, w_scales=ws)
    y = (out[1] if gelu else out).cpu().double()
    _, _, xd = _mx_emulate(x)
    _, _, wd = _mx_emulate(w)
    ref = xd @ wd.t() + b.double()
    err = (y - ref).abs()
    assert bool((err <= ref.abs() * 2 ** -7 + 1e-5 * float(ref.abs().max())).all()), float(err.max())
    exact = _ref(x, w, b)
    rel_rms = float((y - exact).norm() / exact.norm())
    print(f"fp8 token GEMM {M}x{N}x{K}: vs dequantised max {float(err.max()):.2e}, vs bf16 operands rel-RMS {rel_rms:.3e}")
    assert rel_rms <= 0.06
    if gelu:
        pre = y
        gel = 0.5 * pre * (1 + torch.erf(pre / math.sqrt(2)))
        e2 = (out[0].cpu().double() - gel).abs()
        assert bool((e2 <= gel.abs() * 2 ** -8 + 1e-6).all()), float(e2.max())


@pytest.mark.parametrize("fp8", [False, True])
def test_linear_gelu_autograd_vs_f64(monkeypatch, fp8):
    """linear.linear_gelu_tokens vs torch autograd in f64 on the same bf16 operands: bf16 at
    this shape = the GEMM + the GELU pass (ops.activation), the backward through the fused
    GELU-derivative + column-sum pass; fp8 = the token GEMM with the GELU epilogue on the MX
    MFMA, the backward straight-through, so the gradients match the bf16 formula up to the fp8
    forward's pre-activation error."""
    from visionseg.linear import linear_gelu_tokens
    g = torch.Generator().manual_seed(11)
    M, K, N = 20000, 384, 1536
    x = _rand((M, K), g)
    w = _rand((N, K), g, 1 / math.sqrt(K))
    b = _rand((N,), g, 0.1)
    gy = _rand((M, N), g, 0.01)
    xd, wd, bd = (t.to(DEV).requires_grad_(True) for t in (x, w, b))
    y = linear_gelu_tokens(xd, wd, bd, fp8=fp8)
    y.backward(gy.to(DEV))
    xr, wr, br = (t.double().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.gelu(xr @ wr.t() + br)
    yr.backward(gy.double())
    tol = 0.05 if fp8 else 0.01
    for got, exp in ((y, yr), (xd.grad, xr.grad), (wd.grad, wr.grad), (bd.grad, br.grad)):
        rel = float((got.detach().cpu().double() - exp.detach()).norm() / exp.detach().norm())
        assert rel <= tol, rel


@pytest.mark.parametrize("M,N,K,fp8", [(1000, 384, 96, False), (777, 3072, 768, True), (4000, 4096, 384, False),
                                       (4000, 4096, 512, True)])
def test_gelu_quantised_output_equals_mx_quantize(M, N, K, fp8):
    """VS_TGEMM_QOUT: the GELU epilogue's MX fp8 copy of its output is bit-identical to
    vs_mx_quantize of the bf16 output (the fc2 operand without a quantisation pass)."""
    ops = _ops()
    g = torch.Generator().manual_seed(M + 5 * N)
    x, w, b = _rand((M, K), g).to(DEV), _rand((N, K), g, 1 / math.sqrt(K)).to(DEV), _rand((N,), g).to(DEV)
    if fp8:
        xq, xs = ops.mx_quantize(x)
        wq, ws = ops.mx_quantize(w)
        y, pre, (yq, ys) = ops.token_gemm(xq, wq, b, gelu=True, x_scales=xs, w_scales=ws, quant_out=True)
        y2, pre2 = ops.token_gemm(xq, wq, b, gelu=True, x_scales=xs, w_scales=ws)
    else:
        y, pre, (yq, ys) = ops.token_gemm(x, w, b, gelu=True, quant_out=True)
        y2, pre2 = ops.token_gemm(x, w, b, gelu=True)
    assert torch.equal(y, y2) and torch.equal(pre, pre2)
    eq, es = ops.mx_quantize(y)
    assert torch.equal(ys, es)
    assert torch.equal(yq, eq)


@pytest.mark.parametrize("backend", ["rows", "mx"])
@pytest.mark.parametrize("C", [384, 192])
def test_mlp_fp8_vs_bf16_mlp(monkeypatch, C, backend):
    """linear.mlp_fp8 (config C5's Swin MLP: fc1 + GELU on the MX fp8 token GEMM writing fc2's
    fp8 operand in its epilogue, fc2 on the MX fp8 GEMM, straight-through backward; C = 192:
    fc1 too shallow for fp8, the vendor GEMM + GELU, fc2 on fp8) vs the same MLP in f64 on
    the bf16 operands: output rel-RMS <= 0.06 (the fp8 budget of two chained products),
    input / weight / bias gradients rel-L2 <= 0.06.  M above the token-GEMM threshold."""
    from visionseg import linear
    from visionseg.linear import mlp_fp8
    monkeypatch.setattr(linear, "FP8_GEMM", backend)
    g = torch.Generator().manual_seed(21)
    M = 20000
    x = _rand((M, C), g)
    w1, b1 = _rand((4 * C, C), g, 1 / math.sqrt(C)), _rand((4 * C,), g, 0.1)
    w2, b2 = _rand((C, 4 * C), g, 1 / math.sqrt(4 * C)), _rand((C,), g, 0.1)
    gy = _rand((M, C), g, 0.01)
    dev = [t.to(DEV).requires_grad_(True) for t in (x, w1, b1, w2, b2)]
    y = mlp_fp8(*dev)
    y.backward(gy.to(DEV))
    ref = [t.double().requires_grad_(True) for t in (x, w1, b1, w2, b2)]
    yr = torch.nn.functional.linear(torch.nn.functional.gelu(torch.nn.functional.linear(ref[0], ref[1], ref[2])),
                                    ref[3], ref[4])
    yr.backward(gy.double())
    rel = float((y.detach().cpu().double() - yr.detach()).norm() / yr.detach().norm())
    print(f"mlp fp8 vs f64: output rel-RMS {rel:.3e}")
    assert rel <= 0.06
    for d, r in zip(dev, ref):
        e = float((d.grad.cpu().double() - r.grad).norm() / r.grad.norm())
        assert e <= 0.06, e


@pytest.mark.parametrize("C,shift", [(384, 0), (768, 6)])
def test_layer_norm_fp8_copy_equals_mx_quantize(C, shift):
    """The LayerNorms' MX fp8 copy of their output (vs_layer_norm_forward_rows_q,
    vs_add_layer_norm_forward_q; the qkv / fc1 operand of config C5's fp8 Swin block) is
    bit-identical to vs_mx_quantize of the bf16 output they store, padding rows zero, and
    the bf16 output itself equals the plain kernels'."""
    from visionseg.linear import TokenLayerNorm
    ops = _ops()
    g = torch.Generator().manual_seed(C + shift)
    B, H, W, ws = 2, 30, 26, 12
    x = _rand((B, H * W, C), g).to(DEV)
    r = _rand((B, H * W, C), g).to(DEV)
    ln = TokenLayerNorm(C).to(DEV).to(torch.bfloat16)
    with torch.no_grad():
        ln.weight.copy_(_rand((C,), g).to(DEV))
        ln.bias.copy_(_rand((C,), g).to(DEV))
    wr = ops.window_rows(B, H, W, ws, shift, x.device)
    y, (yq, ys) = ln.forward_windows(x, wr, quant=True)
    assert torch.equal(y, ln.forward_windows(x, wr))
    eq, es = ops.mx_quantize(y)
    assert torch.equal(yq, eq) and torch.equal(ys, es)
    s, y2, (q2, s2) = ln.add_forward_windows(x, r, wr, quant=True)
    s_ref, y2_ref = ln.add_forward_windows(x, r, wr)
    assert torch.equal(s, s_ref) and torch.equal(y2, y2_ref)
    eq, es = ops.mx_quantize(y2)
    assert torch.equal(q2, eq) and torch.equal(s2, es)
    s3, y3, (q3, s3q) = ln.add_forward(x, r, quant=True)
    eq, es = ops.mx_quantize(y3)
    assert torch.equal(q3, eq) and torch.equal(s3q, es)


@pytest.mark.parametrize("choice", [None, True, False])
def test_linear_tokens_forward_dispatch(monkeypatch, choice):
    """linear.linear_tokens with the static forward rule (token GEMM vs vendor GEMM by
    shape, linear._use_token_gemm) or forced either way: the output and the gradients equal
    torch autograd in f64 within bf16 rounding, and the rule is deterministic."""
    from visionseg import linear
    assert linear._use_token_gemm(20000, 576, 192) and linear._use_token_gemm(262144, 96, 384)
    assert not linear._use_token_gemm(589824, 576, 192) and not linear._use_token_gemm(262144, 384, 96)
    if choice is not None:
        monkeypatch.setattr(linear, "_use_token_gemm", lambda M, N, K: choice)
    g = torch.Generator().manual_seed(3)
    M, K, N = 20000, 192, 576
    x, w, b = _rand((M, K), g), _rand((N, K), g, 1 / math.sqrt(K)), _rand((N,), g, 0.1)
    gy = _rand((M, N), g, 0.01)
    xd, wd, bd = (t.to(DEV).requires_grad_(True) for t in (x, w, b))
    y = linear.linear_tokens(xd, wd, bd)
    y.backward(gy.to(DEV))
    xr, wr, br = (t.double().requires_grad_(True) for t in (x, w, b))
    yr = xr @ wr.t() + br
    yr.backward(gy.double())
    for got, exp in ((y, yr), (xd.grad, xr.grad), (wd.grad, wr.grad), (bd.grad, br.grad)):
        rel = float((got.detach().cpu().double() - exp.detach()).norm() / exp.detach().norm())
        assert rel <= 0.01, rel


@pytest.mark.parametrize("fp8_dgrad,backend", [(False, "mx"), (True, "mx"), (False, "rows")])
def test_fp8_linear_dgrad_modes(monkeypatch, fp8_dgrad, backend):
    """linear_fp8_tokens' backward with dX on the bf16 vendor GEMM (default) or on the MX fp8
    token GEMM (VS_FP8_DGRAD=1): dX, dW, db vs f64 autograd on the bf16 operands (fp8
    forward: output rel-RMS <= 0.05; gradients rel-L2 <= 0.05, dX on bf16 <= 0.01)."""
    from visionseg import linear
    monkeypatch.setattr(linear, "FP8_DGRAD", fp8_dgrad)
    monkeypatch.setattr(linear, "FP8_GEMM", backend)
    g = torch.Generator().manual_seed(5)
    M, K, N = 20000, 768, 384
    x, w, b = _rand((M, K), g), _rand((N, K), g, 1 / math.sqrt(K)), _rand((N,), g, 0.1)
    gy = _rand((M, N), g, 0.01)
    xd, wd, bd = (t.to(DEV).requires_grad_(True) for t in (x, w, b))
    y = linear.linear_fp8_tokens(xd, wd, bd)
    y.backward(gy.to(DEV))
    xr, wr, br = (t.double().requires_grad_(True) for t in (x, w, b))
    yr = xr @ wr.t() + br
    yr.backward(gy.double())
    for got, exp, tol in ((y, yr, 0.05), (xd.grad, xr.grad, 0.05 if fp8_dgrad else 0.01), (wd.grad, wr.grad, 0.05),
                          (bd.grad, br.grad, 0.05)):
        rel = float((got.detach().cpu().double() - exp.detach()).norm() / exp.detach().norm())
        assert rel <= tol, rel


def _row_emulate(x):
    """The row quantiser's rule in torch: (e4m3 bytes [rows, K], scale f32 [rows, 1], dequantised f64)."""
    xf = x.float()
    amax = xf.abs().amax(-1, keepdim=True)
    k = torch.where(amax > 0, torch.floor(torch.log2(448.0 / amax.clamp_min(1e-38))), torch.zeros_like(amax))
    k = k.clamp(-126, 126)
    q = (xf * torch.exp2(k)).to(torch.float8_e4m3fn)
    return q.view(torch.uint8), torch.exp2(-k), q.double() * torch.exp2(-k.double())


@pytest.mark.parametrize("rows,K,scale", [(64, 192, 1.0), (333, 768, 1e-3), (100, 6144, 30.0), (7, 40, 2.0)])
def test_row_quantize_fp8_bit_exact(rows, K, scale):
    """ops.row_quantize_fp8 (csrc/fp8_rows.hip: per-row power-of-two scale, e4m3 RNE) ==
    the rule emulated in torch, bit for bit, incl. an all-zero row; the GELU variant ==
    F.gelu (exact erf) in bf16 and its quantisation."""
    ops = _ops()
    g = torch.Generator().manual_seed(rows + K)
    x = _rand((rows, K), g, scale)
    x[0] = 0                                        # an all-zero row
    x[1, 5] = 0.0
    q, s = ops.row_quantize_fp8(x.to(DEV))
    eq, es, _ = _row_emulate(x)
    assert torch.equal(q.view(torch.uint8).cpu(), eq)
    assert torch.equal(s.cpu(), es)
    y, qg, sg = ops.row_quantize_fp8(x.to(DEV), gelu=True)
    ey = torch.nn.functional.gelu(x.float()).to(torch.bfloat16)
    assert float((y.cpu().float() - ey.float()).abs().max()) <= 2.0 ** -7 * float(ey.float().abs().max())
    eq2, es2, _ = _row_emulate(y.cpu())
    assert torch.equal(qg.view(torch.uint8).cpu(), eq2) and torch.equal(sg.cpu(), es2)


@pytest.mark.parametrize("M,N,K", [(20000, 384, 768), (16384, 1536, 384), (20000, 768, 3072)])
def test_fp8_rows_linear_vs_dequantised(M, N, K):
    """The rowwise vendor fp8 GEMM path (linear._LinearFp8RowFn: ops.row_quantize_fp8 +
    torch._scaled_mm with the bias) vs the product of the dequantised operands in f64
    (rel-RMS <= 1e-2: bf16 output rounding and f32 accumulation), and vs the exact bf16
    product (rel-RMS <= 0.06, the e4m3 budget)."""
    from visionseg import linear
    g = torch.Generator().manual_seed(M + N + K)
    x, w, b = _rand((M, K), g), _rand((N, K), g, 1 / math.sqrt(K)), _rand((N,), g, 0.1)
    assert linear.fp8_rows_ok(M, N, K)
    y = linear._LinearFp8RowFn.apply(x.to(DEV), w.to(DEV), b.to(DEV)).cpu().double()
    _, _, xd = _row_emulate(x)
    _, _, wd = _row_emulate(w)
    ref = xd @ wd.t() + b.double()
    rel = float((y - ref).norm() / ref.norm())
    exact = x.double() @ w.double().t() + b.double()
    rel2 = float((y - exact).norm() / exact.norm())
    print(f"fp8 rows {M}x{N}x{K}: vs dequantised {rel:.2e}, vs exact {rel2:.2e}")
    assert rel <= 1e-2 and rel2 <= 0.06


@pytest.mark.parametrize("C,shift,res", [(768, 0, False), (384, 6, True), (1536, 0, True), (192, 0, False)])
def test_layer_norm_row_quant_equals_row_quantize(C, shift, res):
    """The LayerNorm forwards' row-scaled e4m3 copy (quant="rows", csrc/norm.hip Q == 2, the
    rowwise fp8 GEMM's operand) == ops.row_quantize_fp8 of the bf16 output they store, bit for
    bit, in the window layout (with shift) and token-major with the residual add."""
    from visionseg import ops
    from visionseg.linear import TokenLayerNorm
    g = torch.Generator().manual_seed(C + shift)
    B, H, W, ws = 1, 24, 24, 12
    ln = TokenLayerNorm(C).to(DEV).to(torch.bfloat16)
    with torch.no_grad():
        ln.weight.copy_(torch.randn(C, generator=g) * 0.5 + 1)
        ln.bias.copy_(torch.randn(C, generator=g) * 0.1)
    x = _rand((B, H * W, C), g, 2.0).to(DEV)
    r = _rand((B, H * W, C), g).to(DEV)
    if res:
        s, y, (yq, ys) = ln.add_forward(x, r, quant="rows")
        s_ref, y_ref = ln.add_forward(x, r)
        assert torch.equal(s, s_ref)
    else:
        wr = ops.window_rows(B, H, W, ws, shift, x.device)
        y, (yq, ys) = ln.forward_windows(x, wr, quant="rows")
        y_ref = ln.forward_windows(x, wr)
    assert torch.equal(y.view(-1, C), y_ref.view(-1, C))
    eq, es = ops.row_quantize_fp8(y.view(-1, C))
    assert torch.equal(yq.view(torch.uint8), eq.view(torch.uint8)) and torch.equal(ys.view(-1, 1), es)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_plane_projections_vs_conv1x1(dtype):
    """linear.token_plane_projection (token-major -> NCHW planes, the pixel decoder's lateral
    conv) and linear.plane_projection (NCHW planes -> channels-last planes, the mask projection) vs
    F.conv2d with a 1x1 kernel: outputs and all three gradients (f32: 1e-4 relative; bf16:
    one output rounding + f32-accumulated products, 2e-2 relative)."""
    import torch.nn.functional as F
    from visionseg.linear import plane_projection, token_plane_projection
    g = torch.Generator().manual_seed(5)
    B, Ci, Co, H, W = 2, 96, 256, 24, 20
    x = torch.randn(B, H * W, Ci, generator=g).to(DEV, dtype)
    w = (torch.randn(Co, Ci, 1, 1, generator=g) / Ci ** 0.5).to(DEV, dtype)
    b = torch.randn(Co, generator=g).to(DEV, dtype)
    gy = torch.randn(B, Co, H, W, generator=g).to(DEV, dtype)
    tol = 1e-4 if dtype == torch.float32 else 2e-2

    def rel(a, r):
        return float((a.float() - r.float()).norm() / r.float().norm())

    xs, ws, bs = (t.clone().requires_grad_() for t in (x, w, b))
    y = token_plane_projection(xs, ws, bs, H, W)
    y.backward(gy)
    xr, wr, br = (t.float().clone().requires_grad_() for t in (x, w, b))
    yr = F.conv2d(xr.view(B, H, W, Ci).permute(0, 3, 1, 2), wr, br)
    yr.backward(gy.float())
    assert y.shape == (B, Co, H, W) and y.is_contiguous()
    for a, r in ((y, yr), (xs.grad, xr.grad), (ws.grad, wr.grad), (bs.grad, br.grad)):
        assert rel(a, r) <= tol
    # the reverse direction: planes [B, Co, H, W] -> channels-last planes [B, Ci, H, W]
    w2 = (torch.randn(Ci, Co, 1, 1, generator=g) / Co ** 0.5).to(DEV, dtype)
    p = gy.clone().requires_grad_()
    w2s = w2.clone().requires_grad_()
    t = plane_projection(p, w2s, None)
    gt = torch.randn(t.shape, generator=g).to(DEV, dtype)
    t.backward(gt)
    pr, w2r = gy.float().clone().requires_grad_(), w2.float().clone().requires_grad_()
    tr = F.conv2d(pr, w2r)
    tr.backward(gt.float())
    assert t.shape == tr.shape and rel(t, tr) <= tol
    assert rel(p.grad, pr.grad) <= tol and rel(w2s.grad, w2r.grad) <= tol


@pytest.mark.parametrize("T,N,K,ld_pad", [(5000, 96, 288, 0), (4096, 288, 96, 0), (20000, 1536, 384, 0),
                                          (4200, 256, 1024, 0), (6001, 136, 200, 24)])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_token_wgrad_vs_f64(T, N, K, ld_pad, out_dtype):
    """csrc/token_wgrad.hip: dW = gY^T X and db = column sums of gY vs f64 on the same bf16
    operands: ragged token chunks (T % 64), ragged output / input tiles (N, K not multiples of
    128 / 256), strided rows (ld_pad > 0: views of wider tensors).  f32 accumulation over T
    products, one rounding to out_dtype: |err| <= 2^-8 |ref| (bf16 out; 1e-6 f32) + 1e-5
    max|ref| (summation order over up to 20000 tokens)."""
    ops = _ops()
    g = torch.Generator().manual_seed(T + N + K)
    gyw = _rand((T, N + ld_pad), g).to(DEV)
    xw = _rand((T, K + ld_pad), g).to(DEV)
    gy, x = gyw[:, :N], xw[:, :K]
    dw, db = ops.token_wgrad(gy, x, out_dtype, bias=True)
    ref = gy.double().t() @ x.double()
    rb = gy.double().sum(0)
    rel = 2.0 ** -8 if out_dtype == torch.bfloat16 else 1e-6
    for a, r in ((dw, ref), (db, rb)):
        assert a.dtype == out_dtype
        err = (a.double() - r).abs()
        assert bool((err <= rel * r.abs() + 1e-5 * r.abs().max()).all()), float(err.max())


def test_linear_backward_token_wgrad_matches_vendor(monkeypatch):
    """linear_tokens' backward with the token weight-gradient kernel (bias fused) vs the vendor
    batched-GEMM path: the same gradients up to f32 summation order (bf16 outputs: 1e-2
    relative RMS, both one rounding of the f32 sum)."""
    from visionseg import linear as lin
    g = torch.Generator().manual_seed(11)
    x = _rand((4, 2048, 192), g).to(DEV)
    w = _rand((576, 192), g, 0.05).to(DEV)
    b = _rand((576,), g).to(DEV)
    gy = _rand((4, 2048, 576), g).to(DEV)

    def run(flag):
        monkeypatch.setattr(lin, "_TOKEN_WGRAD", flag)
        xs, ws, bs = (t.clone().requires_grad_() for t in (x, w, b))
        lin.linear_tokens(xs, ws, bs).backward(gy)
        return xs.grad.float(), ws.grad.float(), bs.grad.float()

    a, v = run(True), run(False)
    for p, q in zip(a, v):
        assert float((p - q).norm() / q.norm()) < 1e-2


def test_token_wgrad_grouped_vs_f64():
    """ops.token_wgrad_grouped: one launch for Linears of different shapes (both tile widths,
    with and without bias, a strided operand, a ragged token count); every dW / db vs f64 with
    the single-Linear bound (one f32 sum, one rounding)."""
    ops = _ops()
    g = torch.Generator().manual_seed(21)
    shapes = [(4096, 288, 96, True), (6001, 96, 384, False), (20000, 1536, 384, True), (4200, 256, 1024, True),
              (65536, 576, 192, False), (3000, 136, 200, True)]
    items, refs = [], []
    for T, N, K, bias in shapes:
        gyw = _rand((T, N + 8), g).to(DEV)
        gy, x = gyw[:, :N], _rand((T, K), g).to(DEV)
        dw = torch.empty(N, K, device=DEV, dtype=torch.bfloat16)
        db = torch.empty(N, device=DEV, dtype=torch.bfloat16) if bias else None
        items.append((gy, x, dw, db))
        refs.append((gy.double().t() @ x.double(), gy.double().sum(0) if bias else None))
    ops.token_wgrad_grouped(items, torch.bfloat16)
    for (gy, x, dw, db), (rw, rb) in zip(items, refs):
        for a, r in ((dw, rw), (db, rb)):
            if r is None:
                continue
            err = (a.double() - r).abs()
            assert bool((err <= 2.0 ** -8 * r.abs() + 1e-5 * r.abs().max()).all()), (tuple(gy.shape), float(err.max()))



def test_transpose_batched_bit_exact():
    """ops.transpose_batched: one launch for matrices of different shapes (edge tiles, a
    64-divisible one, the Swin-T weight shapes) equals src.t() bit for bit."""
    ops = _ops()
    g = torch.Generator().manual_seed(5)
    shapes = [(288, 96), (96, 384), (1536, 384), (8, 8), (72, 200), (384, 1536), (64, 128), (3072, 768)]
    pairs = []
    for R, C in shapes:
        src = _rand((R, C), g).to(DEV)
        pairs.append((src, torch.full((C, R), float("nan"), device=DEV, dtype=torch.bfloat16)))
    ops.transpose_batched(pairs)
    for src, dst in pairs:
        assert torch.equal(dst, src.t().contiguous()), tuple(src.shape)


def test_linear_dgrad_weight_transposes_bit_exact(monkeypatch):
    """The dX GEMMs of a stack of token Linears read the W^T copies written by ONE batched
    launch at the first backward use (linear._WT): dX equals the per-call weight.t().contiguous()
    path bit for bit, and nothing stays pending after the backward."""
    from visionseg import linear as lin
    g = torch.Generator().manual_seed(9)
    x = _rand((4, 4096, 192), g).to(DEV)
    w1, b1 = _rand((576, 192), g, 0.05).to(DEV), _rand((576,), g).to(DEV)
    w2, b2 = _rand((192, 576), g, 0.05).to(DEV), _rand((192,), g).to(DEV)
    gy = _rand((4, 4096, 192), g).to(DEV)
    assert lin._dgrad_on_token_gemm(4 * 4096, w2, torch.bfloat16)

    def run(batched):
        if not batched:
            monkeypatch.setattr(lin._WT, "request", lambda w: None)
        ps = [t.clone().requires_grad_() for t in (x, w1, b1, w2, b2)]
        xs, a1, c1, a2, c2 = ps
        lin.linear_tokens(lin.linear_tokens(xs, a1, c1), a2, c2).backward(gy)
        monkeypatch.undo()
        return [p.grad for p in ps]

    a, b = run(True), run(False)
    assert not lin._WT.pending
    for p, q in zip(a, b):
        assert torch.equal(p, q)


@pytest.mark.parametrize("act", ["gelu", "relu"])
@pytest.mark.parametrize("M,N,K", [(32768, 384, 96), (40000, 768, 192), (16384, 1536, 384), (4096, 3072, 768),
                                   (86016, 1024, 256), (1000, 256, 64)])
def test_token_gemm_act_backward_epilogue(M, N, K, act):
    """token_gemm(dY, W2^T, gelu_pre=pre / relu_out=y) -- an MLP's activation backward in fc2's
    dX epilogue (stream kernel at K <= 192 and >= 32768 rows, tile kernels otherwise, the
    256 x 256 one at the encoder FFN shape) -- equals the composition it replaces: dH =
    token_gemm(dY, W2^T) stored in bf16, then the activation backward kernel
    (vs_act_backward_colsum) on (dH, pre).  Same formula, each product rounded once: at most
    1 bf16 ulp apart (FMA contraction may differ) and identical almost everywhere."""
    from visionseg import _lib as L
    ops = _ops()
    g = torch.Generator().manual_seed(M + N)
    gy = _rand((M, K), g).to(DEV)
    wt = _rand((N, K), g, K ** -0.5).to(DEV)               # W2^T: [hidden, C]
    pre = _rand((M, N), g, 2.0).to(DEV)
    if act == "relu":
        pre = pre.clamp_min(0)                             # a ReLU output (exact zeros where masked)
    got = ops.token_gemm(gy, wt, **({"gelu_pre": pre} if act == "gelu" else {"relu_out": pre}))
    dh = ops.token_gemm(gy, wt)
    ref = torch.empty_like(dh)
    cs = torch.empty(N, device=DEV, dtype=torch.bfloat16)
    ws = torch.empty(int(L.lib().vs_column_sum_workspace_bytes(M, N)), device=DEV, dtype=torch.uint8)
    L.check(L.lib().vs_act_backward_colsum(L.VS_BF16, 1 if act == "gelu" else 0, L.ptr(dh), L.ptr(pre), L.ptr(ref),
                                           L.ptr(cs), L.ptr(ws), M, N, L.stream(dh)), "act_backward_colsum")
    torch.cuda.synchronize()
    a = got.view(torch.int16).int()
    b = ref.view(torch.int16).int()
    ulp = (a - b).abs()
    same_sign = (a >= 0) == (b >= 0)
    assert bool((ulp[same_sign] <= 1).all()), int(ulp[same_sign].max())
    assert bool(((got.float() - ref.float()).abs()[~same_sign] <= 1e-30).all())    # +-0
    assert float((ulp == 0).float().mean()) > 0.99


@pytest.mark.parametrize("stage", [1, 3])
def test_mlp_gelu_backward_sink_vs_composition(stage):
    """Swin MLP fc1 -> GELU -> fc2 with the GELU backward folded into fc2's dX GEMM
    (ops.GeluBackwardSink; stage 1: fc1 + GELU on the streaming kernel, stage 3: vendor fc1 +
    the activation node) vs the same MLP without the sink: every gradient within bf16 summation
    order (fc1's bias gradient now comes from the split-K kernel's column sums)."""
    from visionseg import linear as lin
    ops = _ops()
    C, T = (96, 4 * 128 * 128) if stage == 1 else (384, 4 * 64 * 64)
    g = torch.Generator().manual_seed(stage)
    x = _rand((T, C), g).to(DEV)
    w1, b1 = _rand((4 * C, C), g, C ** -0.5).to(DEV), _rand((4 * C,), g, 0.1).to(DEV)
    w2, b2 = _rand((C, 4 * C), g, (4 * C) ** -0.5).to(DEV), _rand((C,), g, 0.1).to(DEV)
    gy = _rand((T, C), g).to(DEV)

    def run(fused):
        ps = [t.clone().requires_grad_() for t in (x, w1, b1, w2, b2)]
        xs, a1, c1, a2, c2 = ps
        gs = ops.GeluBackwardSink() if fused else None
        h = lin.linear_gelu_tokens(xs, a1, c1, gelu_sink=gs)
        lin.linear_tokens(h, a2, c2, gelu_sink=gs).backward(gy)
        if fused:
            assert gs.pre is not None and not gs.done
        return [p.grad.float() for p in ps]

    a, b = run(True), run(False)
    for name, p, q in zip(("x", "w1", "b1", "w2", "b2"), a, b):
        assert float((p - q).norm() / q.norm()) < 1e-2, name


def test_ffn_relu_backward_sink_vs_composition():
    """The encoder FFN (fc1 + bias + ReLU in the GEMM epilogue, fc2) with the ReLU backward
    folded into fc2's dX GEMM (ops.ActBackwardSink("relu")) vs without: every gradient within
    bf16 summation order."""
    from visionseg import linear as lin
    ops = _ops()
    T, C, F = 4 * 5376, 256, 1024
    g = torch.Generator().manual_seed(7)
    x = _rand((T, C), g).to(DEV)
    w1, b1 = _rand((F, C), g, C ** -0.5).to(DEV), _rand((F,), g, 0.1).to(DEV)
    w2, b2 = _rand((C, F), g, F ** -0.5).to(DEV), _rand((C,), g, 0.1).to(DEV)
    gy = _rand((T, C), g).to(DEV)

    def run(fused):
        ps = [t.clone().requires_grad_() for t in (x, w1, b1, w2, b2)]
        xs, a1, c1, a2, c2 = ps
        rs = ops.ActBackwardSink("relu") if fused else None
        f = lin.linear_relu_tokens(xs, a1, c1, act_sink=rs)
        lin.linear_tokens(f, a2, c2, gelu_sink=rs).backward(gy)
        if fused:
            assert rs.pre is not None and not rs.done
        return [p.grad.float() for p in ps]

    a, b = run(True), run(False)
    for name, p, q in zip(("x", "w1", "b1", "w2", "b2"), a, b):
        assert float((p - q).norm() / q.norm()) < 1e-2, name
