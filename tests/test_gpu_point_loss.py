"""The set criterion's mask losses through the mask head's factors
(ops.MatchedPointLogitsFunction) vs autograd through the full logits.

The function replaces the full-size [B, Q, H, W] logits gradients of every decoder step
(zero except the matched rows) with a scatter into the matched maps and one adjoint GEMM
pair for all steps; mathematically the same gradient.  f32: <= 1e-5 of max|grad|; bf16
factors: the adjoint GEMMs round G to bf16 (2^-8 relative) -> 1e-2 of max|grad|.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("S,B,Q,Kc,C,H,W,n", [(3, 2, 20, 3, 128, 32, 48, 300), (10, 4, 100, 3, 256, 64, 64, 1000)])
def test_matched_point_logits_grad(dtype, tol, S, B, Q, Kc, C, H, W, n):
    from visionseg import ops
    g = torch.Generator(device=DEV).manual_seed(S * 100 + Q)
    E = [torch.randn(B, Q, C, device=DEV, generator=g).to(dtype).requires_grad_() for _ in range(S)]
    P0 = (torch.randn(B, H * W, C, device=DEV, generator=g) / C ** 0.5).to(dtype).requires_grad_()
    # distinct matched queries per (step, image): a matching; last slot padded (-> Q-1, no loss)
    qsel = torch.stack([torch.stack([torch.randperm(Q, device=DEV, generator=g)[:Kc] for _ in range(B)])
                        for _ in range(S)])
    coords = torch.rand(S * B * Kc, n, 2, device=DEV, generator=g)
    wts = torch.randn(S * B * Kc, n, device=DEV, generator=g)
    keep = torch.ones(S, B, Kc, dtype=torch.bool, device=DEV)
    keep[:, :, -1] = False

    def loss_of(plog):
        return (torch.where(keep.reshape(-1, 1), plog * wts, torch.zeros((), device=DEV))).sum()

    # product path: logits from the HIP mask head, loss through the factors
    masks = [ops.mask_head(e, P0, H, W) for e in E]
    maps, fac = ops.matched_maps(masks, qsel)
    assert fac is not None and not maps.requires_grad
    loss_of(ops.point_logits(maps, coords, qsel, fac)).backward()
    gE = [e.grad.float().clone() for e in E]
    gP = P0.grad.float().clone()
    for t in E + [P0]:
        t.grad = None
    # reference: the same sampling, autograd through the full logits (f32 einsum)
    Ef = [e.detach().float().requires_grad_() for e in E]
    Pf = P0.detach().float().requires_grad_()
    full = [torch.einsum("bqc,bnc->bqn", e, Pf).view(B, Q, H, W) for e in Ef]
    bidx = torch.arange(B, device=DEV)[:, None].expand(B, Kc)
    pred = torch.stack([full[s][bidx, qsel[s]] for s in range(S)]).reshape(S * B * Kc, 1, H, W)
    ref = torch.nn.functional.grid_sample(pred, 2 * coords.unsqueeze(2) - 1, align_corners=False).squeeze(3).squeeze(1)
    loss_of(ref).backward()
    for a, b in zip(gE, Ef):
        assert float((a - b.grad).abs().max()) <= tol * float(b.grad.abs().max()) + 1e-30
    assert float((gP - Pf.grad).abs().max()) <= tol * float(Pf.grad.abs().max())
    # unmatched query rows get exactly zero
    hit = torch.zeros(S, B, Q, dtype=torch.bool, device=DEV)
    hit.scatter_(2, qsel[..., :-1], True)
    for s in range(S):
        assert float(gE[s][~hit[s]].abs().max()) == 0.0


@pytest.mark.parametrize("S,B,K,n,H,W", [(2, 3, 2, 500, 40, 56), (10, 4, 3, 12544, 256, 256), (1, 1, 1, 7, 300, 9)])
def test_point_scatter_vs_grid_sampler_backward(S, B, K, n, H, W):
    """vs_point_scatter == torch's grid_sampler_2d_backward (same float weights; only the
    summation order differs), pairs reordered (s, b, k) -> (b, s, k); points include the
    border and outside-the-map cases."""
    from visionseg import _lib as L
    g = torch.Generator(device=DEV).manual_seed(n)
    N = S * B * K
    coords = torch.rand(N, n, 2, device=DEV, generator=g) * 1.2 - 0.1      # some taps outside
    coords[:, :3] = torch.tensor([[0.0, 0.0], [1.0, 1.0], [0.5 / W, 0.5 / H]], device=DEV)
    grid = (2.0 * coords.unsqueeze(2) - 1.0).contiguous()
    gp = torch.randn(N, n, device=DEV, generator=g)
    ref = torch.ops.aten.grid_sampler_2d_backward(gp.view(N, 1, n, 1), torch.empty(N, 1, H, W, device=DEV), grid,
                                                  0, 0, False, [True, False])[0]
    ref = ref.view(S, B, K, H, W).transpose(0, 1).reshape(B, S * K, H, W)
    out = torch.full((B, S * K, H, W), float("nan"), device=DEV)
    L.check(L.lib().vs_point_scatter(L.ptr(gp), L.ptr(grid), L.ptr(out), S, B, K, n, H, W, L.stream(gp)),
            "point_scatter")
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    assert float((out - ref).abs().max()) <= 1e-5 * max(1.0, float(ref.abs().max()))


def test_point_sample_masks_equals_grid_sample():
    """ops.point_sample_masks (csrc/mask_head.hip, the criterion's target labels straight from
    the bool masks) == grid_sample on the f32 copy (HF:m2f:245-275 point_sample), in both
    coordinate modes: [0, 1] coords with a row map (the loss labels, pair (s, i) -> target i)
    and grid-space coords shared by an image's targets (the matcher), incl. points on the
    border and outside [0, 1]."""
    import torch.nn.functional as F
    from visionseg import ops
    g = torch.Generator(device="cuda").manual_seed(11)
    for B, Kc, H, W, P, S in ((2, 3, 37, 53, 100, 2), (4, 2, 1024, 1024, 12544, 10)):
        masks = torch.rand(B, Kc, H, W, device="cuda", generator=g) > 0.7
        # a bool tensor may hold any non-zero byte as True (views / casts of byte data)
        masks.view(torch.uint8)[masks.view(torch.uint8) > 0] = 255 if H < 100 else 1
        # matcher: one point set per image in [-1, 1]
        grid = torch.rand(B, P, 1, 2, device="cuda", generator=g) * 2.2 - 1.1
        grid[0, :3, 0] = torch.tensor([[-1.0, -1.0], [1.0, 1.0], [0.0, 0.0]], device="cuda")
        exp = F.grid_sample(masks.float(), grid, align_corners=False).squeeze(3)
        got = ops.point_sample_masks(masks.view(B * Kc, H, W), grid.squeeze(2), grid_space=True,
                                     sets_per_coord=Kc).view(B, Kc, P)
        assert float((got - exp).abs().max()) <= 1e-6
        # loss labels: S x B*Kc point sets in [0, 1], set n reads mask n % (B*Kc)
        NP = B * Kc
        coords = torch.rand(S * NP, P, 2, device="cuda", generator=g) * 1.2 - 0.1
        rows = torch.arange(S * NP, device="cuda") % NP
        exp = F.grid_sample(masks.view(NP, 1, H, W).float()[rows], 2.0 * coords.unsqueeze(2) - 1.0,
                            align_corners=False).view(S * NP, P)
        got = ops.point_sample_masks(masks.view(NP, H, W), coords, rows=rows)
        assert float((got - exp).abs().max()) <= 1e-6


def test_point_sample_f32_maps_equals_grid_sample():
    """ops.point_sample (the criterion's uncertainty / matched-logit points and MaskDINO's, on
    csrc/mask_head.hip point_sample_rows_kernel with no row map) == grid_sample (HF:m2f:245-275
    point_sample) on f32 maps, incl. points on the border and outside [0, 1]; autograd inputs
    keep grid_sample."""
    import torch.nn.functional as F
    from visionseg import ops
    g = torch.Generator(device="cuda").manual_seed(12)
    for N, H, W, P in ((3, 37, 53, 100), (80, 256, 256, 37632)):
        maps = torch.randn(N, 1, H, W, device="cuda", generator=g) * 4
        coords = torch.rand(N, P, 2, device="cuda", generator=g) * 1.2 - 0.1
        coords[0, :3] = torch.tensor([[0.0, 0.0], [1.0, 1.0], [0.5, 0.5]], device="cuda")
        exp = F.grid_sample(maps, 2.0 * coords.unsqueeze(2) - 1.0, align_corners=False).view(N, P)
        got = ops.point_sample(maps, coords)
        assert float((got - exp).abs().max()) <= 1e-5 * float(maps.abs().max())
    m = maps[:2].clone().requires_grad_(True)
    ops.point_sample(m, coords[:2]).sum().backward()
    assert m.grad is not None
