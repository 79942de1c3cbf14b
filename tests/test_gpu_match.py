"""Device Hungarian matching (csrc/match.hip) vs scipy.optimize.linear_sum_assignment
(the reference matcher's solver, HF:m2f:489-491), and the set criterion with the device
matcher vs the same criterion with scipy."""
import numpy as np
import pytest
import torch
from scipy.optimize import linear_sum_assignment

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ops():
    from visionseg import ops
    return ops


@pytest.mark.parametrize("Q,ks", [(100, [7, 0, 1, 50]), (100, [100, 3]), (10, [10, 9, 1]), (300, [40]),
                                  (1, [1]), (64, [64, 63, 2, 17])])
def test_lsa_matches_scipy(Q, ks):
    ops = _ops()
    g = torch.Generator().manual_seed(Q * 31 + sum(ks))
    S, B, kmax = 3, len(ks), max(1, max(ks))
    cost = torch.randn(S, B, Q, kmax, generator=g) * 3 + torch.rand(S, B, Q, kmax, generator=g)
    got = ops.linear_sum_assignment_batch(cost.to(DEV), ks).cpu().numpy()
    assert got.shape == (S, B, kmax)
    for s in range(S):
        for b, k in enumerate(ks):
            assert (got[s, b, k:] == -1).all()
            if k == 0:
                continue
            r, cidx = linear_sum_assignment(cost[s, b, :, :k].double().numpy())
            exp = np.full(k, -1)
            exp[cidx] = r
            np.testing.assert_array_equal(got[s, b, :k], exp)


@pytest.mark.parametrize("Q,ks,kc", [(100, [7, 0, 1, 50], 50), (100, [3, 2], 8), (20, [20, 0, 5], 20)])
def test_lsa_device_counts_matches_scipy(Q, ks, kc):
    """Counts read from device memory (graph-replayable launch): same assignments as scipy
    on each image's first count columns, -1 past them, whatever the padded capacity."""
    ops = _ops()
    g = torch.Generator().manual_seed(Q + kc)
    S, B = 2, len(ks)
    cost = torch.randn(S, B, Q, kc, generator=g) * 3
    got = ops.linear_sum_assignment_padded(cost.to(DEV), torch.tensor(ks, dtype=torch.int32, device=DEV)).cpu().numpy()
    assert got.shape == (S, B, kc)
    for s in range(S):
        for b, k in enumerate(ks):
            assert (got[s, b, k:] == -1).all()
            if k:
                r, cidx = linear_sum_assignment(cost[s, b, :, :k].double().numpy())
                exp = np.full(k, -1)
                exp[cidx] = r
                np.testing.assert_array_equal(got[s, b, :k], exp)


def test_lsa_ties_reach_the_optimum():
    """Duplicate target columns make the optimum non-unique: the total cost must still be
    scipy's minimum and the assignment a valid matching."""
    ops = _ops()
    g = torch.Generator().manual_seed(1)
    base = torch.randint(0, 5, (1, 1, 30, 6), generator=g).float()      # integer costs: many ties
    got = ops.linear_sum_assignment_batch(base.to(DEV), [6]).cpu().numpy()[0, 0]
    assert len(set(got.tolist())) == 6 and (got >= 0).all()
    r, c = linear_sum_assignment(base[0, 0].numpy())
    assert float(base[0, 0][got, np.arange(6)].sum()) == float(base[0, 0].numpy()[r, c].sum())


def test_lsa_rejects_bad_sizes():
    ops = _ops()
    with pytest.raises(RuntimeError):
        ops.linear_sum_assignment_batch(torch.zeros(1, 1, 5, 6, device=DEV), [6])      # more targets than queries


def test_criterion_device_matcher_equals_scipy_matcher():
    from visionseg.criterion import SetCriterion
    from visionseg.data import synthetic_batch
    from visionseg.model import M2FConfig
    cfg = M2FConfig.preset("swin_t", num_queries=100, train_num_points=1024)
    _, ml, cl = synthetic_batch(3, 256, seed=4, device=DEV)
    g = torch.Generator(device=DEV).manual_seed(0)
    S, B, Q = 4, len(ml), 100
    masks = [torch.randn(B, Q, 64, 64, device=DEV, generator=g) for _ in range(S)]
    classes = [torch.randn(B, Q, 2, device=DEV, generator=g) for _ in range(S)]
    out = []
    for matcher in ("device", "host"):
        crit = SetCriterion(cfg, matcher=matcher)
        assign = crit.match(masks, torch.stack(classes), ml, cl)
        torch.manual_seed(7)
        torch.cuda.manual_seed(7)
        loss, parts = crit(masks, classes, ml, cl)
        out.append((assign.cpu(), float(loss), {k: float(v) for k, v in parts.items()}))
    # the matcher's point sample is random too: compare the assignment with a fixed seed
    torch.cuda.manual_seed(3)
    a_dev = SetCriterion(cfg, matcher="device").match(masks, torch.stack(classes), ml, cl).cpu()
    torch.cuda.manual_seed(3)
    a_host = SetCriterion(cfg, matcher="host").match(masks, torch.stack(classes), ml, cl).cpu()
    assert torch.equal(a_dev, a_host)
    assert abs(out[0][1] - out[1][1]) <= 1e-4 * abs(out[1][1])


@pytest.mark.parametrize("Kc", [1, 3, 9])
def test_match_cost_kernel_vs_torch(Kc):
    """Fused matcher cost (csrc/match.hip match_cost_kernel) vs the torch formulation of
    HF:m2f:413-481 on the same points (some outside the map: zero padding)."""
    import torch.nn.functional as F
    ops = _ops()
    g = torch.Generator(device=DEV).manual_seed(Kc)
    S, B, Q, H, W, P = 3, 2, 20, 32, 48, 777
    masks = [torch.randn(B, Q, H, W, device=DEV, generator=g) * 3 for _ in range(S)]
    probs = torch.softmax(torch.randn(S, B, Q, 3, device=DEV, generator=g), -1)
    tcls = torch.randint(0, 3, (B, Kc), device=DEV, generator=g)
    pts = torch.rand(B, P, 2, device=DEV, generator=g) * 2.2 - 1.1
    tmask = (torch.rand(B, Kc, 64, 96, device=DEV, generator=g) > 0.5).float()
    tp = F.grid_sample(tmask, pts.unsqueeze(2), align_corners=False).squeeze(3)
    got = ops.match_cost(masks, probs, tcls, pts, tp, 5.0, 2.0, 5.0)
    pp = torch.stack([F.grid_sample(m, pts.unsqueeze(2), align_corners=False).squeeze(3) for m in masks])
    tpt = tp.transpose(1, 2)[None]
    cm = torch.matmul(F.softplus(-pp) / P, tpt) + torch.matmul(F.softplus(pp) / P, 1 - tpt)
    sg = pp.sigmoid()
    cd = 1 - (2 * torch.matmul(sg, tpt) + 1) / (sg.sum(-1)[..., None] + tp.sum(-1)[None, :, None, :] + 1)
    cc = -torch.gather(probs, 3, tcls[None, :, None, :].expand(S, B, Q, Kc))
    exp = 5.0 * cm + 2.0 * cc + 5.0 * cd
    torch.testing.assert_close(got, exp, atol=3e-5, rtol=1e-5)
