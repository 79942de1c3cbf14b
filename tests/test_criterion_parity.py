"""Set criterion (visionseg.criterion.SetCriterion, the product) vs the oracle criterion
(oracle.ref_model.RefCriterion, pinned to HF:m2f:378-794 by tests/test_oracle_golden.py)
on CPU, fed the same keyed point draws (tests/_draws.py): matching, every weighted loss
component of every decoder step, and the gradients w.r.t. mask and class logits."""
import pytest
import torch

from _draws import KeyedDraws
from oracle.ref_model import RefConfig, RefCriterion


@pytest.mark.parametrize("ks,matcher", [([2, 1], "host"), ([3, 0, 1], "host"), ([1, 1], "host"), ([4, 2], "host")])
def test_criterion_matches_oracle(ks, matcher):
    from visionseg.criterion import SetCriterion
    from visionseg.model import M2FConfig
    cfg = M2FConfig.preset("swin_t", num_queries=12, train_num_points=512)
    rcfg = RefConfig.from_dict(cfg.to_dict())
    g = torch.Generator().manual_seed(7 + sum(ks))
    S, B, Q, H = 4, len(ks), 12, 40
    masks = [(3 * torch.randn(B, Q, H, H, generator=g)).requires_grad_(True) for _ in range(S)]
    classes = [torch.randn(B, Q, 2, generator=g).requires_grad_(True) for _ in range(S)]
    rmasks = [m.detach().clone().requires_grad_(True) for m in masks]
    rclasses = [c.detach().clone().requires_grad_(True) for c in classes]
    ml = [torch.rand(k, 160, 160, generator=g) > 0.6 for k in ks]
    cl = [torch.zeros(k, dtype=torch.int64) for k in ks]
    draws = KeyedDraws(B, max(ks) + 1, seed=3)
    loss, parts = SetCriterion(cfg, matcher=matcher, point_source=draws)(masks, classes, ml, cl)
    rloss, rparts = RefCriterion(rcfg, point_source=draws)(rmasks, rclasses, [m.float() for m in ml], cl)
    assert set(parts) == set(rparts)
    for k in rparts:
        a, b = float(parts[k]), float(rparts[k])
        assert abs(a - b) <= 1e-5 * max(1e-3, abs(b)), (k, a, b)
    assert abs(float(loss) - float(rloss)) <= 1e-5 * abs(float(rloss))
    ga = torch.autograd.grad(loss, masks + classes)
    gb = torch.autograd.grad(rloss, rmasks + rclasses)
    for a, b in zip(ga, gb):
        assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max()) + 1e-12
