"""MaskDINO on the GPU (config C4, row f3; parity UNPINNED -- no MaskDINO oracle in the
container): forward structure, training steps through the product Trainer in fp32 and
bf16 (finite losses and gradients, weights move), graph replay vs eager, and the
Swin-T / 300-query model at 256^2."""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _tiny(**kw):
    from visionseg.maskdino import MaskDINOConfig
    d = dict(embed_dim=32, depths=(2, 2, 2, 2), num_heads=(1, 2, 4, 8), feature_size=64, mask_feature_size=64,
             hidden_dim=64, enc_ffn=128, dec_ffn=128, dec_heads=2, enc_layers=2, dec_layers=3, num_queries=20,
             num_labels=1, dn_num=16, train_num_points=256)
    d.update(kw)
    return MaskDINOConfig(**d)


def test_forward_structure():
    from visionseg.criterion import PaddedTargets
    from visionseg.data import synthetic_batch
    from visionseg.maskdino import MaskDINO, masks_to_boxes
    cfg = _tiny()
    m = MaskDINO(cfg).init_weights(0).to(DEV).train()
    imgs, ml, cl = synthetic_batch(2, 128, seed=2, device=DEV)
    tg = PaddedTargets.from_lists(ml, cl, kc=4, device=DEV)
    boxes = masks_to_boxes(tg.masks)
    out = m(imgs, tg, boxes)
    pad = out["dn"]["pad"]
    assert pad == cfg.dn_num
    S = cfg.dec_layers + 1
    assert len(out["classes"]) == len(out["masks"]) == len(out["boxes"]) == S
    for c, mk, b in zip(out["classes"], out["masks"], out["boxes"]):
        assert c.shape == (2, pad + cfg.num_queries, cfg.num_labels)
        assert mk.shape == (2, pad + cfg.num_queries, 32, 32) and b.shape == (2, pad + cfg.num_queries, 4)
        assert bool(((b >= 0) & (b <= 1)).all())
    assert out["interm"]["masks"].shape == (2, cfg.num_queries, 32, 32)
    m.eval()
    with torch.no_grad():
        ev = m(imgs)
    assert ev["dn"] is None and ev["classes"][0].shape[1] == cfg.num_queries


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_training_steps(precision):
    from visionseg.data import synthetic_batch
    from visionseg.maskdino import MaskDINO, MaskDINOCriterion
    from visionseg.train import SolverConfig, Trainer
    cfg = _tiny()
    m = MaskDINO(cfg).init_weights(0)
    s = SolverConfig(warmup_iters=0, amp=precision == "bf16", lr=1e-3)
    tr = Trainer(m, MaskDINOCriterion(cfg), s, device=DEV)
    imgs, ml, cl = synthetic_batch(2, 128, seed=3, device=DEV)
    w0 = tr.opt.master.clone()
    losses = [float(tr.step(imgs, ml, cl)) for _ in range(3)]
    assert all(torch.isfinite(torch.tensor(losses))), losses
    assert bool(torch.isfinite(tr.opt.master).all()) and float((tr.opt.master - w0).abs().max()) > 0
    assert bool(torch.isfinite(tr.opt.reduced_grads()).all())
    print(precision, "maskdino losses", losses)


def test_graph_replay_matches_eager():
    from visionseg.data import synthetic_batch
    from visionseg.maskdino import MaskDINO, MaskDINOCriterion
    from visionseg.train import SolverConfig, Trainer
    cfg = _tiny()
    m = MaskDINO(cfg).init_weights(0)
    b1 = synthetic_batch(2, 128, seed=1, device=DEV)
    ta = Trainer(copy.deepcopy(m), MaskDINOCriterion(cfg), SolverConfig(warmup_iters=0), device=DEV)
    tb = Trainer(copy.deepcopy(m), MaskDINOCriterion(cfg), SolverConfig(warmup_iters=0), device=DEV, graphs=True)
    la, lb = [], []
    for i in range(5):
        torch.manual_seed(100 + i)
        la.append(float(ta.step(*b1)))
        torch.manual_seed(100 + i)
        lb.append(float(tb.step(*b1)))
    torch.cuda.synchronize()
    assert len(tb._graph_states) == 1
    for a, b in zip(la, lb):
        assert abs(a - b) <= 3e-2 * max(1.0, abs(a)), (la, lb)


def test_swin_t_300_queries_256():
    from visionseg.data import synthetic_batch
    from visionseg.maskdino import MaskDINO, MaskDINOConfig, MaskDINOCriterion
    from visionseg.train import SolverConfig, Trainer
    cfg = MaskDINOConfig.preset("swin_t", train_num_points=2048)
    m = MaskDINO(cfg).init_weights(0)
    tr = Trainer(m, MaskDINOCriterion(cfg), SolverConfig(warmup_iters=0), device=DEV)
    imgs, ml, cl = synthetic_batch(2, 256, seed=5, device=DEV)
    losses = [float(tr.step(imgs, ml, cl)) for _ in range(2)]
    assert all(torch.isfinite(torch.tensor(losses))), losses


def test_point_sample_rows_kernel_vs_grid_sample():
    """csrc/mask_head.hip point_sample_rows_kernel (the MaskDINO mask losses' per-query label
    sampler) == grid_sample on the gathered maps, incl. points outside [0, 1] and the border;
    a C4-sized call (4 images x 400 queries x 12544 points) against the same reference."""
    import torch.nn.functional as F
    from visionseg.maskdino import _point_sample_rows
    g = torch.Generator(device="cuda").manual_seed(3)
    for M, H, W, N, P in ((6, 17, 23, 8, 50), (40, 256, 256, 1600, 12544)):
        maps = (torch.rand(M, H, W, device="cuda", generator=g) > 0.5).float()
        rows = torch.randint(0, M, (N,), device="cuda", generator=g)
        coords = torch.rand(N, P, 2, device="cuda", generator=g) * 1.2 - 0.1
        coords[0, :4] = torch.tensor([[0.0, 0.0], [1.0, 1.0], [0.0, 1.0], [1.0, 0.0]], device="cuda")
        exp = F.grid_sample(maps[rows][:, None], 2.0 * coords.unsqueeze(2) - 1.0,
                            align_corners=False).squeeze(3).squeeze(1)
        got = _point_sample_rows(maps, rows, coords)
        assert float((got - exp).abs().max()) <= 1e-6


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_factor_mask_losses_equal_full_logit_autograd(precision):
    """MaskDINOCriterion's mask losses through the mask head's factors on the selected rows
    (ops.RowPointLogitsFunction: point scatter + the head's adjoint on R rows, dP summed in
    one GradSink) vs autograd through the full logits (grid_sample backward, index
    backward, mask-head backward over all queries): the same loss and the same gradient
    of every parameter (bf16: mask features of 128 channels, the fused MFMA backward)."""
    from visionseg.criterion import PaddedTargets
    from visionseg.data import synthetic_batch
    from visionseg.maskdino import MaskDINO, MaskDINOCriterion, masks_to_boxes
    cfg = (_tiny(mask_feature_size=128, feature_size=128, hidden_dim=128, dec_heads=4) if precision == "bf16"
           else _tiny())
    m = MaskDINO(cfg).init_weights(0).to(DEV).train()
    if precision == "bf16":
        m = m.to(torch.bfloat16)
    imgs, ml, cl = synthetic_batch(2, 128, seed=4, device=DEV)
    tg = PaddedTargets.from_lists(ml, cl, kc=4, device=DEV)
    boxes = masks_to_boxes(tg.masks)
    res = []
    for fl in (True, False):
        m.zero_grad(set_to_none=True)
        torch.manual_seed(0)
        torch.cuda.manual_seed(0)
        out = m(imgs.to(next(m.parameters()).dtype), tg, boxes)
        loss, _ = MaskDINOCriterion(cfg, factor_losses=fl)(out, tg, boxes)
        loss.backward()
        res.append((float(loss), {n: p.grad.float().clone() for n, p in m.named_parameters() if p.grad is not None}))
    (l1, g1), (l2, g2) = res
    assert abs(l1 - l2) <= 1e-5 * abs(l2), (l1, l2)
    assert set(g1) == set(g2)
    tol = 2e-2 if precision == "bf16" else 1e-4
    # Structural zeros: an attention key bias adds the same constant to every score of a
    # query's row, which softmax cancels, so its exact gradient is 0 and both paths give
    # pure rounding noise (bf16: ~1e-6-1e-5 norms).  Those are checked in ABSOLUTE terms
    # against the model's gradient scale; every other parameter relatively, with a norm
    # floor of 1e-2 x the median parameter-gradient norm (no gate divides by ~0).
    gnorm = float(torch.sqrt(sum((g.double() ** 2).sum() for g in g2.values())))
    # (a key bias is a structural zero where its softmax runs over the keys it feeds: the
    # decoders' self-attention; identified by the reference path's gradient being ~0)
    zero = {n for n in g2 if n.endswith("k_proj.bias") and float(g2[n].norm()) <= 1e-4 * gnorm}
    floor = 1e-2 * float(np.median([float(g2[n].norm()) for n in g2]))
    zmax = max([max(float(g1[n].norm()), float(g2[n].norm())) for n in zero] + [0.0])
    errs = sorted(((float((g1[n] - g2[n]).norm()) / max(float(g2[n].norm()), floor), n) for n in g2 if n not in zero),
                  reverse=True)
    worst = errs[0][0]
    print(f"maskdino {precision}: factor vs full-logit mask losses, loss {l1:.6f} / {l2:.6f}, worst grad rel-L2 "
          f"{worst:.2e}; {[(f'{e:.1e}', n, float(g2[n].norm())) for e, n in errs[:6]]}; structural zeros "
          f"{len(zero)}: max norm {zmax:.2e} of global {gnorm:.2e}")
    assert worst <= tol
    assert zmax <= 1e-3 * gnorm


def test_factor_matcher_equals_full_logit_matcher():
    """MaskDINOCriterion.match with the mask costs from the mask head's factors
    (csrc/match_factors.hip over E_s . F(p)) vs point-sampling the full logits: the same
    assignment on a bf16 forward (mask features of 128 channels)."""
    from visionseg.criterion import PaddedTargets
    from visionseg.data import synthetic_batch
    from visionseg.maskdino import MaskDINO, MaskDINOCriterion, masks_to_boxes
    cfg = _tiny(mask_feature_size=128, feature_size=128, hidden_dim=128, dec_heads=4)
    m = MaskDINO(cfg).init_weights(0).to(DEV).to(torch.bfloat16).train()
    imgs, ml, cl = synthetic_batch(2, 128, seed=6, device=DEV)
    tg = PaddedTargets.from_lists(ml, cl, kc=4, device=DEV)
    boxes = masks_to_boxes(tg.masks)
    with torch.no_grad():
        out = m(imgs.to(torch.bfloat16), tg, boxes)
    pad = out["dn"]["pad"]
    S = len(out["classes"])
    cls_m = torch.stack([x[:, pad:] for x in out["classes"]] + [out["interm"]["classes"]])
    box_m = torch.stack([x[:, pad:] for x in out["boxes"]] + [out["interm"]["boxes"]])
    masks_m = [x[:, pad:] for x in out["masks"]] + [out["interm"]["masks"]]
    srcs = [mk._vs_src for mk in out["masks"]] + [out["interm"]["masks"]._vs_src]
    fulls = out["masks"] + [out["interm"]["masks"]]
    facs = [(sr[0], sr[1], pad if i < S else 0, None, fulls[i]) for i, sr in enumerate(srcs)]
    crit = MaskDINOCriterion(cfg)
    got = []
    for f in (facs, None):
        torch.cuda.manual_seed(11)
        got.append(crit.match(cls_m, box_m, masks_m, tg, boxes, f))
    assert torch.equal(got[0], got[1])
