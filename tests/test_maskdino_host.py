"""MaskDINO host logic on CPU (config C4, row f3): box utilities, anchor proposals,
denoising-query construction and its attention mask, the focal loss and the criterion
(matching + losses) on synthetic predictions.  Parity is UNPINNED: no MaskDINO source
exists in the container, so these are properties of the published
algorithm (upstream maskdino/modeling/transformer_decoder/maskdino_decoder.py,
criterion.py, matcher.py), not comparisons against a reference run."""
import itertools
import math

import numpy as np
import pytest
import torch

from visionseg.criterion import PaddedTargets
from visionseg.maskdino import (MaskDINOConfig, MaskDINOCriterion, MaskDINODecoder, box_cxcywh_to_xyxy,
                                generalized_box_iou, inverse_sigmoid, masks_to_boxes, sigmoid_focal_loss,
                                sine_embed_boxes)


def _tiny_cfg(**kw):
    d = dict(embed_dim=32, depths=(2, 2, 2, 2), num_heads=(1, 2, 4, 8), feature_size=64, mask_feature_size=64,
             hidden_dim=64, enc_ffn=128, dec_ffn=128, dec_heads=2, enc_layers=1, dec_layers=3, num_queries=12,
             num_labels=2, dn_num=8, train_num_points=64)
    d.update(kw)
    return MaskDINOConfig(**d)


def test_giou_matches_definition():
    g = torch.Generator().manual_seed(0)
    a = torch.rand(5, 4, generator=g)
    b = torch.rand(7, 4, generator=g)
    a = box_cxcywh_to_xyxy(torch.cat((a[:, :2], a[:, 2:] * 0.5 + 0.05), 1))
    b = box_cxcywh_to_xyxy(torch.cat((b[:, :2], b[:, 2:] * 0.5 + 0.05), 1))
    got = generalized_box_iou(a, b)
    for i, j in itertools.product(range(5), range(7)):
        x0, y0 = max(a[i, 0], b[j, 0]), max(a[i, 1], b[j, 1])
        x1, y1 = min(a[i, 2], b[j, 2]), min(a[i, 3], b[j, 3])
        inter = max(0.0, float(x1 - x0)) * max(0.0, float(y1 - y0))
        aa = float((a[i, 2] - a[i, 0]) * (a[i, 3] - a[i, 1]))
        ab = float((b[j, 2] - b[j, 0]) * (b[j, 3] - b[j, 1]))
        union = aa + ab - inter
        hull = float((max(a[i, 2], b[j, 2]) - min(a[i, 0], b[j, 0])) * (max(a[i, 3], b[j, 3]) - min(a[i, 1], b[j, 1])))
        assert abs(float(got[i, j]) - (inter / union - (hull - union) / hull)) < 1e-6
    assert torch.allclose(torch.diagonal(generalized_box_iou(a, a)), torch.ones(5))


def test_masks_to_boxes():
    m = torch.zeros(2, 3, 40, 60, dtype=torch.bool)
    m[0, 0, 10:20, 5:35] = True
    m[1, 2, 0:40, 59:60] = True
    b = masks_to_boxes(m)
    assert torch.allclose(b[0, 0], torch.tensor([20 / 60, 15 / 40, 30 / 60, 10 / 40]))
    assert torch.allclose(b[1, 2], torch.tensor([59.5 / 60, 0.5, 1 / 60, 1.0]))
    assert float(b[0, 1].abs().sum()) == 0.0                       # empty mask


def test_sine_embedding_and_inverse_sigmoid():
    bx = torch.tensor([[0.25, 0.5, 0.1, 0.2]])
    e = sine_embed_boxes(bx, 64)
    assert e.shape == (1, 128)
    # first block is y: sin(y * 2pi / 1), cos(...)
    assert abs(float(e[0, 0]) - math.sin(0.5 * 2 * math.pi)) < 1e-6
    assert abs(float(e[0, 32]) - math.sin(0.25 * 2 * math.pi)) < 1e-6
    x = torch.tensor([0.1, 0.5, 0.9])
    assert torch.allclose(inverse_sigmoid(x).sigmoid(), x, atol=1e-6)


def test_proposals_and_dn_queries():
    cfg = _tiny_cfg()
    dec = MaskDINODecoder(cfg)
    unsig, valid = dec._proposals([(2, 2), (4, 4)], torch.device("cpu"))
    assert unsig.shape == (20, 4) and valid.shape == (20,)
    p = unsig[valid].sigmoid()
    assert torch.allclose(p[0], torch.tensor([0.25, 0.25, 0.05, 0.05]), atol=1e-6)
    # dn: counts 2 and 1, capacity 4 (bucketed) -> K = 2: 8 // 2 = 4 groups of 2 slots
    ml = [torch.zeros(2, 16, 16, dtype=torch.bool), torch.zeros(1, 16, 16, dtype=torch.bool)]
    ml[0][0, 2:8, 2:8] = True
    ml[0][1, 10:14, 3:9] = True
    ml[1][0, 5:9, 5:9] = True
    cl = [torch.tensor([0, 1]), torch.tensor([1])]
    tg = PaddedTargets.from_lists(ml, cl, kc=4)
    boxes = masks_to_boxes(tg.masks)
    torch.manual_seed(0)
    emb, unsig_dn, blocked, meta = dec._dn(tg, boxes, 2, torch.device("cpu"), torch.float32)
    assert int(meta["groups"]) == 4 and meta["pad"] == 8 and bool(meta["active"].all())
    assert meta["slot"].tolist() == [0, 1] * 4
    assert emb.shape == (2, 8, 64) and unsig_dn.shape == (2, 8, 4)
    valid_dn = meta["valid"]
    assert valid_dn.tolist() == [[True, True] * 4, [True, False] * 4]
    assert float(emb[~valid_dn].abs().sum()) == 0.0 and float(unsig_dn[~valid_dn].abs().sum()) == 0.0
    Qt = 8 + cfg.num_queries
    assert blocked.shape == (Qt, Qt)
    # matching queries see each other but no DN query; DN groups see only themselves
    assert not blocked[8:, 8:].any() and blocked[8:, :8].all()
    for gi in range(4):
        lo, hi = 2 * gi, 2 * gi + 2
        assert not blocked[lo:hi, lo:hi].any()
        assert blocked[lo:hi, :lo].all() and blocked[lo:hi, hi:8].all()
    assert not blocked[:8, 8:].any()
    # noised boxes stay in the unit square, near their targets
    bx = unsig_dn.sigmoid()[valid_dn]
    tb = boxes[:, :2].repeat(1, 4, 1)[valid_dn]
    assert bool(((bx >= 0) & (bx <= 1)).all())
    assert float((bx - tb).abs().max()) <= cfg.noise_scale * float(tb[:, 2:].max()) + 1e-5


def test_dn_layout_independent_of_target_capacity():
    """Eager steps pad the targets to the batch's largest count, graph-replayed steps to
    a multiple of 4 (train.Trainer.target_capacity): the denoising layout (groups, slots,
    validity, attention mask, noised queries) must be the same for both (upstream
    prepare_for_dn: dn_num // max count groups)."""
    cfg = _tiny_cfg(dn_num=8)
    dec = MaskDINODecoder(cfg)
    ml, cl = _targets(B=3)                      # counts 2, 1, 3 -> K = 3: 2 groups, 2 inactive queries
    res = []
    for kc in (3, 4, 8):
        tg = PaddedTargets.from_lists(ml, cl, kc=kc)
        boxes = masks_to_boxes(tg.masks)
        torch.manual_seed(7)
        res.append(dec._dn(tg, boxes, 3, torch.device("cpu"), torch.float32))
    for emb, unsig, blocked, meta in res[1:]:
        assert torch.equal(emb, res[0][0]) and torch.equal(unsig, res[0][1]) and torch.equal(blocked, res[0][2])
        for k in ("slot", "active", "valid"):
            assert torch.equal(meta[k], res[0][3][k])
    meta, blocked = res[0][3], res[0][2]
    assert int(meta["groups"]) == 2 and meta["active"].tolist() == [True] * 6 + [False] * 2
    assert meta["valid"][2].tolist() == [True] * 6 + [False] * 2
    assert meta["valid"][1].tolist() == [True, False, False] * 2 + [False] * 2
    # an inactive query is seen by nobody else and sees no other DN query
    for q in (6, 7):
        others = [j for j in range(8 + cfg.num_queries) if j != q]
        assert blocked[others, q].all() and blocked[q, [j for j in range(8) if j != q]].all()
    # no targets anywhere (a graph step's padded capacity): every DN query inactive
    tg = PaddedTargets.from_lists([torch.zeros(0, 96, 96, dtype=torch.bool)] * 2,
                                  [torch.zeros(0, dtype=torch.int64)] * 2, kc=4)
    _, _, blocked, meta = dec._dn(tg, masks_to_boxes(tg.masks), 2, torch.device("cpu"), torch.float32)
    assert not meta["valid"].any() and not meta["active"].any() and blocked[8:, :8].all()


def test_focal_loss_formula():
    x = torch.tensor([[-2.0, 0.5], [3.0, -1.0]])
    t = torch.tensor([[0.0, 1.0], [1.0, 0.0]])
    got = sigmoid_focal_loss(x, t, 0.25, 2.0)
    p = x.sigmoid()
    exp = torch.where(t > 0, -0.25 * (1 - p) ** 2 * p.log(), -0.75 * p ** 2 * (1 - p).log())
    assert torch.allclose(got, exp, atol=1e-6)


def _fake_outputs(cfg, tg, boxes, dec, B, H=24, seed=0, dn=True):
    g = torch.Generator().manual_seed(seed)
    meta = None
    pad = 0
    if dn:
        torch.manual_seed(seed)
        _, _, _, meta = dec._dn(tg, boxes, B, torch.device("cpu"), torch.float32)
        pad = meta["pad"]
    Qt = pad + cfg.num_queries
    S = cfg.dec_layers + 1
    mk = lambda *s: torch.randn(*s, generator=g).requires_grad_(True)  # noqa: E731
    out = dict(classes=[mk(B, Qt, cfg.num_labels) for _ in range(S)],
               masks=[mk(B, Qt, H, H) for _ in range(S)],
               boxes=[torch.rand(B, Qt, 4, generator=g).mul(0.5).add(0.1).requires_grad_(True) for _ in range(S)],
               interm=dict(classes=mk(B, cfg.num_queries, cfg.num_labels), masks=mk(B, cfg.num_queries, H, H),
                           boxes=torch.rand(B, cfg.num_queries, 4, generator=g).mul(0.5).add(0.1)), dn=meta)
    return out


def _targets(B=2, seed=1, size=96):
    g = torch.Generator().manual_seed(seed)
    ks = [2, 1, 3][:B]
    ml = []
    for k in ks:
        m = torch.zeros(k, size, size, dtype=torch.bool)
        for i in range(k):
            y, x = torch.randint(0, size // 2, (2,), generator=g).tolist()
            m[i, y:y + 20 + 5 * i, x:x + 15] = True
        ml.append(m)
    cl = [torch.randint(0, 2, (k,), generator=g) for k in ks]
    return ml, cl


def test_criterion_losses_and_matching():
    cfg = _tiny_cfg()
    dec = MaskDINODecoder(cfg)
    ml, cl = _targets()
    tg = PaddedTargets.from_lists(ml, cl, kc=4)
    boxes = masks_to_boxes(tg.masks)
    out = _fake_outputs(cfg, tg, boxes, dec, 2)
    crit = MaskDINOCriterion(cfg, matcher="host")
    loss, parts = crit(out, tg, boxes)
    S = cfg.dec_layers + 1
    assert torch.isfinite(loss)
    for pre in ("loss_ce", "loss_bbox", "loss_giou", "loss_mask", "loss_dice"):
        assert pre in parts and f"{pre}_interm" in parts and f"{pre}_dn" in parts and f"{pre}_0" in parts
    assert len(parts) == 5 * (S + 1) + 5 * S
    grads = torch.autograd.grad(loss, out["classes"] + out["masks"] + out["boxes"])
    assert all(torch.isfinite(x).all() for x in grads)
    # matching = the optimum of the cost it builds (brute force on one image / step)
    cls_m = torch.stack([x[:, out["dn"]["pad"]:] for x in out["classes"]]).detach()
    box_m = torch.stack([x[:, out["dn"]["pad"]:] for x in out["boxes"]]).detach()
    masks_m = [x[:, out["dn"]["pad"]:].detach() for x in out["masks"]]
    torch.manual_seed(3)
    a1 = crit.match(cls_m, box_m, masks_m, tg, boxes)
    for s, b in itertools.product(range(S), range(2)):
        q = a1[s, b, :len(cl[b])].tolist()
        assert len(set(q)) == len(q) and all(0 <= x < cfg.num_queries for x in q)
        assert (a1[s, b, len(cl[b]):] == -1).all()


def test_criterion_without_targets_and_without_dn():
    cfg = _tiny_cfg()
    dec = MaskDINODecoder(cfg)
    ml = [torch.zeros(0, 96, 96, dtype=torch.bool)] * 2
    cl = [torch.zeros(0, dtype=torch.int64)] * 2
    tg = PaddedTargets.from_lists(ml, cl)
    boxes = masks_to_boxes(tg.masks)
    out = _fake_outputs(cfg, tg, boxes, dec, 2, dn=False)
    loss, parts = MaskDINOCriterion(cfg, matcher="host")(out, tg, boxes)
    assert torch.isfinite(loss) and all(k.startswith("loss_ce") for k in parts)
    ml, cl = _targets()
    tg = PaddedTargets.from_lists(ml, cl)
    boxes = masks_to_boxes(tg.masks)
    out = _fake_outputs(cfg, tg, boxes, dec, 2, dn=False)
    loss, parts = MaskDINOCriterion(cfg, matcher="host")(out, tg, boxes)
    assert torch.isfinite(loss) and not any("_dn" in k for k in parts)


def test_init_detector_maskdino_backbone_from_config_or_checkpoint(tmp_path):
    """A MaskDINO checkpoint served by init_detector takes its backbone from the config
    argument (object or JSON file) when one is given and from its own backbone tensors
    otherwise -- not silently from the swin_t preset (inference.py)."""
    import json
    from visionseg.inference import backbone_from_state_dict, init_detector
    from visionseg.maskdino import MaskDINO
    # non-backbone parts at the MaskDINO defaults: a checkpoint alone must then be enough
    cfg = MaskDINOConfig(embed_dim=64, depths=(1, 1, 3, 1), num_heads=(2, 4, 8, 16), window_size=5, num_labels=3)
    m = MaskDINO(cfg)
    path = tmp_path / "md.pth"
    torch.save({"model": m.state_dict()}, path)
    got = backbone_from_state_dict(m.state_dict())
    assert got == dict(embed_dim=64, depths=(1, 1, 3, 1), num_heads=(2, 4, 8, 16), window_size=5)
    for config in (None, cfg, str(tmp_path / "c.json")):
        if isinstance(config, str):
            with open(config, "w") as f:
                json.dump(cfg.to_dict(), f)
        det = init_detector(config, str(path), device="cpu")
        c = det.model.cfg
        assert (c.embed_dim, tuple(c.depths), tuple(c.num_heads), c.window_size, c.num_labels) == \
            (64, (1, 1, 3, 1), (2, 4, 8, 16), 5, 3)
    with pytest.raises(ValueError):
        backbone_from_state_dict({"backbone.patch_embed.proj.weight": torch.zeros(8, 3, 4, 4)})


def test_point_sample_rows_matches_grid_sample():
    """The criterion's per-query label sampler (each query reads only its own target map)
    == grid_sample on the gathered maps, incl. points outside [0, 1] and the border."""
    from visionseg.maskdino import _point_sample, _point_sample_rows
    g = torch.Generator().manual_seed(3)
    maps = (torch.rand(6, 17, 23, generator=g) > 0.5).float()
    rows = torch.tensor([0, 5, 2, 2, 3, 1, 4, 0], dtype=torch.int64)
    coords = torch.rand(8, 50, 2, generator=g) * 1.2 - 0.1
    coords[0, :4] = torch.tensor([[0.0, 0.0], [1.0, 1.0], [0.0, 1.0], [1.0, 0.0]])
    exp = _point_sample(maps[rows][:, None], coords)
    got = _point_sample_rows(maps, rows, coords)
    assert float((got - exp).abs().max()) <= 1e-6


def test_criterion_vectorised_equals_per_step():
    """The criterion's class / box losses computed for all decoder steps at once (and the
    DN set's) equal the per-step formulation (`_pair_losses` / `_dn_losses`, one call per
    step) component by component, on the same matching and point draws."""
    cfg = _tiny_cfg()
    dec = MaskDINODecoder(cfg)
    ml, cl = _targets()
    tg = PaddedTargets.from_lists(ml, cl, kc=4)
    boxes = masks_to_boxes(tg.masks)
    out = _fake_outputs(cfg, tg, boxes, dec, 2)
    crit = MaskDINOCriterion(cfg, matcher="host")
    torch.manual_seed(5)
    _, parts = crit(out, tg, boxes)
    # the per-step reference, same RNG order: matcher, then the pair sets, then the DN sets
    torch.manual_seed(5)
    pad = out["dn"]["pad"]
    S = len(out["classes"])
    cls_m = torch.stack([x[:, pad:] for x in out["classes"]] + [out["interm"]["classes"]])
    box_m = torch.stack([x[:, pad:] for x in out["boxes"]] + [out["interm"]["boxes"]])
    masks_m = [x[:, pad:] for x in out["masks"]] + [out["interm"]["masks"]]
    nb = crit._num_boxes(tg)
    assign = crit.match(cls_m.detach(), box_m.detach(), [m.detach() for m in masks_m], tg, boxes)
    valid, tmf = tg.valid(), tg.masks.float()
    ref = {}
    names = [("" if s == S - 1 else f"_{s}") for s in range(S)] + ["_interm"]
    for s, nm in enumerate(names):
        part = crit._pair_losses(cls_m[s], box_m[s], masks_m[s], assign[s].long(), valid & (assign[s] >= 0), tg, tmf,
                                 boxes, nb)
        ref.update({k + nm: v for k, v in part.items()})
    for s in range(S):
        part = crit._dn_losses(out["classes"][s], out["boxes"][s], out["masks"][s], out["dn"], tg, tmf, boxes, nb)
        ref.update({k + ("_dn" if s == S - 1 else f"_dn_{s}"): v for k, v in part.items()})
    assert set(parts) == set(ref)
    for k in ref:
        a, b = float(parts[k]), float(ref[k])
        assert abs(a - b) <= 1e-5 * max(1.0, abs(b)), (k, a, b)
