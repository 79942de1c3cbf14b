"""Host-side logic on CPU: COCO data path, mask-AP evaluator, state-dict conversion,
LR schedule, instance post-processing."""
import json
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from visionseg.data import write_coco_dataset, CocoInstanceDataset, collate_padded, synthetic_batch, normalize
from visionseg.evaluate import MaskAPEvaluator
from visionseg.convert import from_hf_state_dict, to_hf_state_dict
from visionseg.model import M2FConfig, Mask2Former
from visionseg.train import SolverConfig, lr_at
from visionseg.inference import instance_inference


def test_coco_roundtrip(tmp_path):
    coco = write_coco_dataset(str(tmp_path), n_images=3, size=96, seed=1)
    assert set(coco) == {"images", "annotations", "categories"}
    ds = CocoInstanceDataset(str(tmp_path), train=False, keep_size=True)
    assert len(ds) == 3
    img, m, c = ds[0]
    assert img.dtype == torch.uint8 and img.shape == (3, 96, 96)
    assert m.dtype == torch.bool and m.shape[1:] == (96, 96) and m.shape[0] == c.shape[0] >= 1
    assert (c == 0).all()
    # annotation areas match the rasterised masks
    areas = [a["area"] for a in coco["annotations"] if a["image_id"] == 0]
    assert np.allclose(sorted(areas), sorted(m.flatten(1).sum(1).tolist()))
    ds2 = CocoInstanceDataset(str(tmp_path), min_size=(64,), max_size=80, train=True, seed=0)
    batch = collate_padded([ds2[0], ds2[1]])
    assert batch[0].shape[-1] % 32 == 0 and batch[0].shape[-2] % 32 == 0
    assert batch[1][0].shape[-2:] == batch[0].shape[-2:]


def test_synthetic_batch_shapes():
    imgs, ml, cl = synthetic_batch(2, 128, seed=42)
    assert imgs.shape == (2, 3, 128, 128) and imgs.dtype == torch.float32
    for m, c in zip(ml, cl):
        assert 1 <= m.shape[0] <= 3 and m.shape[0] == c.shape[0]
        frac = m.float().mean((1, 2))
        assert bool(((frac > 0.001) & (frac < 0.2)).all())
    n = normalize(torch.full((1, 3, 2, 2), 128, dtype=torch.uint8))[0, :, 0, 0]
    assert torch.allclose(n, torch.tensor([(128 - 123.675) / 58.395, (128 - 116.28) / 57.12, (128 - 103.53) / 57.375]))


def test_mask_ap_evaluator():
    g = torch.Generator().manual_seed(0)
    gt = torch.zeros(3, 32, 32, dtype=torch.bool)
    gt[0, 2:10, 2:10] = True
    gt[1, 15:30, 5:12] = True
    gt[2, 20:25, 20:31] = True
    lab = torch.zeros(3, dtype=torch.int64)
    ev = MaskAPEvaluator(1)
    ev.add(torch.tensor([0.9, 0.8, 0.7]), lab, gt.clone(), gt, lab)
    r = ev.summarize()
    assert r["mAP"] == pytest.approx(1.0) and r["mAP50"] == pytest.approx(1.0)
    assert r["precision"] == 1.0 and r["recall"] == 1.0
    ev = MaskAPEvaluator(1)
    pred = gt.clone()
    pred[0] = False
    pred[0, 2:10, 2:7] = True            # IoU 5/8 = 0.625
    ev.add(torch.tensor([0.9, 0.8, 0.7]), lab, pred, gt, lab)
    r = ev.summarize()
    assert r["mAP50"] == pytest.approx(1.0)
    assert r["mAP75"] < 1.0 and 0.5 < r["mAP"] < 1.0
    ev = MaskAPEvaluator(1)
    ev.add(torch.zeros(0), torch.zeros(0, dtype=torch.int64), torch.zeros(0, 32, 32, dtype=torch.bool), gt, lab)
    assert ev.summarize()["mAP"] == 0.0


def test_state_dict_conversion_roundtrip():
    cfg = M2FConfig(embed_dim=32, depths=(2, 2, 2, 2), num_heads=(1, 2, 4, 8), feature_size=64, mask_feature_size=64,
                    hidden_dim=64, enc_ffn=128, dec_ffn=128, dec_heads=2, enc_layers=2, dec_layers=4, num_queries=10)
    sd = Mask2Former(cfg).init_weights(0).state_dict()
    hf = to_hf_state_dict(sd)
    assert any(k.endswith("attention.q_proj.weight") for k in hf)
    back = from_hf_state_dict(hf)
    assert set(back) == set(sd) and all(torch.equal(back[k], sd[k]) for k in sd)


def test_lr_schedules():
    s = SolverConfig(warmup_iters=200, steps=(3500, 4500), lr=1.0)
    f = lambda it: lr_at(s, it)  # noqa: E731
    assert f(0) == pytest.approx(0.001) and f(200) == 1.0 and f(3600) == pytest.approx(0.1) and f(4600) == pytest.approx(0.01)
    sc = SolverConfig(warmup_iters=0, schedule="cosine", max_iter=100, lr=1.0)
    c = lambda it: lr_at(sc, it)  # noqa: E731
    assert c(0) == 1.0 and c(50) == pytest.approx(0.5) and c(100) == pytest.approx(0.0, abs=1e-12)


def test_instance_inference():
    Q, K = 4, 1
    ml = torch.full((Q, 8, 8), -5.0)
    ml[1, 2:6, 2:6] = 5.0
    cl = torch.tensor([[0.0, 3.0], [4.0, 0.0], [0.0, 0.0], [-2.0, 2.0]])
    s, lab, m = instance_inference(ml, cl, (32, 32))
    assert m.shape == (4, 32, 32) and m.dtype == torch.bool
    best = int(torch.argmax(s))
    assert m[best].sum() > 0 and (lab == 0).all()
    assert float(s.max()) > 0.9


def _pair_independent_rand(monkeypatch):
    """torch.rand whose point draws depend only on the point index, not on the number of
    (step, image, target) pairs: a loss over padded pairs is then comparable bit for bit
    with a loss over fewer pairs."""
    base = torch.rand(200000, 2, generator=torch.Generator().manual_seed(9))

    def fake_rand(*shape, device=None, generator=None, **kw):
        if len(shape) == 1 and isinstance(shape[0], (tuple, list)):
            shape = tuple(shape[0])
        n = shape[-2]
        return base[:n].expand(*shape[:-2], n, 2).clone().to(device if device is not None else "cpu")
    monkeypatch.setattr(torch, "rand", fake_rand)


@pytest.mark.parametrize("ks", [[2, 0, 3], [1, 1], [0, 0], [3, 1, 2, 0]])
def test_criterion_padding_invariance(monkeypatch, ks):
    """Padded targets (criterion.PaddedTargets, what a graph-replayed step feeds the
    criterion) give the same matching, loss and gradients whatever the padded capacity,
    and the same as the reference's per-image lists (HF:m2f:378-794 semantics)."""
    from visionseg.criterion import SetCriterion, PaddedTargets
    cfg = M2FConfig.preset("swin_t", num_queries=12, train_num_points=256)
    g = torch.Generator().manual_seed(sum(ks) + len(ks))
    S, B, Q, H = 3, len(ks), 12, 32
    masks = [torch.randn(B, Q, H, H, generator=g, requires_grad=True) for _ in range(S)]
    classes = [torch.randn(B, Q, 2, generator=g, requires_grad=True) for _ in range(S)]
    ml = [torch.rand(k, 96, 96, generator=g) > 0.7 for k in ks]
    cl = [torch.zeros(k, dtype=torch.int64) for k in ks]
    _pair_independent_rand(monkeypatch)
    res = []
    for tg in ((ml, cl), (PaddedTargets.from_lists(ml, cl), None), (PaddedTargets.from_lists(ml, cl, kc=5), None)):
        crit = SetCriterion(cfg, matcher="host")
        assign = crit.match([m.detach() for m in masks], torch.stack(classes).detach(), *tg)
        loss, parts = crit(masks, classes, *tg)
        grads = torch.autograd.grad(loss, masks + classes)
        res.append((assign, loss.detach(), grads))
    kmax = max(ks)
    for i, (assign, loss, grads) in enumerate(res[1:]):
        assert torch.equal(assign[..., :kmax], res[0][0][..., :kmax])
        assert (assign[..., kmax:] == -1).all()
        if i == 0:      # same capacity: bit-identical
            assert torch.equal(loss, res[0][1])
            assert all(torch.equal(a, b) for a, b in zip(grads, res[0][2]))
        else:           # extra zero pairs change only the summation tree
            assert abs(float(loss) - float(res[0][1])) <= 1e-6 * abs(float(res[0][1]))
            for a, b in zip(grads, res[0][2]):
                assert float((a - b).abs().max()) <= 1e-6 * max(1e-6, float(b.abs().max()))
    # every valid target matched to a distinct query
    a = res[0][0]
    for s in range(S):
        for b, k in enumerate(ks):
            q = a[s, b, :k].tolist()
            assert len(set(q)) == k and all(0 <= x < Q for x in q)


def test_instance_inference_vs_hf_postprocess(golden):
    """visionseg.inference.instance_inference vs HF post_process_instance_segmentation
    (HF:m2f-proc:627-746), fixture tests/golden/postproc.npz (gen_golden.py): HF resizes
    the logits to 384^2 and keeps the instances scoring >= threshold; the same selection
    from the product's output gives the same scores, labels and binary masks."""
    d = golden("postproc.npz")
    thr = float(d["threshold"])
    for i in range(d["class_queries_logits"].shape[0]):
        s, lab, m = instance_inference(torch.from_numpy(d["masks_queries_logits"][i]),
                                       torch.from_numpy(d["class_queries_logits"][i]), (384, 384))
        keep = (s >= thr) & m.flatten(1).any(1)
        got = sorted(zip(np.round(s[keep].numpy().astype(np.float64), 6).tolist(), lab[keep].tolist(),
                         [np.packbits(x, axis=-1).tobytes() for x in m[keep].numpy()]))
        exp_maps = d[f"binary_maps_{i}"]
        exp = sorted(zip(d[f"scores_{i}"].tolist(), d[f"labels_{i}"].tolist(), [x.tobytes() for x in exp_maps]))
        assert len(got) == len(exp)
        for (gs, gl, gm), (es, el, em) in zip(got, exp):
            assert abs(gs - es) <= 2e-6 and gl == el and gm == em


def test_predictor_crop_follows_sem_seg_postprocess():
    """Stride-4 logits -> padded input size -> crop -> original size (upstream
    sem_seg_postprocess), for sizes that are not multiples of 4."""
    g = torch.Generator().manual_seed(0)
    ml = torch.randn(3, 25, 40, generator=g)            # stride 4 of a 100 x 160 padded input
    cl = torch.randn(3, 2, generator=g)
    s, lab, m = instance_inference(ml, cl, (77, 130), valid_hw=(97, 158), pad_hw=(100, 160))
    up = F.interpolate(ml[None], size=(100, 160), mode="bilinear", align_corners=False)[..., :97, :158]
    exp = F.interpolate(up, size=(77, 130), mode="bilinear", align_corners=False)[0] > 0
    order = torch.softmax(cl, -1)[:, 0].topk(3, sorted=False)[1]
    assert torch.equal(m, exp[order])


def _rle_encode(mask):
    """Uncompressed COCO RLE of a bool mask (column-major runs, background first) and
    its compressed string (pycocotools rleToString semantics), for the decoder test."""
    flat = mask.T.reshape(-1).astype(np.uint8)
    counts, cur, n = [], 0, 0
    for v in flat:
        if v != cur:
            counts.append(n)
            cur, n = v, 0
        n += 1
    counts.append(n)
    s = []
    for i, x in enumerate(counts):
        x = x - counts[i - 2] if i > 2 else x
        more = True
        while more:
            c = x & 0x1F
            x >>= 5
            more = (x != -1) if (c & 0x10) else (x != 0)
            if more:
                c |= 0x20
            s.append(chr(c + 48))
    return {"counts": counts, "size": list(mask.shape)}, {"counts": "".join(s), "size": list(mask.shape)}


def test_rle_annotations(tmp_path):
    """CocoInstanceDataset decodes RLE segmentations (uncompressed and compressed COCO
    strings) as the reference mapper does (train_full.py:116-129)."""
    from visionseg.data import decode_rle
    rng = np.random.default_rng(3)
    m = np.zeros((37, 53), dtype=bool)
    m[5:20, 8:30] = True
    m[25:33, 40:50] = rng.random((8, 10)) > 0.3
    un, comp = _rle_encode(m)
    assert np.array_equal(decode_rle(un), m) and np.array_equal(decode_rle(comp), m)
    coco = write_coco_dataset(str(tmp_path), n_images=1, size=64, seed=2)
    big = np.zeros((64, 64), dtype=bool)
    big[10:30, 20:50] = True
    coco["annotations"].append({"id": 999, "image_id": 0, "category_id": 0, "segmentation": _rle_encode(big)[1],
                                "area": float(big.sum()), "bbox": [20, 10, 30, 20], "iscrowd": 0})
    with open(os.path.join(str(tmp_path), "annotations.json"), "w") as f:
        json.dump(coco, f)
    ds = CocoInstanceDataset(str(tmp_path), train=False, keep_size=True)
    _, masks, classes = ds[0]
    assert any(np.array_equal(x.numpy(), big) for x in masks)


def test_prefetch_loader_matches_serial_batches(tmp_path):
    """visionseg.data.PrefetchLoader (2 worker processes, host collate + device-side
    normalisation) yields the serial loop's batches: same per-epoch seeded permutation,
    rank slots, padding and normalisation as collate_padded (no random augmentation here:
    train=False), across an epoch boundary and for rank 1 of 2."""
    from visionseg.data import PrefetchLoader
    write_coco_dataset(str(tmp_path), 7, 96, seed=1)
    ds = CocoInstanceDataset(str(tmp_path), train=False, fixed_size=96)
    for rank, world in ((0, 1), (1, 2)):
        per_rank, iters = 2, 5
        ld = PrefetchLoader(ds, per_rank, iters, rank=rank, world=world, seed=5, num_workers=2, device="cpu")
        rng = np.random.default_rng(5)
        epoch_iters = -(-len(ds) // (per_rank * world))
        got = list(ld)
        assert len(got) == iters
        k = 0
        while k < iters:
            order = rng.permutation(len(ds))
            for j in range(epoch_iters):
                if k >= iters:
                    break
                a = (j * world + rank) * per_rank
                idx = order[a:a + per_rank]
                if len(idx) == 0:
                    idx = order[:per_rank]
                ei, em, ec = collate_padded([ds[int(i)] for i in idx])
                gi, gm, gc = got[k]
                assert torch.allclose(gi, ei) and all(torch.equal(x, y) for x, y in zip(gm, em))
                assert all(torch.equal(x, y) for x, y in zip(gc, ec))
                k += 1


def test_pad_buckets_and_mixed_aspect_loader(tmp_path):
    """The seam's padding canvases: (512, 640, 800) for the reference's MIN_SIZE_TRAIN
    480..640 / MAX_SIZE_TRAIN 800 (train_full.py:244-245); a bucketed batch equals the
    detectron2-padded batch zero-extended to the canvas (image and masks), so only the
    amount of zero padding changes; multi-scale mixed-aspect data gives at most 9 shapes."""
    from visionseg.adapters import MAX_SIZE_TRAIN, MIN_SIZE_TRAIN
    from visionseg.data import PrefetchLoader, bucket_size, default_pad_buckets
    bk = default_pad_buckets(MIN_SIZE_TRAIN, MAX_SIZE_TRAIN)
    assert bk == (512, 640, 800)
    assert [bucket_size(n, 32, bk) for n in (480, 481, 512, 513, 640, 641, 800, 801)] == \
        [512, 512, 512, 640, 640, 800, 800, 832]
    assert bucket_size(481) == 512 and bucket_size(480) == 480
    write_coco_dataset(str(tmp_path), 12, [(120, 160), (160, 120), (100, 100)], seed=2)
    ds = CocoInstanceDataset(str(tmp_path), min_size=(60, 64, 68, 72, 76, 80), max_size=100, train=True, seed=4)
    small = default_pad_buckets(ds.min_size, ds.max_size)
    assert small == (64, 96, 128)     # 64, 80 -> 96, 100 -> 128 (rounded to 32)
    shapes = set()
    for buckets in (None, small):
        ds.rng = np.random.default_rng(4)
        ld = PrefetchLoader(ds, 3, 8, seed=5, num_workers=0, device="cpu", pad_buckets=buckets)
        for imgs, masks, classes in ld:
            H, W = imgs.shape[-2:]
            if buckets:
                assert H in small and W in small
                shapes.add((H, W))
            assert all(m.shape[-2:] == (H, W) for m in masks)
    assert len(shapes) <= 9
    # bucketed == exact padding, zero-extended
    ds.rng = np.random.default_rng(9)
    samples = [ds[i] for i in range(3)]
    from visionseg.data import collate_host
    ei, es, em, ec = collate_host(samples)
    bi, bs, bm, bc = collate_host(samples, buckets=small)
    h, w = ei.shape[-2:]
    assert torch.equal(bi[..., :h, :w], ei) and int(bi[..., h:, :].sum()) == 0 and int(bi[..., :, w:].sum()) == 0
    assert torch.equal(es, bs) and all(torch.equal(x[:, :h, :w], y) and not x[:, h:].any() for x, y in zip(bm, em))


def test_factored_list_validation():
    """ops.factored accepts only the decoder's own factored output (one entry per step of E,
    the same E / F objects, entry s = step s); a subset or a reordered list is not treated
    as factored (its consumers materialise it instead)."""
    from visionseg import ops
    E = torch.zeros(3, 2, 5, 8)
    Fm = torch.zeros(2, 16, 8)
    full = [ops.FactoredLogits(E, Fm, s, 4, 4) for s in range(3)]
    assert ops.factored(full)
    assert ops.factored([m.detach() for m in full])        # detached views of the same factors
    assert not ops.factored(full[1:])                       # a subset (last steps only)
    assert not ops.factored([full[1], full[0], full[2]])    # reordered
    assert not ops.factored(full[:2] + [ops.FactoredLogits(E.clone(), Fm, 2, 4, 4)])
    assert not ops.factored([])
    assert full[0].shape == (2, 5, 4, 4)


@pytest.mark.gpu
def test_decoder_returns_tensors_by_default():
    """Mask2Former.forward keeps its contract ([B,Q,H/4,W/4] f32 tensors) with grad on, in
    train() and eval(): factored logits are only for a consumer that asks for them
    (decoder.emit_factors, set by train.Trainer for the visionseg SetCriterion)."""
    from visionseg.criterion import SetCriterion
    cfg = M2FConfig(embed_dim=32, depths=(1, 1, 1, 1), num_heads=(1, 2, 4, 8), feature_size=128,
                    mask_feature_size=128, hidden_dim=128, enc_ffn=64, dec_ffn=64, dec_heads=4, enc_layers=1,
                    dec_layers=2, num_queries=4, train_num_points=64)      # 128 channels: the factorable width
    m = Mask2Former(cfg).cuda().to(torch.bfloat16)
    assert m.decoder.emit_factors is False
    assert SetCriterion.accepts_factored_logits
    for mode in (True, False):
        m.train(mode)
        masks, classes = m(torch.randn(1, 3, 64, 64, device="cuda"))
        assert all(isinstance(x, torch.Tensor) and x.shape == (1, 4, 16, 16) for x in masks)
