"""Training seam of training/train_template.py.

The reference dispatches `--model` to `train_<model>(exp_name, train_dir, test_dir,
output_dir, hyperparams) -> dict` (training/train_template.py:104, 197-205) and writes
the returned metrics (`mAP50, mAP75, mAP, precision, recall`, :139-145) plus
exp_name / model_type / hyperparams to `output_dir/results.json` (:207-214).  Its
MaskDINO slot is a stub returning zeros (:104-145).  `train_maskdino` implements that
contract on the MI355X path with the MaskDINO decoder (visionseg.maskdino: Swin backbone,
4-level deformable encoder, two-stage query selection, denoising queries, box
refinement; parity unpinned), `train_mask2former` with Mask2Former (the
`--model mask2former` branch); both read the COCO json in `train_dir/annotations.json`
through the prefetching loader (visionseg.data.PrefetchLoader: worker processes, pinned
host batches, H2D one batch ahead on a side stream) and evaluate mask AP on `test_dir`.
Missing annotations -> None, as the caller expects (:188-194).

Multi-GPU: run the caller under torchrun; images are sharded by rank, gradients are
all-reduced by the Trainer (RCCL), rank 0 writes checkpoints and evaluates.
"""
from __future__ import annotations

import math
import os
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

from .criterion import SetCriterion
from .data import CocoInstanceDataset, PrefetchLoader, default_pad_buckets
from .evaluate import MaskAPEvaluator
from .inference import Predictor
from .model import M2FConfig, Mask2Former
from .train import SolverConfig, Trainer, init_distributed

HYPERPARAMS = {   # defaults of training/train_template.py:45-57
    "epochs": 100, "batch_size": 8, "learning_rate": 1e-4, "weight_decay": 1e-4, "optimizer": "AdamW",
    "lr_scheduler": "cosine", "warmup_epochs": 5, "img_size": 640, "random_seed": 42,
    "early_stopping_patience": 15, "save_period": 10,
}
# INPUT.MIN_SIZE_TRAIN / MAX_SIZE_TRAIN of training/maskdino/train_full.py:244-245 (at
# img_size 640; scaled with img_size otherwise)
MIN_SIZE_TRAIN = (480, 512, 544, 576, 608, 640)
MAX_SIZE_TRAIN = 800


def evaluate_dir(model: Mask2Former, test_dir, img_size: int = 640, device="cuda", max_images: int | None = None):
    """COCO mask AP of `model` on `test_dir/annotations.json` (original resolution)."""
    test_dir = Path(test_dir)
    if not (test_dir / "annotations.json").exists():
        return None
    ds = CocoInstanceDataset(str(test_dir), train=False, keep_size=True)
    pred = Predictor(model, device=device, min_size=img_size, max_size=int(round(img_size * 1.25)))
    ev = MaskAPEvaluator(num_classes=model.cfg.num_labels)
    n = len(ds) if max_images is None else min(len(ds), max_images)
    for i in range(n):
        img, masks, classes = ds[i]
        bgr = img.permute(1, 2, 0).numpy()[:, :, ::-1]
        r = pred(np.ascontiguousarray(bgr)).pred_instances
        ev.add(r.scores, r.labels, r.masks, masks.to(r.masks.device), classes)
    model.train()
    return ev.summarize()


def train_mask2former(exp_name, train_dir, test_dir, output_dir, hyperparams, backbone: str = "swin_t",
                      device=None, max_iters: int | None = None, arch: str = "mask2former", step_callback=None):
    """Multi-scale training as the reference's mapper does it (ResizeShortestEdge over
    MIN_SIZE_TRAIN / MAX_SIZE_TRAIN, random flip; hyperparams "min_size_train",
    "max_size_train" override).  Batches are padded to a few canvases
    (`data.default_pad_buckets`, hyperparams "pad_buckets": a list, or [] for detectron2's
    pad-to-the-batch-max); the trainer keeps one HIP graph per padded shape (LRU, one
    memory pool).  `step_callback(it, trainer, images)` runs after every step (timing
    tools)."""
    hp = dict(HYPERPARAMS)
    hp.update(hyperparams or {})
    train_dir, output_dir = Path(train_dir), Path(output_dir)
    if not (train_dir / "annotations.json").exists():
        print(f"annotations not found: {train_dir / 'annotations.json'}")
        return None
    rank, local, world = init_distributed()
    if device is None:
        device = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
    seed = int(hp["random_seed"])
    torch.manual_seed(seed + rank)
    img = int(hp["img_size"])
    min_sizes = tuple(int(v) for v in hp.get("min_size_train") or
                      [int(round(m * img / 640)) for m in MIN_SIZE_TRAIN])
    max_size = int(hp.get("max_size_train") or int(round(MAX_SIZE_TRAIN * img / 640)))
    pad_buckets = hp.get("pad_buckets", "auto")
    if pad_buckets == "auto":
        pad_buckets = default_pad_buckets(min_sizes, max_size)
    ds = CocoInstanceDataset(str(train_dir), min_size=min_sizes, max_size=max_size, train=True, seed=seed + rank)
    backbone = str(hp.get("backbone", backbone))
    if arch == "maskdino":
        from .maskdino import MaskDINO, MaskDINOConfig, MaskDINOCriterion
        cfg = MaskDINOConfig.preset(backbone, num_labels=max(1, len(ds.cat_to_label)))
        model = MaskDINO(cfg).init_weights(seed)
        criterion = MaskDINOCriterion(cfg)
    else:
        cfg = M2FConfig.preset(backbone, num_labels=max(1, len(ds.cat_to_label)))
        model = Mask2Former(cfg).init_weights(seed)
        criterion = SetCriterion(cfg)
    bs = int(hp["batch_size"])
    per_rank = max(1, bs // world)
    iters_per_epoch = max(1, math.ceil(len(ds) / (per_rank * world)))
    total = iters_per_epoch * int(hp["epochs"])
    if max_iters is not None:
        total = min(total, max_iters)
    solver = SolverConfig(lr=float(hp["learning_rate"]), weight_decay=float(hp["weight_decay"]),
                          optimizer="adamw" if str(hp.get("optimizer", "")).lower() == "adamw" else "sgd",
                          schedule="cosine" if hp.get("lr_scheduler") == "cosine" else "multistep",
                          warmup_iters=int(hp.get("warmup_epochs", 0)) * iters_per_epoch, max_iter=total,
                          amp=device.type == "cuda")
    # HIP-graph replay of the step for every batch signature seen more than twice (image
    # size after ResizeShortestEdge + padding, padded target capacity)
    trainer = Trainer(model, criterion, solver, device=device, graphs=device.type == "cuda",
                      max_graphs=int(hp.get("max_graphs", 16)))
    output_dir.mkdir(parents=True, exist_ok=True)
    # the serial loop's batches (per-epoch seeded permutation, rank r takes its slots of
    # each global batch), mapped in worker processes and prefetched to the device
    loader = PrefetchLoader(ds, per_rank, total, rank=rank, world=world, seed=seed,
                            num_workers=int(hp.get("workers", 4)), device=device, pad_buckets=pad_buckets)
    save_every = int(hp.get("save_period") or 0) * iters_per_epoch
    for it, (images, masks, classes) in enumerate(loader, start=1):
        trainer.step(images, masks, classes)
        if step_callback is not None:
            step_callback(it, trainer, images)
        if save_every and it % save_every == 0:
            trainer.save(str(output_dir / f"model_epoch{it // iters_per_epoch:04d}.pth"))
    trainer.save(str(output_dir / "model_final.pth"))
    metrics = {"mAP50": 0.0, "mAP75": 0.0, "mAP": 0.0, "precision": 0.0, "recall": 0.0}
    if rank == 0 and device.type == "cuda":
        r = evaluate_dir(model, test_dir, img_size=img, device=device)
        if r is not None:
            metrics.update(r)
    if world > 1:
        dist.barrier()
    return metrics


def train_maskdino(exp_name, train_dir, test_dir, output_dir, hyperparams, backbone: str = "swin_t", device=None,
                   max_iters: int | None = None):
    """The reference's seam (train_template.py:104): MaskDINO on the MI355X path."""
    return train_mask2former(exp_name, train_dir, test_dir, output_dir, hyperparams, backbone=backbone, device=device,
                             max_iters=max_iters, arch="maskdino")
