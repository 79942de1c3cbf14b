"""Steady-state images/s of the TRAINING SEAM on reference-shaped data.

A COCO-format dataset in the reference's layout (PNG images + polygon annotations,
data.write_coco_dataset) with MIXED aspect ratios goes through
adapters.train_mask2former exactly as train_template.py would call it: the loader
workers run the reference mapper's multi-scale ResizeShortestEdge (MIN_SIZE_TRAIN
480..640, MAX_SIZE_TRAIN 800, train_full.py:244-245) + flip + polygon raster, batches are
padded (to the seam's canvases, or detectron2-exact with --buckets exact), the Trainer
replays one HIP graph per padded shape.  The last `--timed` steps are timed.

The comparison: the same sequence of padded batch shapes replayed through a fresh
Trainer on device-resident synthetic batches (no loader, every shape's graph captured
before the timed region) -- the synthetic-step rate "at the same shapes".

Prints one JSON line per mode.  Usage:
    python tools/seam_bench.py [--images 96] [--iters 140] [--timed 60] [--batch 4] [--workers 12]
                               [--modes auto,exact] [--backbone swin_t]
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-instance-seg_amd")]
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
import numpy as np  # noqa: E402
import visionseg  # noqa: E402,F401  (before HIP initialises)
import torch  # noqa: E402

from visionseg.data import normalize, synthetic_sample, write_coco_dataset  # noqa: E402

SHAPES = [(1024, 1024), (768, 1024), (1024, 768), (720, 1280), (1280, 720), (960, 1280), (1200, 900)]


def synthetic_shaped(rng, B, H, W, dev):
    imgs, masks, classes = [], [], []
    for _ in range(B):
        im, m, c, _ = synthetic_sample(rng, H, W)
        imgs.append(torch.from_numpy(im))
        masks.append(torch.from_numpy(m).to(dev))
        classes.append(torch.from_numpy(c).to(dev))
    return normalize(torch.stack(imgs).to(dev)), masks, classes


def run_seam(root, out, a, buckets):
    from visionseg.adapters import train_mask2former
    rec = {"shapes": [], "t0": None, "t1": None, "cap0": 0, "cap1": 0, "eager0": 0, "eager1": 0}
    start = a.iters - a.timed

    def cb(it, tr, images):
        rec["shapes"].append(tuple(images.shape[-2:]))
        if it in (start, a.iters):
            torch.cuda.synchronize()
            k = "0" if it == start else "1"
            rec["t" + k] = time.perf_counter()
            rec["cap" + k] = tr.captures
            rec["eager" + k] = sum(tr._eager_seen.values())
            rec["graphs"] = len(tr._graph_states)
        if it % 20 == 0:
            print(f"  seam step {it}/{a.iters} shape {tuple(images.shape[-2:])} graphs {len(tr._graph_states)} "
                  f"captures {tr.captures}", flush=True)

    hp = {"batch_size": a.batch, "img_size": 640, "workers": a.workers, "epochs": 10 ** 6, "save_period": 0,
          "optimizer": "SGD", "lr_scheduler": "multistep", "warmup_epochs": 0, "pad_buckets": buckets,
          "backbone": a.backbone}
    t = time.perf_counter()
    train_mask2former("seam_bench", root, os.path.join(root, "no_test"), out, hp, max_iters=a.iters,
                      step_callback=cb)
    wall = time.perf_counter() - t
    dt = rec["t1"] - rec["t0"]
    return rec, dt, wall


def run_synthetic(shapes, a):
    """The seam's timed shape sequence through a fresh graph Trainer on resident batches."""
    from visionseg.criterion import SetCriterion
    from visionseg.model import M2FConfig, Mask2Former
    from visionseg.train import SolverConfig, Trainer
    dev = torch.device("cuda", 0)
    cfg = M2FConfig.preset(a.backbone)
    tr = Trainer(Mask2Former(cfg).init_weights(0), SetCriterion(cfg), SolverConfig(), device=dev, graphs=True,
                 max_graphs=16)
    rng = np.random.default_rng(0)
    batches = {s: synthetic_shaped(rng, a.batch, s[0], s[1], dev) for s in sorted(set(shapes))}
    for s, b in batches.items():                  # 2 eager steps + the capture of every shape
        for _ in range(tr.graph_warmup + 1):
            tr.step(*b)
    torch.cuda.synchronize()
    cap = tr.captures
    t0 = time.perf_counter()
    for s in shapes:
        tr.step(*batches[s])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert tr.captures == cap
    del tr
    return dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=96)
    ap.add_argument("--iters", type=int, default=140)
    ap.add_argument("--timed", type=int, default=60)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--workers", type=int, default=12)
    ap.add_argument("--modes", default="auto,exact")
    ap.add_argument("--backbone", default="swin_t")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as root:
        t = time.perf_counter()
        write_coco_dataset(root, a.images, SHAPES, seed=1)
        print(f"wrote {a.images} images of {len(SHAPES)} aspect ratios in {time.perf_counter() - t:.1f} s", flush=True)
        for mode in a.modes.split(","):
            buckets = "auto" if mode == "auto" else []
            out = os.path.join(root, f"out_{mode}")
            rec, dt, wall = run_seam(root, out, a, buckets)
            timed_shapes = rec["shapes"][a.iters - a.timed:]
            sdt = run_synthetic(timed_shapes, a)
            n = a.timed * a.batch
            line = {"tool": "seam_bench", "mode": mode, "backbone": a.backbone, "batch": a.batch,
                    "images_per_s_seam": round(n / dt, 2), "images_per_s_synthetic_same_shapes": round(n / sdt, 2),
                    "seam_over_synthetic": round(sdt / dt, 3), "timed_steps": a.timed, "total_steps": a.iters,
                    "distinct_shapes_total": len(set(rec["shapes"])), "distinct_shapes_timed": len(set(timed_shapes)),
                    "captures_in_timed": rec["cap1"] - rec["cap0"], "eager_steps_in_timed": rec["eager1"] - rec["eager0"],
                    "captures_total": rec["cap1"], "live_graphs": rec.get("graphs"), "seam_wall_s": round(wall, 1),
                    "workers": a.workers, "data": f"{a.images} PNG images, shapes {SHAPES}, 1-3 polygon instances, "
                    "ResizeShortestEdge 480..640 / 800 + flip",
                    "shape_counts": {f"{h}x{w}": timed_shapes.count((h, w)) for h, w in sorted(set(timed_shapes))}}
            print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
