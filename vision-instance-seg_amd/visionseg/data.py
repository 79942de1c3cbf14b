"""COCO-format instance data for the training path.

* `synthetic_batch` — BASELINE's synthetic "COCO-format defect" batches:
  uint8 images ~ U[0,255], 1..3 thin "thunderbolt"-like polygon instances per image,
  single class 0 (the reference remaps category 1 -> 0 for detectron2,
  scripts/data_utils/fix_category_ids.py:25-36), masks rasterised to bool.
* `write_coco_dataset` / `CocoInstanceDataset` — the on-disk format the reference's
  callers hand over (`train_dir/annotations.json` + images; guide.md:144-161,
  training/train_template.py:188-194), mapped the way the reference's
  MaskDINODatasetMapper does (training/maskdino/train_full.py:69-147): polygon ->
  bitmask, ResizeShortestEdge, random horizontal flip, class ids kept.
* `normalize` — ImageNet pixel mean/std (detectron2 PIXEL_MEAN/STD in RGB order).
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch
from PIL import Image, ImageDraw

PIXEL_MEAN = (123.675, 116.28, 103.53)
PIXEL_STD = (58.395, 57.12, 57.375)


def normalize(images_u8: torch.Tensor) -> torch.Tensor:
    """uint8 [B,3,H,W] -> float32 normalised."""
    m = torch.tensor(PIXEL_MEAN, device=images_u8.device).view(1, 3, 1, 1)
    s = torch.tensor(PIXEL_STD, device=images_u8.device).view(1, 3, 1, 1)
    return (images_u8.float() - m) / s


def thunderbolt_polygon(rng: np.random.Generator, H: int, W: int) -> list:
    """A thin zig-zag stroke as a closed polygon (8..16 vertices), area ~0.5-5% of the image."""
    n = int(rng.integers(4, 9))                 # polyline joints -> 2n polygon vertices
    L = rng.uniform(0.25, 0.6) * min(H, W)
    ang = rng.uniform(0, 2 * np.pi)
    cx, cy = rng.uniform(0.2, 0.8) * W, rng.uniform(0.2, 0.8) * H
    t = np.linspace(-0.5, 0.5, n) * L
    zig = rng.uniform(0.03, 0.09) * L * np.where(np.arange(n) % 2 == 0, 1.0, -1.0)
    px = cx + t * np.cos(ang) - zig * np.sin(ang)
    py = cy + t * np.sin(ang) + zig * np.cos(ang)
    wid = rng.uniform(0.012, 0.04) * min(H, W)
    nx, ny = -np.sin(ang) * wid, np.cos(ang) * wid
    left = list(zip(px + nx, py + ny))
    right = list(zip(px - nx, py - ny))[::-1]
    pts = np.clip(np.array(left + right), 0, [W - 1, H - 1])
    return pts.reshape(-1).tolist()


def _rle_counts_from_string(s: str) -> list:
    """COCO compressed RLE string -> run lengths (pycocotools rleFrString: 5-bit groups
    with a continuation bit, sign-extended, each count after the second delta-coded
    against the count two places back)."""
    counts, p, m = [], 0, 0
    while p < len(s):
        x, k, more = 0, 0, True
        while more:
            c = ord(s[p]) - 48
            x |= (c & 0x1F) << (5 * k)
            more = bool(c & 0x20)
            p += 1
            k += 1
            if not more and (c & 0x10):
                x |= -1 << (5 * k)
        if m > 2:
            x += counts[m - 2]
        counts.append(x)
        m += 1
    return counts


def decode_rle(rle: dict) -> np.ndarray:
    """COCO RLE segmentation ({"counts": list or compressed string, "size": [h, w]}) ->
    bool mask [h, w].  Runs alternate background / foreground starting with background,
    in column-major order."""
    h, w = (int(v) for v in rle["size"])
    counts = rle["counts"]
    if isinstance(counts, (bytes, str)):
        counts = _rle_counts_from_string(counts.decode() if isinstance(counts, bytes) else counts)
    flat = np.zeros(h * w, dtype=bool)
    pos = 0
    for i, n in enumerate(counts):
        n = int(n)
        if i % 2 == 1:
            flat[pos:pos + n] = True
        pos += n
    return flat.reshape(w, h).T


def _resize_nearest(m: np.ndarray, H: int, W: int) -> np.ndarray:
    if m.shape == (H, W):
        return m
    ys = np.minimum((np.arange(H) + 0.5) * m.shape[0] / H, m.shape[0] - 1).astype(np.int64)
    xs = np.minimum((np.arange(W) + 0.5) * m.shape[1] / W, m.shape[1] - 1).astype(np.int64)
    return m[ys][:, xs]


def rasterize(poly_flat: list, H: int, W: int) -> np.ndarray:
    img = Image.new("1", (W, H), 0)
    ImageDraw.Draw(img).polygon([(poly_flat[i], poly_flat[i + 1]) for i in range(0, len(poly_flat), 2)], fill=1)
    return np.array(img, dtype=bool)


def synthetic_sample(rng: np.random.Generator, H: int, W: int):
    img = rng.integers(0, 256, size=(3, H, W), dtype=np.uint8)
    k = int(rng.integers(1, 4))
    polys = [thunderbolt_polygon(rng, H, W) for _ in range(k)]
    masks = np.stack([rasterize(p, H, W) for p in polys])
    return img, masks, np.zeros(k, dtype=np.int64), polys


def synthetic_batch(batch: int, size: int, seed: int = 42, device="cpu"):
    """-> (images float [B,3,S,S] normalised, [masks bool [K_i,S,S]], [classes int64 [K_i]])."""
    rng = np.random.default_rng(seed)
    imgs, masks, classes = [], [], []
    for _ in range(batch):
        im, m, c, _ = synthetic_sample(rng, size, size)
        imgs.append(torch.from_numpy(im))
        masks.append(torch.from_numpy(m).to(device))
        classes.append(torch.from_numpy(c).to(device))
    images = normalize(torch.stack(imgs).to(device))
    return images, masks, classes


def write_coco_dataset(root: str, n_images: int, size, seed: int = 42, category: str = "thunderbolt"):
    """Write `root/annotations.json` + `root/images/*.png` in the reference's COCO layout.
    `size`: a side length (square images) or a list of (height, width) cycled over the
    images (mixed aspect ratios)."""
    os.makedirs(os.path.join(root, "images"), exist_ok=True)
    rng = np.random.default_rng(seed)
    shapes = [(int(size), int(size))] if isinstance(size, int) else [(int(h), int(w)) for h, w in size]
    images, anns = [], []
    aid = 1
    for i in range(n_images):
        H, W = shapes[i % len(shapes)]
        im, masks, _, polys = synthetic_sample(rng, H, W)
        fn = f"{i:06d}.png"
        Image.fromarray(np.transpose(im, (1, 2, 0))).save(os.path.join(root, "images", fn))
        images.append({"id": i, "file_name": fn, "height": H, "width": W})
        for m, p in zip(masks, polys):
            ys, xs = np.nonzero(m)
            bbox = [float(xs.min()), float(ys.min()), float(xs.max() - xs.min() + 1), float(ys.max() - ys.min() + 1)] \
                if len(xs) else [0.0, 0.0, 0.0, 0.0]
            anns.append({"id": aid, "image_id": i, "category_id": 0, "segmentation": [p], "area": float(m.sum()),
                         "bbox": bbox, "iscrowd": 0})
            aid += 1
    coco = {"images": images, "annotations": anns, "categories": [{"id": 0, "name": category}]}
    with open(os.path.join(root, "annotations.json"), "w") as f:
        json.dump(coco, f)
    return coco


class CocoInstanceDataset:
    """Reads a COCO instance json (+ images) -> (uint8 image [3,H,W], bool masks [K,H,W],
    int64 classes [K]) per image, with the reference mapper's train augmentations."""

    def __init__(self, root: str, ann_file: str = "annotations.json", image_dir: str | None = None,
                 min_size=(480, 512, 544, 576, 608, 640), max_size=800, train=True, fixed_size: int | None = None,
                 seed: int = 42, keep_size: bool = False):
        with open(os.path.join(root, ann_file)) as f:
            coco = json.load(f)
        self.root = root
        self.image_dir = image_dir or (os.path.join(root, "images") if os.path.isdir(os.path.join(root, "images")) else root)
        self.images = coco["images"]
        self.by_img = {}
        for a in coco.get("annotations", []):
            self.by_img.setdefault(a["image_id"], []).append(a)
        cats = sorted(c["id"] for c in coco.get("categories", [{"id": 0}]))
        self.cat_to_label = {c: i for i, c in enumerate(cats)}
        self.min_size, self.max_size, self.train, self.fixed_size = min_size, max_size, train, fixed_size
        self.keep_size = keep_size
        self.rng = np.random.default_rng(seed)

    def __len__(self):
        return len(self.images)

    def _target_size(self, h, w):
        if self.keep_size:
            return h, w
        if self.fixed_size:
            return self.fixed_size, self.fixed_size
        s = int(self.rng.choice(self.min_size)) if self.train else int(self.min_size[-1])
        scale = s / min(h, w)
        if max(h, w) * scale > self.max_size:
            scale = self.max_size / max(h, w)
        return int(round(h * scale)), int(round(w * scale))

    def __getitem__(self, i):
        info = self.images[i]
        img = Image.open(os.path.join(self.image_dir, info["file_name"])).convert("RGB")
        w0, h0 = img.size
        H, W = self._target_size(h0, w0)
        sx, sy = W / w0, H / h0
        img = img.resize((W, H), Image.BILINEAR)
        masks, classes = [], []
        for a in self.by_img.get(info["id"], []):
            if a.get("iscrowd", 0):
                continue
            segm = a["segmentation"]
            if isinstance(segm, dict):            # RLE (train_full.py:116-129 decodes both forms)
                m = _resize_nearest(decode_rle(segm), H, W)
            else:
                m = np.zeros((H, W), dtype=bool)
                for poly in segm:
                    p = np.array(poly, dtype=np.float64).reshape(-1, 2) * [sx, sy]
                    m |= rasterize(p.reshape(-1).tolist(), H, W)
            masks.append(m)
            classes.append(self.cat_to_label[a["category_id"]])
        arr = np.asarray(img, dtype=np.uint8).transpose(2, 0, 1)
        if self.train and self.rng.random() < 0.5:
            arr = arr[:, :, ::-1]
            masks = [m[:, ::-1] for m in masks]
        m = np.stack(masks) if masks else np.zeros((0, H, W), dtype=bool)
        return (torch.from_numpy(np.ascontiguousarray(arr)), torch.from_numpy(np.ascontiguousarray(m)),
                torch.tensor(classes, dtype=torch.int64))


def collate_padded(samples, size_divisibility: int = 32, device="cpu"):
    """Pad a list of samples to a common size divisible by 32 (detectron2 ImageList)."""
    H = max(s[0].shape[1] for s in samples)
    W = max(s[0].shape[2] for s in samples)
    H = (H + size_divisibility - 1) // size_divisibility * size_divisibility
    W = (W + size_divisibility - 1) // size_divisibility * size_divisibility
    imgs = torch.zeros(len(samples), 3, H, W, dtype=torch.float32, device=device)
    masks, classes = [], []
    for i, (im, m, c) in enumerate(samples):
        imgs[i, :, :im.shape[1], :im.shape[2]] = normalize(im[None].to(device))[0]   # pad after normalising
        mm = torch.zeros(m.shape[0], H, W, dtype=torch.bool)
        mm[:, :m.shape[1], :m.shape[2]] = m
        masks.append(mm.to(device))
        classes.append(c.to(device))
    return imgs, masks, classes


# ----------------------------------------------------------------------------------
# Loader: worker processes + pinned host batches + H2D on a side stream, one batch ahead
# ----------------------------------------------------------------------------------


def bucket_size(n: int, size_divisibility: int = 32, buckets=None) -> int:
    """A padded side: n rounded up to `size_divisibility` (detectron2 ImageList), then --
    with `buckets` (ascending side lengths) -- up to the smallest bucket that holds it (a
    side above the largest bucket keeps its 32-rounded size)."""
    n = (n + size_divisibility - 1) // size_divisibility * size_divisibility
    for b in buckets or ():
        if n <= b:
            return int(b)
    return n


def default_pad_buckets(min_sizes, max_size, size_divisibility: int = 32):
    """The seam's padding canvases for ResizeShortestEdge(min_sizes, max_size): per side
    the second-smallest and the largest short-edge choice and the long-edge limit, each
    rounded up to `size_divisibility` -- (512, 640, 800) for the reference's
    MIN_SIZE_TRAIN 480..640 / MAX_SIZE_TRAIN 800 (train_full.py:244-245): at most 9
    padded shapes per run, so the trainer's graphs and MIOpen's per-shape solver search
    are paid a bounded number of times."""
    r = lambda n: (int(n) + size_divisibility - 1) // size_divisibility * size_divisibility   # noqa: E731
    ms = sorted(int(m) for m in min_sizes)
    return tuple(sorted({r(ms[min(1, len(ms) - 1)]), r(ms[-1]), r(max_size)}))


def collate_host(samples, size_divisibility: int = 32, buckets=None):
    """CPU half of collate_padded, run inside the loader workers: uint8 images padded to a
    common size divisible by 32 [B,3,H,W] (or to a bucket canvas, `bucket_size`), the
    (unpadded) image sizes, masks padded to the same size (bool [K,H,W] per image),
    classes.  Normalisation happens on the device."""
    H = bucket_size(max(s[0].shape[1] for s in samples), size_divisibility, buckets)
    W = bucket_size(max(s[0].shape[2] for s in samples), size_divisibility, buckets)
    imgs = torch.zeros(len(samples), 3, H, W, dtype=torch.uint8)
    sizes = torch.zeros(len(samples), 2, dtype=torch.int64)
    masks, classes = [], []
    for i, (im, m, c) in enumerate(samples):
        imgs[i, :, :im.shape[1], :im.shape[2]] = im
        sizes[i, 0], sizes[i, 1] = im.shape[1], im.shape[2]
        mm = torch.zeros(m.shape[0], H, W, dtype=torch.bool)
        mm[:, :m.shape[1], :m.shape[2]] = m
        masks.append(mm)
        classes.append(c)
    return imgs, sizes, masks, classes


def normalize_padded(imgs_u8: torch.Tensor, sizes: torch.Tensor) -> torch.Tensor:
    """Device half of collate_padded: normalise, then zero the padding (detectron2 pads the
    normalised image with 0; collate_padded does the same)."""
    out = normalize(imgs_u8)
    H, W = out.shape[-2:]
    rows = torch.arange(H, device=out.device).view(1, H, 1)
    cols = torch.arange(W, device=out.device).view(1, 1, W)
    s = sizes.to(out.device)
    keep = (rows < s[:, 0].view(-1, 1, 1)) & (cols < s[:, 1].view(-1, 1, 1))
    return out * keep[:, None].to(out.dtype)


class _EpochSampler(torch.utils.data.Sampler):
    """Batches of this rank's share of a seeded permutation per epoch (the serial loop of
    adapters.train_mask2former: rank r takes slots r, r + world, ... of each global batch)."""

    def __init__(self, n, per_rank, rank, world, seed, iters):
        self.n, self.per_rank, self.rank, self.world, self.seed, self.iters = n, per_rank, rank, world, seed, iters

    def __iter__(self):
        rng = np.random.default_rng(self.seed)
        it, epoch_iters = 0, max(1, -(-self.n // (self.per_rank * self.world)))
        while it < self.iters:
            order = rng.permutation(self.n)
            for k in range(epoch_iters):
                if it >= self.iters:
                    return
                a = (k * self.world + self.rank) * self.per_rank
                idx = order[a:a + self.per_rank]
                if len(idx) == 0:
                    idx = order[:self.per_rank]
                yield [int(i) for i in idx]
                it += 1

    def __len__(self):
        return self.iters


def _seed_worker(worker_id):
    info = torch.utils.data.get_worker_info()
    ds = info.dataset
    if hasattr(ds, "rng"):      # independent augmentation streams per worker
        ds.rng = np.random.default_rng(int(info.seed % (2 ** 32)))


class PrefetchLoader:
    """The data path of the training seam at speed (the reference runs the
    detectron2 mapper in loader workers, train_full.py:50-67, 116-143): `num_workers`
    processes decode / resize / flip / rasterise (CocoInstanceDataset) and collate padded
    uint8 batches into pinned host memory; the iterator copies batch i+1 to the device on a
    side stream (non-blocking) while the caller trains on batch i, and normalises on the
    device.  Yields (images f32 [B,3,H,W], masks [bool [K,H,W]], classes [int64 [K]]) on
    `device`, like collate_padded.  `pad_buckets`: pad each batch to a canvas side from
    this list (`bucket_size`) instead of its largest image rounded to 32: more zero
    padding -- what detectron2 does to a batch whose largest image has that size -- in
    exchange for a handful of distinct batch shapes."""

    def __init__(self, dataset, per_rank: int, iters: int, rank: int = 0, world: int = 1, seed: int = 42,
                 num_workers: int = 4, device="cuda", prefetch_factor: int = 2, pad_buckets=None):
        import functools
        self.device = torch.device(device)
        pin = self.device.type == "cuda"
        sampler = _EpochSampler(len(dataset), per_rank, rank, world, seed, iters)
        collate = functools.partial(collate_host, buckets=tuple(pad_buckets) if pad_buckets else None)
        kw = dict(num_workers=num_workers, collate_fn=collate, pin_memory=pin, batch_sampler=sampler)
        if num_workers > 0:
            kw.update(worker_init_fn=_seed_worker, prefetch_factor=prefetch_factor, persistent_workers=False)
        self.loader = torch.utils.data.DataLoader(dataset, **kw)
        self.stream = torch.cuda.Stream(self.device) if pin else None

    def __len__(self):
        return len(self.loader)

    def _to_device(self, batch):
        imgs, sizes, masks, classes = batch
        if self.stream is None:
            return normalize_padded(imgs, sizes), masks, classes, None
        with torch.cuda.stream(self.stream):
            imgs = imgs.to(self.device, non_blocking=True)
            sizes = sizes.to(self.device, non_blocking=True)
            masks = [m.to(self.device, non_blocking=True) for m in masks]
            classes = [c.to(self.device, non_blocking=True) for c in classes]
            imgs = normalize_padded(imgs, sizes)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return imgs, masks, classes, ev

    def __iter__(self):
        it = iter(self.loader)
        nxt = None
        try:
            nxt = self._to_device(next(it))
        except StopIteration:
            return
        while nxt is not None:
            cur = nxt
            try:
                nxt = self._to_device(next(it))       # H2D of the next batch overlaps this step
            except StopIteration:
                nxt = None
            imgs, masks, classes, ev = cur
            if ev is not None:
                torch.cuda.current_stream(self.device).wait_event(ev)
                for t in [imgs, *masks, *classes]:
                    t.record_stream(torch.cuda.current_stream(self.device))
            yield imgs, masks, classes
