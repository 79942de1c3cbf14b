"""Throughput of the training data path (visionseg.data.PrefetchLoader):
a synthetic COCO instance dataset in the reference's layout (PNG images + polygon
annotations, data.write_coco_dataset) is decoded, resized, flipped and rasterised in the
loader workers, collated into pinned uint8 batches and copied + normalised on a side
stream -- the same path adapters.train_mask2former feeds the Trainer with.  Prints one
line per worker count: images/s delivered on the device, to compare with the training
step's img/s (bench.py C2).  Usage:
    python tools/loader_bench.py [--size 1024] [--images 64] [--iters 24] [--workers 4,8,16]"""
import argparse
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-instance-seg_amd")]
import torch  # noqa: E402

from visionseg.data import CocoInstanceDataset, PrefetchLoader, write_coco_dataset  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--images", type=int, default=64)
    ap.add_argument("--iters", type=int, default=24)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--workers", default="4,8,16")
    a = ap.parse_args()
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as root:
        t0 = time.perf_counter()
        write_coco_dataset(root, a.images, a.size, seed=1)
        print(f"wrote {a.images} images {a.size}^2 in {time.perf_counter() - t0:.1f} s", flush=True)
        for nw in [int(v) for v in a.workers.split(",")]:
            ds = CocoInstanceDataset(root, fixed_size=a.size, seed=3)
            # steady state: the workers run prefetch_factor (2) batches each ahead, so the
            # batches delivered while that queue fills say nothing about the rate -- run
            # 8x the queue depth and time the second half of the batches only
            iters = max(a.iters, 16 * max(1, nw))
            ld = PrefetchLoader(ds, a.batch, iters, seed=5, num_workers=nw, device=dev)
            stamps = []
            for imgs, masks, classes in ld:
                if dev == "cuda":
                    torch.cuda.current_stream().synchronize()
                stamps.append(time.perf_counter())
            h = len(stamps) // 2
            n = (len(stamps) - 1 - h) * a.batch
            dt = stamps[-1] - stamps[h]
            print(f"workers {nw:2d}: {n} images in {dt:.2f} s = {n / dt:.1f} img/s on {dev} "
                  f"(batches {h + 1}..{len(stamps)} of {len(stamps)}, batch {a.batch}, {a.size}^2, PNG decode "
                  f"+ resize + flip + polygon raster + H2D + normalise)", flush=True)


if __name__ == "__main__":
    main()
