"""Data-parallel rehearsal on ONE GPU: world_size-2 `gloo` ranks sharing cuda:0 (RCCL refuses two
ranks on one device), the Trainer in graph mode -- so the multi-rank step the driver's N > 1 bench
runs (split graphs: forward + backward with in-graph bucket events, the bucket all-reduces on the
high-priority side stream behind those events, then the optimiser graph) executes on a real GPU.
gloo's CUDA all-reduce stages through host memory; the schedule and the events are the ones RCCL
sees.  Checks: the split path and its captures ran, every loss is finite, the ranks' f32 master
weights stay identical (their batches differ, so only a correct reduction keeps them equal), and
they moved.  Launch:
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29511 tests/ddp_graph_worker.py
"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-instance-seg_amd")]
import visionseg  # noqa: E402,F401  (before anything touches the GPU: graph-capture settings)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from visionseg.train import Trainer, SolverConfig, init_distributed  # noqa: E402
from visionseg.model import M2FConfig, Mask2Former  # noqa: E402
from visionseg.criterion import SetCriterion  # noqa: E402
from visionseg.data import synthetic_batch  # noqa: E402


def checksum(t):
    d = t.double()
    return torch.stack([d.sum(), (d * d).sum(), d.abs().max()])


def main():
    rank, _, world = init_distributed("gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    cfg = M2FConfig.preset("swin_t", num_queries=100)
    model = Mask2Former(cfg).init_weights(seed=0)
    trainer = Trainer(model, SetCriterion(cfg), SolverConfig(), device=dev, graphs=True)
    images, ml, cl = synthetic_batch(1, 512, seed=42 + rank, device=dev)
    w0 = trainer.opt.master.clone()
    losses = []
    for _ in range(trainer.graph_warmup + 4):             # eager warm-ups, the capture, replays
        losses.append(float(trainer.step(images, ml, cl)))
    torch.cuda.synchronize()
    w = trainer.opt.master
    cs = checksum(w).to(dev)
    got = [torch.zeros_like(cs) for _ in range(world)]
    dist.all_gather(got, cs)
    moved = float((w - w0).abs().max())
    ok = (trainer.split and trainer.captures >= 1 and all(math.isfinite(v) for v in losses)
          and all(torch.equal(got[0], g) for g in got) and moved > 0)
    if rank == 0:
        print(f"world {world} split {trainer.split} captures {trainer.captures} losses "
              f"{[round(v, 4) for v in losses]} checksums {[g.tolist() for g in got]} max|dw| {moved:.3e} "
              f"{'OK' if ok else 'FAIL'}", flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
