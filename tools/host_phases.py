"""Is the training step host-bound?  For each phase of Trainer.step (forward, criterion,
backward, optimiser) print the host time to ENQUEUE the phase and the time until the
GPU has finished it.  enqueue ~= done means the GPU waits on the host."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "vision-instance-seg_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: F401  (sets the TunableOp environment before torch initialises)
import torch

from visionseg.model import M2FConfig, Mask2Former
from visionseg.criterion import SetCriterion
from visionseg.train import Trainer, SolverConfig
from visionseg.data import synthetic_batch


def main():
    dev = torch.device("cuda", 0)
    cfg = M2FConfig.preset("swin_t")
    tr = Trainer(Mask2Former(cfg).init_weights(0), SetCriterion(cfg), SolverConfig(), device=dev)
    images, ml, cl = synthetic_batch(4, 1024, seed=42, device=dev)
    for _ in range(3):
        tr.step(images, ml, cl)
    torch.cuda.synchronize()
    rows = []
    for it in range(5):
        r = {}
        for p in tr.model_params:
            p.grad = None
        t = time.perf_counter()
        masks, classes = tr.net(images)
        r["fwd_enq"] = time.perf_counter() - t
        torch.cuda.synchronize()
        r["fwd_done"] = time.perf_counter() - t
        t = time.perf_counter()
        loss, _ = tr.criterion([m.float() for m in masks], [c.float() for c in classes], ml, cl)
        r["crit_enq"] = time.perf_counter() - t
        torch.cuda.synchronize()
        r["crit_done"] = time.perf_counter() - t
        t = time.perf_counter()
        loss.backward()
        r["bwd_enq"] = time.perf_counter() - t
        torch.cuda.synchronize()
        r["bwd_done"] = time.perf_counter() - t
        t = time.perf_counter()
        if tr.params[0].grad is None:
            for m in tr.params:
                m.grad = torch.empty_like(m)
        torch._foreach_copy_([m.grad for m in tr.params], [p.grad for p in tr.model_params])
        tr.clip_gradients()
        tr.opt.step()
        with torch.no_grad():
            torch._foreach_copy_(tr.model_params, tr.params)
        r["opt_enq"] = time.perf_counter() - t
        torch.cuda.synchronize()
        r["opt_done"] = time.perf_counter() - t
        t = time.perf_counter()
        tr.step(images, ml, cl)
        r["step_enq"] = time.perf_counter() - t
        torch.cuda.synchronize()
        r["step_done"] = time.perf_counter() - t
        rows.append(r)
    for k in rows[0]:
        v = sorted(x[k] for x in rows)[len(rows) // 2] * 1e3
        print(f"{k:10s} {v:8.2f} ms")


if __name__ == "__main__":
    main()
