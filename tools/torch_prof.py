"""Attribute the step's small kernels to call sites: torch.profiler over 2 bench steps,
top aten ops by device time with input shapes, and the Python stacks of copies / adds /
sums / cats."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "vision-instance-seg_amd"))
import bench  # noqa: F401  (TunableOp environment)
import torch
from torch.profiler import profile, ProfilerActivity

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
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as p:
        for _ in range(2):
            tr.step(images, ml, cl)
        torch.cuda.synchronize()
    ka = p.key_averages(group_by_input_shape=True)
    rows = sorted(ka, key=lambda e: -e.device_time_total)
    print("== top ops by device time (2 steps), with input shapes")
    for e in rows[:60]:
        print(f"{e.device_time_total / 1e3:8.2f} ms {e.count:5d}  {e.key[:40]:40s} {str(e.input_shapes)[:110]}")
    print("\n== copies / sums / clones / casts by input shape")
    sel = [e for e in rows if e.key in ("aten::copy_", "aten::sum", "aten::clone", "aten::_to_copy", "aten::contiguous",
                                         "aten::add", "aten::cat", "aten::add_", "aten::fill_", "aten::mul")]
    for e in sorted(sel, key=lambda e: -e.device_time_total)[:45]:
        print(f"{e.device_time_total / 1e3:8.2f} ms {e.count:5d}  {e.key:18s} {str(e.input_shapes)[:150]}")
    ks = p.key_averages(group_by_stack_n=6)
    print("\n== copies / adds / sums / cats by stack")
    sel = [e for e in ks if e.key in ("aten::copy_", "aten::add", "aten::add_", "aten::sum", "aten::cat", "aten::mul",
                                      "aten::clone", "aten::contiguous", "aten::_to_copy", "aten::fill_",
                                      "aten::zero_", "aten::where", "aten::index_put_")]
    for e in sorted(sel, key=lambda e: -e.device_time_total)[:40]:
        st = " | ".join(s.split("/")[-1][:60] for s in e.stack[:6] if "torch/" not in s)
        print(f"{e.device_time_total / 1e3:8.2f} ms {e.count:5d}  {e.key:16s} {st[:300]}")


if __name__ == "__main__":
    main()
