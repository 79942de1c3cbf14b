"""Achieved TF/s of every matrix op of one training step, grouped by op and input shapes:
torch.profiler with FLOP annotation (mm / addmm / bmm / baddbmm / convolution), device
time per group, sorted by device time.  Run on the GPU box from the repo root:
    python tools/gemm_census.py [model] [size] [batch]"""
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

OPS = ("aten::mm", "aten::addmm", "aten::bmm", "aten::baddbmm", "aten::convolution", "aten::_convolution",
       "aten::convolution_backward", "aten::cudnn_convolution", "aten::miopen_convolution", "aten::_scaled_dot_product_efficient_attention",
       "aten::_efficient_attention_backward")


def main():
    dev = torch.device("cuda", 0)
    model = sys.argv[1] if len(sys.argv) > 1 else "swin_t"
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    cfg = M2FConfig.preset(model)
    tr = Trainer(Mask2Former(cfg).init_weights(0), SetCriterion(cfg), SolverConfig(), device=dev)
    images, ml, cl = synthetic_batch(batch, size, seed=42, device=dev)
    for _ in range(3):
        tr.step(images, ml, cl)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_flops=True) as p:
        tr.step(images, ml, cl)
        torch.cuda.synchronize()
    rows = [e for e in p.key_averages(group_by_input_shape=True) if e.key in OPS]
    rows.sort(key=lambda e: -e.device_time_total)
    tot_t = sum(e.device_time_total for e in rows) / 1e3
    tot_f = sum(e.flops for e in rows)
    print(f"matrix ops: {tot_t:.2f} ms device, {tot_f / 1e12:.3f} TFLOP annotated")
    for e in rows[:45]:
        t = e.device_time_total / 1e3
        tf = e.flops / max(1e-9, e.device_time_total * 1e-6) / 1e12 if e.flops else 0.0
        print(f"{t:7.3f} ms {e.count:4d} {e.flops / 1e9:9.1f} GF {tf:7.1f} TF/s  {e.key[6:26]:20s} {str(e.input_shapes)[:120]}")


if __name__ == "__main__":
    main()
