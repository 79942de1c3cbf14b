"""Attribute the step's small kernels to call sites: torch.profiler over 2 eager training steps
(C2: Swin-T, 4 x 1024^2, bf16), top aten ops by device time with input shapes, and the glue ops
(copies / adds / sums / cats / casts / fills / GELU) summed per step by the innermost frame of
the package that issued them."""
import collections
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

GLUE = ("aten::copy_", "aten::add", "aten::add_", "aten::sum", "aten::cat", "aten::mul", "aten::clone",
        "aten::contiguous", "aten::_to_copy", "aten::fill_", "aten::zero_", "aten::where", "aten::index_put_",
        "aten::gelu", "aten::gelu_backward", "aten::clamp", "aten::clamp_", "aten::stack", "aten::sub",
        "aten::div", "aten::masked_fill", "aten::grid_sampler_2d", "aten::mm", "aten::bmm", "aten::addmm",
        "aten::_foreach_add_", "aten::_foreach_mul_", "aten::_foreach_zero_")
STEPS = 2


def main():
    dev = torch.device("cuda", 0)
    cfg = M2FConfig.preset("swin_t")
    tr = Trainer(Mask2Former(cfg).init_weights(0), SetCriterion(cfg), SolverConfig(), device=dev)
    images, ml, cl = synthetic_batch(4, 1024, seed=42, device=dev)
    for _ in range(3):
        tr.step(images, ml, cl)
    torch.cuda.synchronize()
    exp = torch._C._profiler._ExperimentalConfig(verbose=True)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True,
                 experimental_config=exp) as p:
        for _ in range(STEPS):
            tr.step(images, ml, cl)
        torch.cuda.synchronize()
    ka = p.key_averages(group_by_input_shape=True)
    rows = sorted(ka, key=lambda e: -e.device_time_total)
    print("== top ops by device time (ms per step), with input shapes")
    for e in rows[:50]:
        print(f"{e.device_time_total / 1e3 / STEPS:8.3f} ms {e.count // STEPS:5d}  {e.key[:40]:40s} {str(e.input_shapes)[:110]}")
    # glue: innermost package frame of each top-level glue op (children's device time is
    # included in the parent's device_time_total, so only ops without a glue ancestor count)
    by_site = collections.defaultdict(lambda: [0.0, 0, set()])
    total = 0.0
    for ev in p.events():
        if ev.name not in GLUE or ev.device_time_total <= 0:
            continue
        par, nested = ev.cpu_parent, False
        while par is not None:
            if par.name in GLUE:
                nested = True
                break
            par = par.cpu_parent
        if nested:
            continue
        site = "?"
        for fr in ev.stack or []:
            if "visionseg" in fr or "bench.py" in fr:
                site = fr.split("vision-instance-seg_amd/")[-1][:90]
                break
        if site == "?":                  # autograd's C++ backward nodes: the nearest named ancestor
            par = ev.cpu_parent
            while par is not None and par.name.startswith("aten::"):
                par = par.cpu_parent
            if par is not None:
                site = par.name[:90]
        s = by_site[(ev.name, site)]
        s[0] += ev.device_time_total / 1e3 / STEPS
        s[1] += 1
        s[2].add(str(ev.input_shapes)[:70])
        total += ev.device_time_total / 1e3 / STEPS
    print(f"\n== glue ops by call site: {total:.3f} ms per step")
    for (name, site), (ms, n, shp) in sorted(by_site.items(), key=lambda kv: -kv[1][0])[:60]:
        print(f"{ms:8.3f} ms {n // STEPS:4d}  {name:22s} {site:90s} {' '.join(sorted(shp)[:8])[:400]}")


if __name__ == "__main__":
    main()
