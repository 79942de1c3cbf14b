"""Census of aten ops of one training step (forward + loss + backward + optimiser): count
and bytes of copies / casts / adds / sums / cats by (op, shape, dtype, first visionseg
call site).  Backward ops are attributed to the autograd node's forward call site when
torch provides it (anomaly-mode stacks are not used)."""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "vision-instance-seg_amd"))
import bench  # noqa: F401
import torch
from torch.utils._python_dispatch import TorchDispatchMode

from visionseg.model import M2FConfig, Mask2Former
from visionseg.criterion import SetCriterion
from visionseg.train import Trainer, SolverConfig
from visionseg.data import synthetic_batch

WATCH = ("copy_", "_to_copy", "add.Tensor", "add_.Tensor", "sum", "cat", "clone", "mul.Tensor", "fill_", "zero_", "clamp", "gelu", "where",
         "native_group_norm", "grid_sampler_2d", "mm.default", "addmm", "bmm")


def site():
    for fr in reversed(traceback.extract_stack()[:-3]):
        if "visionseg" in fr.filename or "criterion" in fr.filename:
            return f"{os.path.basename(fr.filename)}:{fr.lineno}"
    node = torch._C._current_autograd_node()
    return f"<{node.name()}>" if node is not None else "<other>"


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.c = collections.Counter()
        self.b = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func.overloadpacket.__name__) + "." + func._overloadname
        if any(w in name for w in WATCH):
            t = args[0] if args and isinstance(args[0], torch.Tensor) else None
            shp = tuple(t.shape) if t is not None else ()
            dt = str(t.dtype).replace("torch.", "") if t is not None else ""
            nb = t.numel() * t.element_size() if t is not None else 0
            key = (name, shp, dt, site())
            self.c[key] += 1
            self.b[key] += nb
        return out


def main():
    dev = torch.device("cuda", 0)
    cfg = M2FConfig.preset("swin_t")
    tr = Trainer(Mask2Former(cfg).init_weights(0), SetCriterion(cfg), SolverConfig(), device=dev)
    images, ml, cl = synthetic_batch(4, 1024, seed=42, device=dev)
    for _ in range(2):
        tr.step(images, ml, cl)
    torch.cuda.synchronize()
    cen = Census()
    with cen:
        tr.step(images, ml, cl)
    torch.cuda.synchronize()
    print("== by bytes (one step)")
    for k, v in sorted(cen.b.items(), key=lambda x: -x[1])[:70]:
        print(f"{v / 1e6:9.1f} MB x{cen.c[k]:4d}  {k[0]:24s} {str(k[1])[:34]:34s} {k[2]:9s} {k[3]}")
    print("== by count")
    for k, v in sorted(cen.c.items(), key=lambda x: -x[1])[:40]:
        print(f"x{v:4d} {cen.b[k] / 1e6:9.1f} MB  {k[0]:24s} {str(k[1])[:34]:34s} {k[2]:9s} {k[3]}")


if __name__ == "__main__":
    main()
