"""Which branch value_query_projection takes in the C2 bf16 step (fast fused Function or the
plain composition), and why."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-instance-seg_amd")]
import bench  # noqa: F401
import torch

from visionseg import linear
from visionseg.model import M2FConfig, Mask2Former
from visionseg.criterion import SetCriterion
from visionseg.train import Trainer, SolverConfig
from visionseg.data import synthetic_batch

orig = linear.value_query_projection
stats = []


def probe(h, pos, wv, bv, wp, bp, level_embed=None, level_sizes=None, sink=None):
    tokens = h.numel() // max(1, h.shape[-1])
    stats.append(dict(cuda=h.is_cuda, grad=torch.is_grad_enabled(), wv_rg=wv.requires_grad, tokens=tokens,
                      min=linear.MIN_TOKENS, autocast=torch.is_autocast_enabled(),
                      dt=(str(h.dtype), str(pos.dtype), str(wv.dtype), str(wp.dtype))))
    return orig(h, pos, wv, bv, wp, bp, level_embed, level_sizes, sink)


import visionseg.model as M  # noqa: E402
M.value_query_projection = probe
dev = torch.device("cuda", 0)
cfg = M2FConfig.preset("swin_t")
tr = Trainer(Mask2Former(cfg).init_weights(0), SetCriterion(cfg), SolverConfig(precision="bf16"), device=dev)
images, ml, cl = synthetic_batch(4, 1024, seed=42, device=dev)
tr.step(images, ml, cl)
torch.cuda.synchronize()
for s in stats[:3]:
    print(s)
print("calls", len(stats))
