"""Data-parallel path on CPU: world_size-2 gloo processes vs one process on the global
batch (gradient averaging equivalence, identical replicas, num_masks all-reduce)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class TinyNet(torch.nn.Module):
    """CPU stand-in with the model's output contract (mask logits per step, class logits
    per step); the product model's HIP ops need a GPU."""

    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.conv = torch.nn.Conv2d(3, 8, 3, padding=1)
        self.q = torch.nn.Parameter(torch.randn(5, 8))
        self.cls = torch.nn.Linear(8, 2)

    def forward(self, x):
        f = self.conv(x)                                   # [B,8,H,W]
        m = torch.einsum("qc,bchw->bqhw", self.q, f)
        c = self.cls(self.q).unsqueeze(0).expand(x.shape[0], -1, -1)
        return [m * 0.5, m], [c, c]


def _mse_criterion(masks, classes, ml, cl):
    loss = sum((m ** 2).mean() for m in masks) + sum((c ** 2).mean() for c in classes)
    return loss, {}


def _worker(rank, world, port, data, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from visionseg.train import Trainer, SolverConfig, init_distributed
    from visionseg.criterion import SetCriterion, PaddedTargets
    from visionseg.model import M2FConfig
    init_distributed("gloo")
    x = data[rank:rank + 1]
    tr = Trainer(TinyNet(), _mse_criterion, SolverConfig(warmup_iters=0, amp=False, clip_type="none"), device="cpu")
    assert tr.distributed
    tr.step(x, None, None)
    flat = torch.cat([p.detach().flatten() for p in tr.model.parameters()])
    # criterion num_masks is the global mean over ranks (upstream SetCriterion semantics)
    crit = SetCriterion(M2FConfig(num_queries=5))
    tg = PaddedTargets.from_lists([torch.zeros(rank + 1, 4, 4, dtype=torch.bool)],
                                  [torch.zeros(rank + 1, dtype=torch.int64)], device="cpu")
    n = crit._num_masks(tg, torch.device("cpu"))
    out_q.put((rank, flat.numpy().copy(), float(n)))   # by value: no shared-memory tensor handles
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_matches_single_process():
    from visionseg.train import Trainer, SolverConfig
    torch.manual_seed(1)
    data = torch.randn(2, 3, 16, 16)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, data, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, f0, n0), (_, f1, n1) = res
    f0, f1 = torch.from_numpy(f0), torch.from_numpy(f1)
    assert torch.equal(f0, f1), "replicas diverged"
    assert n0 == n1 == pytest.approx(1.5)
    # single process, global batch of 2: mean-reduced loss over per-image terms = DDP average
    tr = Trainer(TinyNet(), lambda m, c, a, b: (sum(_mse_criterion([mm[i:i + 1] for mm in m],
                                                                   [cc[i:i + 1] for cc in c], a, b)[0]
                                                    for i in range(2)) / 2, {}),
                 SolverConfig(warmup_iters=0, amp=False, clip_type="none"), device="cpu", distributed=False)
    tr.step(data, None, None)
    ref = torch.cat([p.detach().flatten() for p in tr.model.parameters()])
    assert torch.allclose(f0, ref, atol=1e-6), float((f0 - ref).abs().max())
