"""Data-parallel path on CPU: world_size-2 gloo processes vs one process on the global
batch, through the product Trainer's flat gradient buffer and bucketed all-reduce
(visionseg.optim.GradReducer, several buckets, an unused parameter), the f32 master
update, identical replicas and the criterion's num_masks all-reduce.  The HIP optimiser
kernel is replaced by its CPU emulation (tests/_flatref.py); everything else is the
product host logic."""
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
        self.norm = torch.nn.GroupNorm(2, 8)
        self.q = torch.nn.Parameter(torch.randn(5, 8))
        self.cls = torch.nn.Linear(8, 2)
        self.unused = torch.nn.Parameter(torch.randn(3))

    def forward(self, x):
        f = self.norm(self.conv(x))                        # [B,8,H,W]
        m = torch.einsum("qc,bchw->bqhw", self.q, f)
        c = self.cls(self.q).unsqueeze(0).expand(x.shape[0], -1, -1)
        return [m * 0.5, m], [c, c]


def _mse_criterion(masks, classes, ml, cl):
    loss = sum((m ** 2).mean() for m in masks) + sum((c ** 2).mean() for c in classes)
    return loss, {}


def _solver(optimizer, clip):
    from visionseg.train import SolverConfig
    # tiny bucket cap: the 8 parameters land in several buckets
    return SolverConfig(warmup_iters=0, amp=False, clip_type=clip, clip_value=0.05, optimizer=optimizer,
                        lr=0.05, bucket_cap_mb=1e-4)


def _worker(rank, world, port, data, optimizer, clip, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import _flatref
    from visionseg import optim
    from visionseg.train import Trainer, init_distributed
    from visionseg.criterion import SetCriterion, PaddedTargets
    from visionseg.model import M2FConfig
    optim.FlatOptimizer.step = _flatref.flat_step_reference
    init_distributed("gloo")
    x = data[rank:rank + 1]
    tr = Trainer(TinyNet(), _mse_criterion, _solver(optimizer, clip), device="cpu")
    assert tr.distributed and len(tr.opt.layout.buckets) > 2
    for _ in range(3):
        tr.step(x, None, None)
    flat = tr.opt.master.detach().clone()
    # criterion num_masks is the global mean over ranks (upstream SetCriterion semantics)
    crit = SetCriterion(M2FConfig(num_queries=5))
    tg = PaddedTargets.from_lists([torch.zeros(rank + 1, 4, 4, dtype=torch.bool)],
                                  [torch.zeros(rank + 1, dtype=torch.int64)], device="cpu")
    n = crit._num_masks(tg, torch.device("cpu"))
    out_q.put((rank, flat.numpy().copy(), float(n)))   # by value: no shared-memory tensor handles
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("optimizer,clip", [("sgd", "norm"), ("adamw", "full_model")])
def test_ddp_matches_single_process(monkeypatch, optimizer, clip):
    import _flatref
    from visionseg import optim
    from visionseg.train import Trainer
    torch.manual_seed(1)
    data = torch.randn(2, 3, 16, 16)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, data, optimizer, clip, q)) for r in range(world)]
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
    # single process, global batch of 2: mean-reduced loss over per-image terms = the
    # average of the ranks' gradients
    monkeypatch.setattr(optim.FlatOptimizer, "step", _flatref.flat_step_reference)
    tr = Trainer(TinyNet(), lambda m, c, a, b: (sum(_mse_criterion([mm[i:i + 1] for mm in m],
                                                                   [cc[i:i + 1] for cc in c], a, b)[0]
                                                    for i in range(2)) / 2, {}),
                 _solver(optimizer, clip), device="cpu", distributed=False)
    init = {n: p.detach().clone() for n, p in TinyNet().named_parameters()}
    for _ in range(3):
        tr.step(data, None, None)
    ref = tr.opt.master.detach()
    assert torch.allclose(f0, ref, atol=1e-6), float((f0 - ref).abs().max())
    # the unused parameter got no gradient on any rank: skipped (torch.optim semantics: no
    # weight decay, no momentum), so it still holds its initial value on every replica
    (o, n), = [off for off, nm in zip(tr.opt.layout.offsets, tr.opt.names) if nm == "unused"]
    for flat in (f0, f1, ref):
        assert torch.equal(flat[o:o + n], init["unused"])
    assert not torch.equal(ref, torch.zeros_like(ref))


def test_flat_layout_buckets_and_groups():
    """Parameter groups (no decay on norm parameters; AdamW: none on embeddings and
    relative-position tables, 0.1 lr on the backbone) and the flat layout: aligned,
    non-overlapping, buckets contiguous and in backward order."""
    from visionseg.optim import FlatLayout, param_hyper, ALIGN
    from visionseg.train import SolverConfig
    from oracle.ref_solver import ref_param_groups

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.backbone = torch.nn.Sequential(torch.nn.Linear(4, 5), torch.nn.LayerNorm(5))
            self.emb = torch.nn.Embedding(7, 3)
            self.head = torch.nn.Linear(5, 2)
            self.gn = torch.nn.GroupNorm(1, 2)
            self.backbone.rel_table = torch.nn.Parameter(torch.zeros(9, 2))

    m = M()
    for opt in ("sgd", "adamw"):
        s = SolverConfig(optimizer=opt)
        got = {n: (lrm * s.lr, wd) for n, _, lrm, wd in param_hyper(m, s)}
        exp = {g["name"]: (g["lr"], g["weight_decay"]) for g in ref_param_groups(m, s.lr, s.weight_decay, opt)}
        assert got.keys() == exp.keys()
        for k in exp:
            assert got[k] == pytest.approx(exp[k]), (opt, k)
    lay = FlatLayout(param_hyper(m, SolverConfig()), bucket_cap_mb=40 * 4 / 2 ** 20)
    end = 0
    for (o, n) in lay.offsets:
        assert o % ALIGN == 0 and o >= end
        end = o + n
    assert lay.entries[0][0] == "gn.bias"                   # reverse registration order
    prev = 0
    for lo, hi, ids in lay.buckets:
        assert lo == prev and hi > lo
        prev = hi
        assert all(lay.bucket_of[i] == lay.buckets.index((lo, hi, ids)) for i in ids)
    assert prev == lay.size and len(lay.buckets) > 1
    # the gradient flags sit after the parameters, inside the last bucket
    assert lay.flag_off == lay.total and lay.size >= lay.total + lay.num_params
    assert lay.buckets[-1][0] <= lay.flag_off and lay.buckets[-1][1] == lay.size
    assert lay.table[:, 4].tolist() == lay.chunk_param


class _StubEvent:
    """Stands in for optim.ExternalEvent on CPU (no HIP): logs record / wait order."""
    log = []

    def __init__(self):
        self.id = len([e for e in _StubEvent.log if e[0] == "new"])
        _StubEvent.log.append(("new", self.id))

    def record(self, stream=None):
        _StubEvent.log.append(("record", self.id))

    def wait(self, stream):
        _StubEvent.log.append(("wait", self.id))


class _StubStream:
    def wait_stream(self, other):
        pass


def _capture_worker(rank, world, port, data, out_q):
    """GradReducer in "capture" mode (what a captured HIP-graph step records) followed by
    replay_collectives() (what the trainer issues after launching the graph), with the
    HIP events and streams stubbed: bucket events recorded in bucket order during the
    backward, one all-reduce per bucket in index order behind its event, the f32 sums of
    the ranks' gradients in the buffer, and the same update as the eager path."""
    import contextlib
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import _flatref
    from visionseg import optim
    from visionseg.train import Trainer, init_distributed
    optim.FlatOptimizer.step = _flatref.flat_step_reference
    optim.ExternalEvent = _StubEvent
    torch.cuda.current_stream = lambda *a, **k: _StubStream()
    torch.cuda.stream = lambda s: contextlib.nullcontext()
    init_distributed("gloo")
    x = data[rank:rank + 1]
    res = {}
    for mode in ("eager", "capture"):
        tr = Trainer(TinyNet(), _mse_criterion, _solver("sgd", "norm"), device="cpu")
        red = tr.reducer
        nb = len(tr.opt.layout.buckets)
        calls = []
        real = dist.all_reduce

        def counting(t, *a, **k):
            calls.append((t.data_ptr() - red.buf.data_ptr()) // t.element_size())
            return real(t, *a, **k)
        dist.all_reduce = counting
        _StubEvent.log = []
        tr._set_lr()
        tr.opt.zero_grad()
        red.begin(mode)
        loss, _ = tr.forward_loss(x, None, None)
        loss.backward()
        red.finish_backward()
        if mode == "capture":
            assert not calls, "a collective was issued during the capture"
            recs = [e[1] for e in _StubEvent.log if e[0] == "record"]
            assert recs == list(range(nb)), recs                       # launch order = bucket index
            red.replay_collectives()
            waits = [e[1] for e in _StubEvent.log if e[0] == "wait"]
            assert waits == list(range(nb)), waits
        dist.all_reduce = real
        assert calls == [lo for lo, _, _ in tr.opt.layout.buckets], calls  # every bucket once, in order
        res[mode] = (red.buf.detach().clone(), None)
        tr.apply_gradients()
        res[mode] = (res[mode][0], tr.opt.master.detach().clone())
    out_q.put((rank, {m: (g.numpy().copy(), w.numpy().copy()) for m, (g, w) in res.items()}))
    dist.barrier()
    dist.destroy_process_group()


def test_grad_reducer_capture_mode_bucket_order():
    torch.manual_seed(1)
    data = torch.randn(2, 3, 16, 16)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_capture_worker, args=(r, world, port, data, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, r0), (_, r1) = res
    for mode in ("eager", "capture"):
        assert (r0[mode][0] == r1[mode][0]).all() and (r0[mode][1] == r1[mode][1]).all()
    # capture + replay == eager: the same reduced f32 gradients (flags included) and update
    assert (r0["capture"][0] == r0["eager"][0]).all()
    assert (r0["capture"][1] == r0["eager"][1]).all()
    # the reduced buffer holds the SUM over ranks: every flag of a used parameter is 2
    from visionseg.optim import FlatLayout, param_hyper
    from visionseg.train import SolverConfig
    lay = FlatLayout(param_hyper(TinyNet(), SolverConfig()), 1e-4)
    flags = r0["capture"][0][lay.flag_off:lay.flag_off + lay.num_params]
    used = [n != "unused" for n, _, _, _ in lay.entries]
    assert [float(f) for f in flags] == [2.0 if u else 0.0 for u in used]
