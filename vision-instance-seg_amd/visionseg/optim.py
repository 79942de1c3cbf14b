"""Flat-buffer optimiser and bucketed gradient all-reduce of the training step.

The reference's solver (detectron2 DefaultTrainer, training/maskdino/train_full.py:153-167,
246-271; restated in oracle/ref_solver.py): parameter groups with no weight decay on
normalisation parameters, SGD momentum 0.9 (or upstream Mask2Former/MaskDINO's AdamW:
also no decay on embeddings / relative-position tables and a 0.1 backbone lr
multiplier), CLIP_GRADIENTS "norm" = clip_grad_norm_(p, 0.01) for every parameter.

MI355X layout: every per-parameter tensor of the optimiser lives in ONE flat buffer —
the model's working weights (bf16, the nn.Parameters become views of it), their
gradients (packed after the backward -- or per bucket, as buckets complete -- with
multi-tensor copies), the f32 master weights and the f32 optimiser state.  The whole optimiser step is then two kernels
(csrc/optim.hip: per-chunk sum of squares, then clip + decay + update + bf16 cast) and a
gradient bucket is a contiguous slice that RCCL reduces in place.

Gradient all-reduce (`GradReducer`, data parallel, one process per GPU): parameters are
laid out in reverse registration order (≈ the order backward produces their gradients)
and cut into ~`bucket_cap_mb` buckets.  A post-accumulate-grad hook counts each
bucket's gradients; when one is complete its slice is widened to f32 (the reduction runs
in f32: summing 8 bf16 gradient replicas in bf16 would round at every ring hop) and
  * eager steps: all-reduced right away with `async_op=True` — RCCL's stream waits for the
    compute stream at that point, so the reduction overlaps the rest of the backward;
  * captured steps (HIP graphs): an EXTERNAL event (`ExternalEvent`, csrc/stream.hip:
    torch refuses `Event(external=True)` on ROCm) is recorded in the graph at that
    point instead; after the graph is launched, the collectives are issued eagerly on a
    side stream that waits on those events, so they again overlap the remaining
    backward kernels of the replay, and no collective is ever captured.
Buckets are launched strictly in index order on every rank (as DDP does), whatever order
their gradients complete in.
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist
import torch.nn as nn

from . import _lib as L
from .profiling import timed

_NORMS = (nn.BatchNorm1d, nn.BatchNorm2d, nn.BatchNorm3d, nn.SyncBatchNorm, nn.GroupNorm, nn.InstanceNorm1d,
          nn.InstanceNorm2d, nn.InstanceNorm3d, nn.LayerNorm, nn.LocalResponseNorm)
ALIGN = 8                 # elements: 16-B vector access of bf16, 32-B of f32
CHUNK = 1 << 14           # elements per optimiser block (a parameter spans one or more chunks)


def param_hyper(model: nn.Module, solver):
    """[(name, param, lr multiplier, weight decay)] for every trainable parameter, in
    registration order (detectron2 get_default_optimizer_params semantics; AdamW adds the
    upstream Mask2Former train_net.py rules)."""
    out, seen = [], set()
    for mname, module in model.named_modules():
        for pname, p in module.named_parameters(recurse=False):
            if not p.requires_grad or id(p) in seen:
                continue
            seen.add(id(p))
            name = f"{mname}.{pname}" if mname else pname
            wd, lrm = solver.weight_decay, 1.0
            if isinstance(module, _NORMS):
                wd = solver.weight_decay_norm
            if solver.optimizer == "adamw":
                if isinstance(module, nn.Embedding) or pname in ("rel_table", "absolute_pos_embed"):
                    wd = solver.weight_decay_embed
                if name.startswith("backbone."):
                    lrm = solver.backbone_multiplier
            out.append((name, p, lrm, wd))
    return out


class FlatLayout:
    """Offsets of the parameters in the flat buffers (reverse registration order,
    ALIGN-aligned), the optimiser chunk table and the all-reduce buckets.

    The gradient buffers carry one FLAG per parameter after the parameters
    ([flag_off, flag_off + num_params)): 1 when the parameter got a gradient this step.
    The flags belong to the last bucket, so the all-reduce sums them across ranks (a
    parameter with a gradient on any rank is updated, as DDP does) and the last bucket
    launches after every other bucket has written its flags."""

    def __init__(self, entries, bucket_cap_mb: float = 25.0):
        self.entries = list(reversed(entries))          # backward order
        self.offsets, off = [], 0
        for _, p, _, _ in self.entries:
            n = p.numel()
            self.offsets.append((off, n))
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        self.total = off                                  # parameter elements (weights, state)
        self.num_params = len(self.entries)
        self.flag_off = off
        self.size = off + (self.num_params + ALIGN - 1) // ALIGN * ALIGN      # gradient buffers
        rows, hyper, self.chunk_param = [], [], []
        for i, ((o, n), (_, _, lrm, wd)) in enumerate(zip(self.offsets, self.entries)):
            first, count = len(rows), max(1, (n + CHUNK - 1) // CHUNK)
            for c in range(count):
                rows.append([o + c * CHUNK, max(0, min(CHUNK, n - c * CHUNK)), first, count, i])
                hyper.append([float(lrm), float(wd)])
                self.chunk_param.append(i)
        self.table = torch.tensor(rows, dtype=torch.int32)
        self.hyper = torch.tensor(hyper, dtype=torch.float32)
        self.num_chunks = len(rows)
        # buckets: consecutive parameters up to the cap (f32 bytes: what is reduced)
        cap = max(1, int(bucket_cap_mb * 2 ** 20 / 4))
        self.buckets, self.bucket_of = [], []
        lo, cur = 0, []
        for i, (o, n) in enumerate(self.offsets):
            if cur and o + n - lo > cap:
                self.buckets.append((lo, o, cur))
                lo, cur = o, []
            cur.append(i)
            self.bucket_of.append(len(self.buckets))
        if cur:
            self.buckets.append((lo, self.size, cur))

    def views(self, flat):
        return [flat[o:o + n].view(p.shape) for (o, n), (_, p, _, _) in zip(self.offsets, self.entries)]


class FlatOptimizer:
    """Owns the flat buffers; re-points the model's parameters (and their .grad) at them.

    dtype of the model's parameters decides the layout: bf16 -> bf16 working weights +
    f32 master copy; f32 -> the f32 master IS the working weight."""

    def __init__(self, model: nn.Module, solver, device, world: int = 1):
        self.solver = solver
        self.device = torch.device(device)
        self.world = int(world)
        entries = param_hyper(model, solver)
        if not entries:
            raise ValueError("the model has no trainable parameters")
        dtypes = {p.dtype for _, p, _, _ in entries}
        if len(dtypes) != 1 or next(iter(dtypes)) not in (torch.float32, torch.bfloat16):
            raise TypeError(f"parameters must all be f32 or all bf16, got {dtypes}")
        self.wdtype = next(iter(dtypes))
        self.layout = lay = FlatLayout(entries, solver.bucket_cap_mb)
        self.names = [n for n, _, _, _ in lay.entries]
        self.params = [p for _, p, _, _ in lay.entries]
        kw = dict(device=self.device)
        self.weights = torch.zeros(lay.total, dtype=self.wdtype, **kw)
        self.grads = torch.zeros(lay.size, dtype=self.wdtype, **kw)
        self.master = self.weights if self.wdtype == torch.float32 else torch.zeros(lay.total, dtype=torch.float32, **kw)
        # f32 all-reduce buffer (bf16 models with more than one rank)
        self.grads32 = (torch.zeros(lay.size, dtype=torch.float32, **kw)
                        if self.world > 1 and self.wdtype != torch.float32 else None)
        self.state1 = torch.zeros(lay.total, dtype=torch.float32, **kw)
        self.state2 = torch.zeros(lay.total, dtype=torch.float32, **kw) if solver.optimizer == "adamw" else None
        self.lr = torch.full((), float(solver.lr), dtype=torch.float32, **kw)
        self.step_count = torch.zeros((), dtype=torch.float32, **kw)
        self.param_steps = torch.zeros(lay.num_params, dtype=torch.float32, **kw)   # per parameter (AdamW)
        self.table = lay.table.to(self.device)
        self.hyper = lay.hyper.to(self.device)
        self.workspace = torch.empty(lay.num_chunks + 1, dtype=torch.float32, **kw)
        with torch.no_grad():
            wv, mv = lay.views(self.weights), lay.views(self.master)
            for p, w, m in zip(self.params, wv, mv):
                m.copy_(p.detach().float())
                if self.master is not self.weights:
                    w.copy_(p.detach())
            for p, w in zip(self.params, wv):
                p.data = w                          # the model now reads the flat buffer
        self.grad_views = lay.views(self.grads)
        self.reduce_views = lay.views(self.reduced_grads())
        self.flags = self.reduced_grads()[lay.flag_off:lay.flag_off + lay.num_params]
        self.flag_views = [self.flags[i:i + 1] for i in range(lay.num_params)]

    def zero_grad(self):
        """Before a backward: no .grad tensors, so autograd hands each parameter its
        gradient without an accumulate kernel (gather_grads packs them afterwards); every
        parameter's gradient flag set (gather_grads clears those that get none)."""
        for p in self.params:
            p.grad = None
        with torch.no_grad():
            self.flags.fill_(1.0)

    def gather_grads(self, ids=None):
        """Pack the parameters' .grad tensors (all, or those listed) into the buffer the
        update reads -- the f32 all-reduce buffer when there is one (the bf16 -> f32
        widening happens in this copy) -- with multi-tensor copies; a parameter that got
        no gradient this step gets zeros and its flag cleared: the step skips it (torch.optim
        skips a parameter whose .grad is None), unless another rank's gradient arrives."""
        idx = range(len(self.params)) if ids is None else ids
        src, dst, missing = [], [], []
        for i in idx:
            g = self.params[i].grad
            if g is None:
                missing.append(self.reduce_views[i])
            else:
                src.append(g)
                dst.append(self.reduce_views[i])
        with torch.no_grad():
            if src:
                torch._foreach_copy_(dst, src)
            if missing:
                torch._foreach_zero_(missing)
                torch._foreach_zero_([self.flag_views[i] for i in idx if self.params[i].grad is None])

    def set_lr(self, value: float):
        self.lr.fill_(float(value))

    def reduced_grads(self):
        """The buffer the update reads: the f32 all-reduce buffer when there is one."""
        return self.grads32 if self.grads32 is not None else self.grads

    @torch.no_grad()
    def step(self):
        """clip (per parameter / global / none) + weight decay + SGD or AdamW + bf16 cast,
        the gradients scaled by 1/world (they hold the all-reduce SUM)."""
        s = self.solver
        g = self.reduced_grads()
        L.require_hip(g)
        clip = {"none": 0, "norm": 1, "full_model": 2}[s.clip_type]
        opt = {"sgd": 0, "adamw": 1}[s.optimizer]
        w16 = self.weights if self.master is not self.weights else None
        nbytes = self.layout.total * (g.element_size() + (16 if opt else 8) + (2 if w16 is not None else 0)
                                      + (12 if opt else 8))
        with timed("flat_step", g, bytes_=nbytes):
            L.check(L.lib().vs_flat_step(
                L.dtype_code(g), L.ptr(g), L.ptr(self.flags), 1.0 / self.world, L.ptr(self.master), L.ptr(self.state1),
                L.ptr(self.state2) if self.state2 is not None else None, L.ptr(w16) if w16 is not None else None,
                L.ptr(self.table), L.ptr(self.hyper), self.layout.num_chunks, opt, clip, float(s.clip_value), 1e-6,
                float(s.momentum), float(s.betas[0]), float(s.betas[1]), float(s.eps), L.ptr(self.lr),
                L.ptr(self.step_count), L.ptr(self.param_steps), L.ptr(self.workspace), L.stream(g)), "flat_step")

    # ---------------------------------------------------------------- checkpoints
    def state_dict(self):
        return {"master": self.master.detach().cpu().clone(), "state1": self.state1.cpu().clone(),
                "state2": None if self.state2 is None else self.state2.cpu().clone(),
                "step": float(self.step_count), "param_steps": self.param_steps.cpu().clone(),
                "names": list(self.names), "optimizer": self.solver.optimizer}

    @torch.no_grad()
    def load_state_dict(self, sd):
        if list(sd["names"]) != self.names:
            raise ValueError("checkpoint parameters do not match the model")
        if sd.get("optimizer") != self.solver.optimizer:
            raise ValueError(f"checkpoint optimiser {sd.get('optimizer')} != {self.solver.optimizer}")
        self.master.copy_(sd["master"])
        self.state1.copy_(sd["state1"])
        if self.state2 is not None and sd["state2"] is not None:
            self.state2.copy_(sd["state2"])
        self.step_count.fill_(float(sd["step"]))
        if sd.get("param_steps") is not None:
            self.param_steps.copy_(sd["param_steps"])
        else:                                   # older checkpoints: one global count
            self.param_steps.fill_(float(sd["step"]))
        if self.master is not self.weights:
            self.weights.copy_(self.master)

    @torch.no_grad()
    def load_master(self, named: dict):
        """Copy f32 weights by parameter name into the master (and working) buffers."""
        for n, m in zip(self.names, self.layout.views(self.master)):
            m.copy_(named[n])
        if self.master is not self.weights:
            self.weights.copy_(self.master)


class ExternalEvent:
    """A HIP event recorded with hipEventRecordExternal (csrc/stream.hip): recorded during
    stream capture it becomes an event-record node of the graph, so an eager stream can
    wait for the point of a replay where it was recorded."""

    def __init__(self):
        h = ctypes.c_void_p()
        L.check(L.lib().vs_event_create(ctypes.byref(h)), "event_create")
        self.handle = h

    def record(self, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream()
        L.check(L.lib().vs_event_record_external(self.handle, ctypes.c_void_p(s.cuda_stream)), "event_record_external")

    def wait(self, stream):
        """`stream` waits for the event's last record."""
        L.check(L.lib().vs_stream_wait_event(ctypes.c_void_p(stream.cuda_stream), self.handle), "stream_wait_event")

    def __del__(self):
        try:
            L.lib().vs_event_destroy(self.handle)
        except Exception:
            pass


class GradReducer:
    """Bucketed gradient all-reduce overlapped with the backward pass (module docstring)."""

    def __init__(self, opt: FlatOptimizer, group=None):
        self.opt = opt
        self.group = group
        self.lay = opt.layout
        self.buf = opt.reduced_grads()
        self.nb = len(self.lay.buckets)
        self.cuda = self.buf.is_cuda
        # high priority: its own hardware queue (a default-priority stream can share the
        # compute stream's queue and then only runs after the replay), and the collectives
        # are scheduled ahead of the backward's kernels
        self.side = torch.cuda.Stream(device=self.buf.device, priority=-1) if self.cuda else None
        self.mode = "off"
        self.events = None
        self.hooks = [p.register_post_accumulate_grad_hook(self._hook(i)) for i, p in enumerate(opt.params)]
        self._reset()

    def _reset(self):
        self.remaining = [len(ids) for (_, _, ids) in self.lay.buckets]
        self.ready = [False] * self.nb
        self.next = 0
        self.works = []

    def begin(self, mode: str):
        """mode: "eager" (issue collectives from the hooks) or "capture" (record external
        events inside the graph being captured)."""
        self.mode = mode
        self._reset()
        if mode == "capture" and self.events is None:
            self.events = [ExternalEvent() for _ in range(self.nb)]     # reused by every capture

    def _hook(self, i):
        def fn(_p):
            if self.mode == "off":
                return
            b = self.lay.bucket_of[i]
            self.remaining[b] -= 1
            if self.remaining[b] == 0:
                self._ready(b)
        return fn

    def _ready(self, b):
        self.ready[b] = True
        while self.next < self.nb and self.ready[self.next]:
            self._launch(self.next)
            self.next += 1

    def _launch(self, b):
        lo, hi, ids = self.lay.buckets[b]
        self.opt.gather_grads(ids)                 # pack (and widen to f32) on the compute stream
        if self.mode == "eager":
            self.works.append(dist.all_reduce(self.buf[lo:hi], group=self.group, async_op=True))
        elif self.mode == "capture":
            self.events[b].record()

    def finish_backward(self):
        """After loss.backward(): buckets with parameters that received no gradient
        this step (unused parameters) are launched now, in order."""
        for b in range(self.nb):
            if not self.ready[b]:
                self.ready[b] = True
        while self.next < self.nb:
            self._launch(self.next)
            self.next += 1
        if self.mode == "eager":
            self.wait()
        self.mode = "off"

    def wait(self):
        for w in self.works:
            w.wait()                      # the current (compute) stream waits for RCCL
        self.works = []

    def replay_collectives(self):
        """After launching a graph captured in "capture" mode: one all-reduce per bucket on
        the side stream, each behind its bucket's in-graph event."""
        main = torch.cuda.current_stream(self.buf.device)
        # the side stream waits only on the in-graph events (waiting on `main` here would
        # wait for the whole replay and serialise the reduction behind the backward)
        with torch.cuda.stream(self.side):
            for b, (lo, hi, _) in enumerate(self.lay.buckets):
                self.events[b].wait(self.side)
                self.works.append(dist.all_reduce(self.buf[lo:hi], group=self.group, async_op=True))
        self.wait()
        main.wait_stream(self.side)
