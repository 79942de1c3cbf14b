"""Data-parallel training step for the Swin + Mask2Former path.

One process per GPU (torchrun-style env: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*),
`torch.distributed` with backend "nccl" (= RCCL on ROCm, over xGMI inside a node) or
"gloo" on CPU.  Image batches are sharded by rank (independent images, per-rank seed
42 + rank); the only exchanges are the bucketed gradient all-reduce, which DDP
launches from autograd hooks on its communication stream while the backward pass is
still running (overlapped with the remaining backward kernels), and the scalar
`num_masks` all-reduce of the criterion (upstream SetCriterion; HF:m2f:781-794).

Solver semantics follow the reference's detectron2 config
(training/maskdino/train_full.py:246-271): AdamW lr 1e-4 (train_template.py:47-50),
WarmupMultiStep (warmup 200 iters, steps 3500/4500, gamma 0.1), bf16 autocast when
AMP is on (train_experiments.py:229-230), and CLIP_GRADIENTS type "norm", value 0.01,
L2 — detectron2's "norm" clips EACH parameter's gradient to norm 0.01 (its
"full_model" type would clip the global norm; both are provided).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist
from torch.nn.parallel import DistributedDataParallel as DDP


@dataclass
class SolverConfig:
    lr: float = 1e-4
    weight_decay: float = 0.05
    betas: tuple = (0.9, 0.999)
    clip_type: str = "norm"          # "norm" (per parameter, detectron2) | "full_model" | "none"
    clip_value: float = 0.01
    warmup_iters: int = 200
    warmup_factor: float = 0.001     # detectron2 SOLVER.WARMUP_FACTOR, linear warmup
    steps: tuple = (3500, 4500)
    gamma: float = 0.1
    amp: bool = True                 # bf16 compute on a cuda device (see `precision`)
    precision: str = "bf16"          # "bf16": bf16 params/activations + f32 master weights in the
                                     # optimizer; "amp": f32 params + bf16 autocast; "fp32"
    bucket_cap_mb: int = 64
    schedule: str = "multistep"      # detectron2 WarmupMultiStep | "cosine" (train_template.py:51)
    max_iter: int = 5000


def dist_env():
    """(rank, local_rank, world_size) from the torchrun environment (defaults 0,0,1)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def init_distributed(backend: str | None = None):
    rank, local, world = dist_env()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, local, world


def _lr_lambda(cfg: SolverConfig):
    import math

    def f(it):
        w = 1.0
        if it < cfg.warmup_iters:
            a = it / max(1, cfg.warmup_iters)
            w = cfg.warmup_factor * (1 - a) + a
        if cfg.schedule == "cosine":
            return w * 0.5 * (1.0 + math.cos(math.pi * min(it, cfg.max_iter) / max(1, cfg.max_iter)))
        return w * cfg.gamma ** sum(1 for s in cfg.steps if it >= s)
    return f


class Trainer:
    """model: nn.Module returning (mask logits per decoder step, class logits per step);
    criterion: callable(masks, classes, mask_labels, class_labels) -> (loss, parts)."""

    def __init__(self, model, criterion, solver: SolverConfig | None = None, device=None,
                 distributed: bool | None = None, graphs: bool = False, graph_warmup: int = 2):
        self.solver = solver or SolverConfig()
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.model = model.to(self.device)
        self.criterion = criterion
        s = self.solver
        self.mode = "fp32"
        if s.amp and self.device.type == "cuda":
            self.mode = s.precision
        if self.mode == "bf16":
            self.model.to(torch.bfloat16)
        if distributed is None:
            distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self.distributed = distributed
        # HIP-graph replay of the whole step (bf16 mode on a device; see step()): with
        # several ranks the gradient all-reduce stays an eager RCCL call between two
        # graphs (no collective inside a capture), so DDP's hooks are not used
        self.graphs = bool(graphs) and self.device.type == "cuda" and self.mode == "bf16"
        self.split = self.graphs and distributed
        # at least two eager steps of a signature before its capture (lazy library state
        # and the optimiser's moments exist before the capture records anything)
        self.graph_warmup = max(2, int(graph_warmup))
        self._graph_states, self._eager_seen = {}, {}
        if self.split:
            self.net = self.model
            with torch.no_grad():                       # DDP's start-up broadcast from rank 0
                for t in list(self.model.parameters()) + list(self.model.buffers()):
                    dist.broadcast(t, 0)
        elif distributed:
            kw = dict(bucket_cap_mb=self.solver.bucket_cap_mb, gradient_as_bucket_view=True, broadcast_buffers=False)
            if self.device.type == "cuda":
                kw["device_ids"] = [self.device.index]
            self.net = DDP(self.model, **kw)
        else:
            self.net = self.model
        params = [p for p in self.model.parameters() if p.requires_grad]
        self.model_params = params
        self.flat = None
        if self.mode == "bf16":
            # f32 master copy owned by the optimiser, packed in one flat buffer (and the f32
            # master grads in another) so the per-parameter clip is two kernels; the model
            # keeps bf16 working weights
            from .ops import FlatParams
            self.flat = FlatParams([p.shape for p in params], self.device)
            self.flat_master, self.flat_grad = self.flat.buffer(), self.flat.buffer()
            self.params = []
            with torch.no_grad():
                for v, g, p in zip(self.flat.views(self.flat_master), self.flat.views(self.flat_grad), params):
                    v.copy_(p.detach().float())
                    m = torch.nn.Parameter(v)
                    m.grad = g
                    self.params.append(m)
        else:
            self.params = params
        fused = self.device.type == "cuda"
        okw = dict(fused=fused, foreach=None if fused else True)
        lr = self.solver.lr
        if self.graphs:
            # device-side step count and a tensor lr: replays see the scheduler's updates
            okw["capturable"] = True
            lr = torch.tensor(lr, device=self.device, dtype=torch.float32)
        self.opt = torch.optim.AdamW(self.params, lr=lr, betas=self.solver.betas,
                                     weight_decay=self.solver.weight_decay, **okw)
        if self.split:
            self.flat_g16 = torch.zeros(self.flat.total, device=self.device, dtype=torch.bfloat16)
            self.g16_views = self.flat.views(self.flat_g16)
            self.num_masks_total = torch.zeros((), device=self.device, dtype=torch.float32)
        self.sched = torch.optim.lr_scheduler.LambdaLR(self.opt, _lr_lambda(self.solver))
        if self.graphs:
            # float bases: the scheduler then fills the lr tensor from a host float (a tensor
            # base would make it read the value back, one host sync per step)
            self.sched.base_lrs = [float(self.solver.lr) for _ in self.opt.param_groups]
        self.iter = 0

    @torch.no_grad()
    def clip_gradients(self):
        s = self.solver
        grads = [p.grad for p in self.params if p.grad is not None]
        if not grads or s.clip_type == "none":
            return
        if s.clip_type == "full_model":
            torch.nn.utils.clip_grad_norm_(self.params, s.clip_value)
            return
        if self.flat is not None and self.device.type == "cuda":
            self.flat.clip_(self.flat_grad, s.clip_value)      # csrc/optim.hip, 2 launches
            return
        # detectron2 "norm": clip_grad_norm_(p, clip_value) for every parameter, fused
        # (one stacked scale vector: a handful of launches instead of several per parameter)
        norms = torch.stack(torch._foreach_norm(grads))
        scales = (s.clip_value / (norms + 1e-6)).clamp_(max=1.0)
        torch._foreach_mul_(grads, list(scales.unbind(0)))

    def forward_loss(self, images, mask_labels, class_labels):
        with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.mode == "amp"):
            masks, classes = self.net(images)
        masks = [m.float() for m in masks]
        classes = [c.float() for c in classes]
        return self.criterion(masks, classes, mask_labels, class_labels)

    # ----------------------------------------------------------- graph-replayed step
    def _phase1(self, images, mask_labels, class_labels):
        """Forward + loss + backward, then the gradients into the flat buffer of the next
        phase (f32 master grads; bf16 all-reduce buffer when split)."""
        for p in self.model_params:
            p.grad = None
        loss, _ = self.forward_loss(images, mask_labels, class_labels)
        loss.backward()
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in self.model_params]
        with torch.no_grad():
            torch._foreach_copy_(self.g16_views if self.split else [m.grad for m in self.params], grads)
        return loss.detach()

    @torch.no_grad()
    def _phase2(self):
        """(split: averaged bf16 grads -> f32 master grads) clip, AdamW, master -> bf16."""
        if self.split:
            torch._foreach_copy_([m.grad for m in self.params], self.g16_views)
            self.flat_grad.mul_(1.0 / dist.get_world_size())
        self.clip_gradients()
        self.opt.step()
        torch._foreach_copy_(self.model_params, self.params)

    def _set_num_masks(self, class_labels):
        """split mode: the criterion's global target count, all-reduced eagerly (it is a
        graph input, not a collective inside the capture)."""
        self.num_masks_total.fill_(float(sum(int(t.shape[0]) for t in class_labels)))
        dist.all_reduce(self.num_masks_total)
        self.criterion.num_masks_total = self.num_masks_total

    def _eager_split_step(self, images, mask_labels, class_labels):
        self._set_num_masks(class_labels)
        loss = self._phase1(images, mask_labels, class_labels)
        dist.all_reduce(self.flat_g16)
        self._phase2()
        return loss

    def _capture(self, images, mask_labels, class_labels, kc):
        # static inputs: the image batch and the targets padded to kc (criterion.PaddedTargets),
        # so every batch with the same image shape and largest target count replays this graph
        from .criterion import PaddedTargets
        st = {"images": images.clone(), "tg": PaddedTargets.from_lists(mask_labels, class_labels, kc=kc,
                                                                       device=self.device), "graphs": []}
        torch.cuda.synchronize(self.device)
        # one live graph per trainer (see _graph_step).  The BLAS workspace cached per
        # (handle, capture stream) is dropped before and after every capture, so each
        # graph allocates its own inside its pool (torch/_inductor/cudagraph_trees.py
        # clear_cublass_cache does the same)
        pool = torch.cuda.graph_pool_handle()
        torch._C._cuda_clearCublasWorkspaces()
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1, pool=pool):
            st["loss"] = self._phase1(st["images"], st["tg"], None)
            if not self.split:
                self._phase2()
        st["graphs"].append(g1)
        if self.split:
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2, pool=pool):
                self._phase2()
            st["graphs"].append(g2)
        torch.cuda.synchronize(self.device)
        torch._C._cuda_clearCublasWorkspaces()
        return st

    def _drop_graphs(self):
        if not self._graph_states:
            return
        for p in self.model_params:          # gradients living in the old graph's pool
            p.grad = None
        for st in self._graph_states.values():
            for g in st["graphs"]:
                g.reset()
        self._graph_states.clear()
        torch.cuda.synchronize(self.device)

    def _graph_step(self, images, mask_labels, class_labels):
        kc = max([int(c.shape[0]) for c in class_labels] + [0])
        key = (tuple(images.shape), images.dtype, kc, tuple(mask_labels[0].shape[-2:]) if mask_labels else ())
        st = self._graph_states.get(key)
        if st is None:
            # one live graph per trainer (bounded pool memory): another signature's graph
            # is destroyed before any eager work of this one, and a returning signature is
            # captured again.  (Replays that faulted after a recapture were ROCm's graph
            # packet capture, disabled in visionseg/__init__.py; tools/graph_diag.py.)
            self._drop_graphs()
            seen = self._eager_seen.get(key, 0)
            if seen < self.graph_warmup:
                # eager steps first: lazy library state and the optimiser's moments exist
                # before the capture (a capture records launches, it runs nothing)
                self._eager_seen[key] = seen + 1
                return self._eager_split_step(images, mask_labels, class_labels) if self.split else \
                    self._eager_bf16_step(images, mask_labels, class_labels)
            st = self._graph_states[key] = self._capture(images, mask_labels, class_labels, kc)
        with torch.no_grad():
            st["images"].copy_(images)
            st["tg"].copy_from_lists(mask_labels, class_labels)
        if self.split:
            self._set_num_masks(class_labels)
            st["graphs"][0].replay()
            dist.all_reduce(self.flat_g16)
            st["graphs"][1].replay()
        else:
            st["graphs"][0].replay()
        return st["loss"].clone()

    def _eager_bf16_step(self, images, mask_labels, class_labels):
        loss = self._phase1(images, mask_labels, class_labels)
        self._phase2()
        return loss

    def step(self, images, mask_labels, class_labels):
        """One optimisation step; returns the (device) loss tensor, no host sync.  With
        graphs=True the step is captured per signature (image shape, largest target count
        of the batch; after `graph_warmup` eager steps of it) and replayed with the batch's
        targets padded into static buffers: one launch per graph instead of ~3200 per
        step.  One signature's graph lives at a time: another signature destroys it and is
        captured in its place."""
        if self.graphs:
            loss = self._graph_step(images, mask_labels, class_labels)
            self.sched.step()
            self.iter += 1
            return loss
        if self.mode != "bf16":
            self.opt.zero_grad(set_to_none=True)
        for p in self.model_params:
            p.grad = None
        loss, _ = self.forward_loss(images, mask_labels, class_labels)
        loss.backward()
        if self.mode == "bf16":
            # (DDP has already averaged the bf16 grads) -> the flat f32 master grads, one
            # multi-tensor cast-copy
            grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in self.model_params]
            torch._foreach_copy_([m.grad for m in self.params], grads)
        self.clip_gradients()
        self.opt.step()
        if self.mode == "bf16":
            with torch.no_grad():
                torch._foreach_copy_(self.model_params, self.params)
        self.sched.step()
        self.iter += 1
        return loss.detach()

    def state_dict(self):
        if self.mode == "bf16":   # checkpoint the f32 master weights under the model's names
            names = [n for n, p in self.model.named_parameters() if p.requires_grad]
            sd = {k: v.float() for k, v in self.model.state_dict().items()}
            sd.update({n: m.detach().clone() for n, m in zip(names, self.params)})
        else:
            sd = self.model.state_dict()
        return {"model": sd, "optimizer": self.opt.state_dict(),
                "scheduler": self.sched.state_dict(), "iter": self.iter}

    def save(self, path):
        """Checkpoint (rank 0 writes; detectron2 PeriodicCheckpointer equivalent)."""
        if not dist.is_initialized() or dist.get_rank() == 0:
            torch.save(self.state_dict(), path)

    def load(self, path):
        sd = torch.load(path, map_location=self.device, weights_only=True)
        self.model.load_state_dict(sd["model"])
        if self.mode == "bf16":
            names = [n for n, p in self.model.named_parameters() if p.requires_grad]
            with torch.no_grad():
                for n, m in zip(names, self.params):
                    m.copy_(sd["model"][n])
        self.opt.load_state_dict(sd["optimizer"])
        self.sched.load_state_dict(sd["scheduler"])
        self.iter = int(sd["iter"])
