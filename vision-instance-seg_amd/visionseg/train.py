"""Data-parallel training step for the Swin + Mask2Former path.

One process per GPU (torchrun-style env: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*),
`torch.distributed` with backend "nccl" (= RCCL on ROCm, over xGMI inside a node) or
"gloo" on CPU.  Image batches are sharded by rank (independent images, per-rank seed
42 + rank); the only exchanges are the bucketed f32 gradient all-reduce, overlapped
with the backward pass (optim.GradReducer: from autograd hooks in eager steps, behind
in-graph events in graph-replayed steps), and the scalar `num_masks` all-reduce of the
criterion (upstream SetCriterion; HF:m2f:781-794).

Solver semantics follow the reference (training/maskdino/train_full.py:246-271 on top of
detectron2's DefaultTrainer, which it does not override, :153-167; restated in
oracle/ref_solver.py): SGD momentum 0.9, BASE_LR 1e-4, WEIGHT_DECAY 0.05 (MaskDINO base
config, upstream) with 0 on normalisation parameters (WEIGHT_DECAY_NORM), WarmupMultiStep
(warmup 200 iters, steps 3500/4500, gamma 0.1), CLIP_GRADIENTS type "norm", value 0.01,
L2: detectron2's "norm" clips EACH parameter's gradient to norm 0.01 ("full_model", one
global norm, is provided too).  `optimizer="adamw"` gives upstream Mask2Former/MaskDINO
train_net.py's AdamW (train_template.py:49's "AdamW" hyper-parameter).  The reference
runs fp32 (SOLVER.AMP.ENABLED False, train_full.py:263); `precision` "bf16" keeps f32
master weights and optimiser state and computes in bf16.

The optimiser is csrc/optim.hip over flat buffers (optim.FlatOptimizer): the model's
parameters and gradients are views of one buffer each, and clip + decay + update + bf16
cast of the whole model is two kernels.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from dataclasses import dataclass

import torch
import torch.distributed as dist

from .optim import FlatOptimizer, GradReducer


@dataclass
class SolverConfig:
    lr: float = 1e-4
    optimizer: str = "sgd"           # "sgd" (the reference: detectron2 DefaultTrainer) | "adamw"
    momentum: float = 0.9            # SOLVER.MOMENTUM
    weight_decay: float = 0.05
    weight_decay_norm: float = 0.0   # SOLVER.WEIGHT_DECAY_NORM
    weight_decay_embed: float = 0.0  # AdamW / upstream train_net only
    backbone_multiplier: float = 0.1  # AdamW / upstream train_net only
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    clip_type: str = "norm"          # "norm" (per parameter, detectron2) | "full_model" | "none"
    clip_value: float = 0.01
    warmup_iters: int = 200
    warmup_factor: float = 0.001     # detectron2 SOLVER.WARMUP_FACTOR, linear warmup
    steps: tuple = (3500, 4500)
    gamma: float = 0.1
    amp: bool = True                 # reduced-precision compute on a cuda device (see `precision`)
    precision: str = "bf16"          # "bf16": bf16 params/activations + f32 master weights and state;
                                     # "amp": f32 params + bf16 autocast; "fp32" (also amp=False)
    bucket_cap_mb: float = 25.0      # f32 all-reduce bucket size
    schedule: str = "multistep"      # detectron2 WarmupMultiStep | "cosine" (train_template.py:51)
    max_iter: int = 5000
    conv_find: bool = True           # MIOpen Find over the convolution solvers (cudnn.benchmark):
                                     # the stride-4 3x3 conv fwd 0.68 -> 0.37 ms at C2 (tools/conv_bench.py)


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


def lr_at(cfg: SolverConfig, it: int) -> float:
    """WarmupMultiStepLR / WarmupCosineLR (detectron2 solver/lr_scheduler.py semantics)."""
    import math
    w = 1.0
    if it < cfg.warmup_iters:
        a = it / max(1, cfg.warmup_iters)
        w = cfg.warmup_factor * (1 - a) + a
    if cfg.schedule == "cosine":
        return cfg.lr * w * 0.5 * (1.0 + math.cos(math.pi * min(it, cfg.max_iter) / max(1, cfg.max_iter)))
    return cfg.lr * w * cfg.gamma ** sum(1 for s in cfg.steps if it >= s)


def graph_capture_safe() -> bool:
    """HIP graphs of the training step need ROCm's graph packet capture off
    (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0, read once when HIP initialises; see
    visionseg/__init__.py and tools/graph_diag.py): False if the flag is not "0" now, or
    if HIP was initialised before `import visionseg` put it in place."""
    import visionseg
    return os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE") == "0" and visionseg.GRAPH_CAPTURE_SAFE


class Trainer:
    """model: nn.Module returning (mask logits per decoder step, class logits per step);
    criterion: callable(masks, classes, mask_labels, class_labels) -> (loss, parts)."""

    def __init__(self, model, criterion, solver: SolverConfig | None = None, device=None,
                 distributed: bool | None = None, graphs: bool = False, graph_warmup: int = 2,
                 max_graphs: int = 8):
        self.solver = s = solver or SolverConfig()
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.model = model.to(self.device)
        self.criterion = criterion
        # the decoder keeps its training logits factored (ops.FactoredLogits) only for a
        # criterion that reads them; any other criterion gets [B,Q,H/4,W/4] tensors
        dec = getattr(model, "decoder", None)
        if dec is not None and hasattr(dec, "emit_factors"):
            dec.emit_factors = bool(getattr(criterion, "accepts_factored_logits", False))
        if s.conv_find and self.device.type == "cuda":
            # the first call of each conv shape benchmarks MIOpen's solvers (eager warm-up
            # steps, before any graph capture); later calls use the fastest
            torch.backends.cudnn.benchmark = True
        self.mode = "fp32"
        if s.amp and self.device.type == "cuda":
            self.mode = s.precision
        if self.mode == "bf16":
            self.model.to(torch.bfloat16)
        if distributed is None:
            distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self.distributed = bool(distributed)
        self.world = dist.get_world_size() if self.distributed else 1
        if self.distributed:
            with torch.no_grad():                       # replicas start identical (rank 0's init)
                for t in list(self.model.parameters()) + list(self.model.buffers()):
                    dist.broadcast(t, 0)
        self.opt = FlatOptimizer(self.model, s, self.device, self.world)
        self.reducer = GradReducer(self.opt) if self.distributed else None
        # HIP-graph replay of the whole step (on a device): with several ranks the step is
        # two graphs (forward+backward, optimiser) with the bucket all-reduces issued
        # between them behind in-graph events
        self.graphs = bool(graphs) and self.device.type == "cuda" and self.mode == "bf16"
        if self.graphs and not graph_capture_safe():
            raise RuntimeError(
                "Trainer(graphs=True) needs DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 set before HIP initialises "
                "(import visionseg before touching the GPU, or export it); graph replays faulted without it")
        self.split = self.graphs and self.distributed
        # at least two eager steps of a signature before its capture (lazy library state
        # and the optimiser's state exist before the capture records anything)
        self.graph_warmup = max(2, int(graph_warmup))
        # live graphs per signature, least recently replayed first; all of them capture into
        # ONE memory pool (see _capture), so keeping several costs the largest graph's
        # activations, not the sum
        self.max_graphs = max(1, int(max_graphs))
        self._graph_states, self._eager_seen = OrderedDict(), {}
        self._pool = None
        self.captures = 0
        if self.split:
            self.num_masks_total = torch.zeros((), device=self.device, dtype=torch.float32)
        self.iter = 0

    @property
    def params(self):
        """The trainable parameters in the optimiser's (flat) order."""
        return self.opt.params

    def master_params(self):
        """f32 master weights, per parameter (views of the flat master buffer)."""
        return self.opt.layout.views(self.opt.master)

    def forward_loss(self, images, mask_labels, class_labels):
        if getattr(self.model, "takes_targets", False):
            # MaskDINO: the targets (padded) and their boxes feed the denoising queries
            # and the box losses
            from .criterion import as_padded
            from .maskdino import masks_to_boxes
            tg = as_padded(mask_labels, class_labels, self.device)
            boxes = masks_to_boxes(tg.masks)
            with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.mode == "amp"):
                out = self.model(images, tg, boxes)
            return self.criterion(out, tg, boxes)
        with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.mode == "amp"):
            masks, classes = self.model(images)
        masks = [m.float() for m in masks]
        classes = [c.float() for c in classes]
        return self.criterion(masks, classes, mask_labels, class_labels)

    # ----------------------------------------------------------------- step phases
    def forward_backward(self, images, mask_labels, class_labels, reduce_mode: str = "eager"):
        """Forward + loss + backward, the gradients packed into the flat buffer; with
        several ranks each bucket is packed and reduced as it completes.
        Returns (loss, loss components)."""
        self.opt.zero_grad()
        if self.reducer is not None:
            self.reducer.begin(reduce_mode)
        loss, parts = self.forward_loss(images, mask_labels, class_labels)
        loss.backward()
        if self.reducer is not None:
            self.reducer.finish_backward()
        else:
            self.opt.gather_grads()
        return loss.detach(), parts

    def apply_gradients(self):
        """clip + weight decay + update + bf16 cast (csrc/optim.hip)."""
        self.opt.step()

    def _set_lr(self):
        self.opt.set_lr(lr_at(self.solver, self.iter))

    def eager_step(self, images, mask_labels, class_labels):
        self._set_lr()
        loss, _ = self.forward_backward(images, mask_labels, class_labels)
        self.apply_gradients()
        return loss

    # ----------------------------------------------------------- graph-replayed step
    def _set_num_masks(self, class_labels):
        """split mode: the criterion's global target count, all-reduced eagerly (it is a
        graph input, not a collective inside the capture)."""
        self.num_masks_total.fill_(float(sum(int(t.shape[0]) for t in class_labels)))
        dist.all_reduce(self.num_masks_total)
        self.criterion.num_masks_total = self.num_masks_total

    def _capture(self, images, mask_labels, class_labels, kc):
        # static inputs: the image batch and the targets padded to kc (criterion.PaddedTargets),
        # so every batch with the same image shape and largest target count replays this graph
        from .criterion import PaddedTargets
        st = {"images": images.clone(), "tg": PaddedTargets.from_lists(mask_labels, class_labels, kc=kc,
                                                                       device=self.device), "graphs": []}
        torch.cuda.synchronize(self.device)
        # every signature's graph captures into the trainer's one private pool: a block that
        # is a temporary of one graph may be a temporary of another, which is safe because
        # the graphs replay one after another on one stream and nothing a graph leaves
        # behind is read after another replay (the loss is cloned right after its replay;
        # gradients, weights and optimiser state live outside the pool).  The BLAS
        # workspace cached per (handle, capture stream) is dropped before and after every
        # capture, so each graph allocates its own inside the pool
        # (torch/_inductor/cudagraph_trees.py clear_cublass_cache does the same)
        # a pool lives while a graph holds it: once the last graph is reset, the allocator
        # releases it and its handle cannot be captured into again
        if self._pool is None or not self._graph_states:
            self._pool = torch.cuda.graph_pool_handle()
        pool = self._pool
        torch._C._cuda_clearCublasWorkspaces()
        # "thread_local" capture: other threads keep using the device while this one
        # captures -- RCCL's watchdog querying the events of earlier collectives (several
        # ranks), and the data loader's pin-memory thread pinning the next batches (the
        # seam: a "global" capture was invalidated by the pinning, tools/seam_bench.py)
        mode = "thread_local"
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1, pool=pool, capture_error_mode=mode):
            st["loss"], _ = self.forward_backward(st["images"], st["tg"], None, reduce_mode="capture")
            if not self.split:
                self.apply_gradients()
        st["graphs"].append(g1)
        if self.split:
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2, pool=pool, capture_error_mode=mode):
                self.apply_gradients()
            st["graphs"].append(g2)
        torch.cuda.synchronize(self.device)
        torch._C._cuda_clearCublasWorkspaces()
        from .model import cached_constants
        st["constants"] = cached_constants()      # alive as long as the graphs that read them
        self.captures += 1
        return st

    def _drop_graphs(self, keep: int = 0):
        """Destroy graphs, least recently replayed first, until at most `keep` remain."""
        if len(self._graph_states) <= keep:
            return
        while len(self._graph_states) > keep:
            _, st = self._graph_states.popitem(last=False)
            for g in st["graphs"]:
                g.reset()
        torch.cuda.synchronize(self.device)

    @staticmethod
    def target_capacity(class_labels) -> int:
        """Padded target capacity of a batch: its largest target count rounded up to a
        multiple of 4 up to 16, to the next power of two above, so batches whose counts
        vary (real COCO data) share a few graphs.  The padding slots carry no loss and
        no matching cost (criterion.PaddedTargets), so the capacity changes no result."""
        kc = max([int(c.shape[0]) for c in class_labels] + [0])
        if kc <= 16:
            return max(4, (kc + 3) // 4 * 4)
        return 1 << (kc - 1).bit_length()

    def _graph_step(self, images, mask_labels, class_labels):
        kc = self.target_capacity(class_labels)
        key = (tuple(images.shape), images.dtype, kc, tuple(mask_labels[0].shape[-2:]) if mask_labels else ())
        st = self._graph_states.get(key)
        if st is not None:
            self._graph_states.move_to_end(key)
        else:
            seen = self._eager_seen.get(key, 0)
            if seen < self.graph_warmup:
                # eager steps first: lazy library state and the optimiser's state exist
                # before the capture (a capture records launches, it runs nothing)
                self._eager_seen[key] = seen + 1
                if self.split:
                    self._set_num_masks(class_labels)
                return self.eager_step(images, mask_labels, class_labels)
            self._drop_graphs(keep=self.max_graphs - 1)      # the least recently replayed goes
            st = self._graph_states[key] = self._capture(images, mask_labels, class_labels, kc)
        self._set_lr()
        with torch.no_grad():
            st["images"].copy_(images)
            st["tg"].copy_from_lists(mask_labels, class_labels)
        if self.split:
            self._set_num_masks(class_labels)
            st["graphs"][0].replay()
            self.reducer.replay_collectives()
            st["graphs"][1].replay()
        else:
            st["graphs"][0].replay()
        return st["loss"].clone()

    def step(self, images, mask_labels, class_labels):
        """One optimisation step; returns the (device) loss tensor, no host sync.  With
        graphs=True the step is captured per signature (image shape, padded target
        capacity of the batch; after `graph_warmup` eager steps of it) and replayed with the batch's
        targets padded into static buffers (capacity: the largest count rounded up to a
        multiple of 4): one launch per graph instead of ~3000 per step.  Up to `max_graphs`
        signatures keep their graphs (least recently replayed dropped first), all in one
        memory pool, so a stream of mixed shapes (multi-scale COCO batches) replays instead
        of recapturing."""
        if self.graphs:
            loss = self._graph_step(images, mask_labels, class_labels)
        else:
            loss = self.eager_step(images, mask_labels, class_labels)
        self.iter += 1
        return loss

    # ------------------------------------------------------------------ checkpoints
    def state_dict(self):
        """The model's state dict with the f32 master weights under the model's names,
        the flat optimiser state, and the iteration."""
        sd = {k: v.float() if v.is_floating_point() else v for k, v in self.model.state_dict().items()}
        sd.update({n: m.detach().cpu().clone() for n, m in zip(self.opt.names, self.master_params())})
        return {"model": sd, "optimizer": self.opt.state_dict(), "iter": self.iter}

    def save(self, path):
        """Checkpoint (rank 0 writes; detectron2 PeriodicCheckpointer equivalent)."""
        if not dist.is_initialized() or dist.get_rank() == 0:
            torch.save(self.state_dict(), path)

    def load(self, path):
        """Resume: weights, optimiser state and iteration.  Captured graphs are dropped
        first (they hold the previous run's static inputs) and recaptured on demand."""
        self._drop_graphs()
        self._eager_seen.clear()
        sd = torch.load(path, map_location="cpu", weights_only=True)
        with torch.no_grad():
            self.model.load_state_dict({k: v for k, v in sd["model"].items() if k not in self.opt.names},
                                       strict=False)
            self.opt.load_master(sd["model"])
        self.opt.load_state_dict(sd["optimizer"])
        self.iter = int(sd["iter"])
