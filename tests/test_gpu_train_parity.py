"""One fp32 TRAINING step of the MI355X path vs the oracle (ROADMAP item 1 of round 2).

Same weights, same batch, same point draws (tests/_draws.py, fed to both criteria), the
oracle's attention-mask decisions forced into the GPU decoder (threshold flips at
|logit| ~ 1e-6 are decisions, not arithmetic; tests/test_gpu_model.py measures them):

* oracle: RefMask2Former + RefCriterion (pinned to HF transformers 5.15.0) on CPU, then
  the reference's solver (oracle/ref_solver.py: detectron2 param groups, clip_grad_norm_
  per parameter = train_full.py:266-271, torch SGD momentum 0.9);
* product: visionseg.train.Trainer in fp32 mode on the GPU (HIP kernels, device
  matcher, flat-buffer optimiser csrc/optim.hip).

Checked: every weighted loss component of every decoder step (rel. 1e-4), every
parameter gradient (max error <= 2e-3 x that parameter's max |grad|, or x 1e-4 of the
largest gradient of the model where a parameter's own gradient is analytically ~0; 2e-2 for
the MSDA sampling-offset weights, whose gradient is discontinuous at cell edges; fp32
arithmetic in different summation orders over a 10-step decoder), and the weight update
of the step (max error <= 2e-3 x max |update| per parameter).
"""
import json
import os

import numpy as np
import pytest
import torch

from _draws import KeyedDraws
from oracle.detinit import det_init
from oracle.ref_model import RefConfig, RefCriterion, RefMask2Former
from oracle.ref_solver import ref_clip_per_parameter, ref_optimizer, ref_param_groups

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
GRAD_TOL = 2e-3
# MSDA sampling-offset weights: their gradient sums d(bilinear)/d(location) over every
# tap, and that derivative jumps where a tap crosses a cell edge (floor of the fp32
# coordinate); the GPU's single-rounding fma(y, H, -0.5) and the oracle's grid_sample
# unnormalisation put a handful of near-edge taps in different cells
OFFSET_GRAD_TOL = 2e-2
LOSS_TOL = 1e-4


def _setup(kind, golden):
    from visionseg.model import M2FConfig
    if kind == "tiny":
        d = golden("model_tiny.npz")
        cfgd = json.loads(str(d["config"]))
        cfg = M2FConfig.from_dict(cfgd)
        ref = RefMask2Former(RefConfig.from_dict(cfgd))
        sd = det_init({k: v.shape for k, v in ref.state_dict().items()}, int(d["weight_seed"]))
        return cfg, sd, 128
    cfg = M2FConfig.preset("swin_t")
    ref = RefMask2Former(RefConfig.from_dict(cfg.to_dict()))
    sd = det_init({k: v.shape for k, v in ref.state_dict().items()}, 77)
    return cfg, sd, 256


@pytest.mark.parametrize("kind", ["tiny", "swin_t"])
def test_training_step_vs_oracle(golden, kind):
    from visionseg.criterion import SetCriterion
    from visionseg.data import synthetic_batch
    from visionseg.model import Mask2Former
    from visionseg.train import SolverConfig, Trainer, lr_at
    cfg, sd, size = _setup(kind, golden)
    rcfg = RefConfig.from_dict(cfg.to_dict())
    ref = RefMask2Former(rcfg)
    ref.load_state_dict(sd)
    ref.train()
    prod = Mask2Former(cfg)
    prod.load_state_dict(sd)
    imgs, ml, cl = synthetic_batch(2, size, seed=4)
    draws = KeyedDraws(2, max(len(c) for c in cl) + 1, seed=5)
    s = SolverConfig(amp=False, optimizer="sgd", warmup_iters=0, lr=0.05)

    # ---- oracle: forward + loss + backward on CPU, then the reference's solver step
    ref.decoder.record = True
    rmasks, rclasses = ref(imgs)
    rloss, rparts = RefCriterion(rcfg, point_source=draws)(rmasks, rclasses, [m.float() for m in ml], cl)
    rloss.backward()
    rparams = dict(ref.named_parameters())
    rgrad = {n: p.grad.detach().clone() for n, p in rparams.items()}
    before = {n: p.detach().clone() for n, p in rparams.items()}
    ref_clip_per_parameter(list(rparams.values()), s.clip_value)
    ref_optimizer(ref_param_groups(ref, lr_at(s, 0), s.weight_decay, "sgd"), "sgd", s.momentum).step()

    # ---- product: the same step on the GPU
    crit = SetCriterion(cfg, matcher="device", point_source=draws)
    tr = Trainer(prod, crit, s, device=DEV)
    assert tr.mode == "fp32"
    prod.decoder.mask_override = [b for b, _ in ref.decoder.trace]
    tr._set_lr()
    loss, parts = tr.forward_backward(imgs.to(DEV), [m.to(DEV) for m in ml], [c.to(DEV) for c in cl])
    ggrad = {n: g.detach().cpu().clone() for n, g in zip(tr.opt.names, tr.opt.grad_views)}
    tr.apply_gradients()
    torch.cuda.synchronize()
    after = {n: m.detach().cpu() for n, m in zip(tr.opt.names, tr.master_params())}

    # ---- loss components
    assert set(parts) == set(rparts)
    worst_l = max(abs(float(parts[k]) - float(rparts[k])) / max(1e-3, abs(float(rparts[k]))) for k in rparts)
    # ---- gradients and weight updates, per parameter
    worst_g, worst_u, wg, wu = 0.0, 0.0, "", ""
    assert set(ggrad) == set(rgrad)
    # parameters whose gradient is analytically ~0 (e.g. the key bias of a softmax
    # attention: a shift of every score of a row) are compared on the global scale
    gscale = max(float(g.abs().max()) for g in rgrad.values())
    errs = {}
    for n in rgrad:
        den = max(float(rgrad[n].abs().max()), 1e-4 * gscale)
        e = errs[n] = float((ggrad[n] - rgrad[n]).abs().max()) / den
        if e > worst_g and "sampling_offsets" not in n:
            worst_g, wg = e, n
        ru = rparams[n].detach() - before[n]
        gu = after[n] - before[n]
        den = float(ru.abs().max())
        e = float((gu - ru).abs().max()) / max(den, 1e-12)
        if den > 0 and e > worst_u:
            worst_u, wu = e, n
    worst_off = max([e for n, e in errs.items() if "sampling_offsets" in n] + [0.0])
    top = sorted(errs.items(), key=lambda kv: -kv[1])[:4]
    print(f"{kind}: loss {float(loss):.6f} vs oracle {float(rloss):.6f}; worst loss-part rel err {worst_l:.2e}; "
          f"worst grad err {worst_g:.2e} ({wg}), sampling offsets {worst_off:.2e}; worst update err {worst_u:.2e} "
          f"({wu}); largest: {[(n, f'{e:.1e}') for n, e in top]}")
    assert worst_off <= OFFSET_GRAD_TOL
    assert worst_l <= LOSS_TOL
    assert abs(float(loss) - float(rloss)) <= LOSS_TOL * abs(float(rloss))
    assert worst_g <= GRAD_TOL, wg
    assert worst_u <= GRAD_TOL, wu


def _rel_l2(a, b, floor):
    """||a - b|| / max(||b||, floor), in f64."""
    a, b = a.double().flatten(), b.double().flatten()
    return float((a - b).norm()) / max(float(b.norm()), floor)


SEEDS_BF16 = ((78, 6, 7), (178, 16, 17), (278, 26, 27))     # (weights, batch, point draws)


def _bf16_step_errors(wseed, bseed, dseed):
    """One seed of test_bf16_training_step_vs_oracle: the per-parameter relative L2 errors
    of the bf16 Trainer step (ours) and of the oracle run in bf16 (yardstick) against the
    fp32 oracle, for the gradients and the weight updates, plus the three losses."""
    from _draws import ForcedDecisions
    from visionseg.criterion import SetCriterion
    from visionseg.data import synthetic_batch
    from visionseg.model import M2FConfig, Mask2Former
    from visionseg.train import SolverConfig, Trainer, lr_at
    cfg = M2FConfig.preset("swin_t")
    rcfg = RefConfig.from_dict(cfg.to_dict())
    ref = RefMask2Former(rcfg)
    sd = det_init({k: v.shape for k, v in ref.state_dict().items()}, wseed)
    sd = {k: (v.to(torch.bfloat16).float() if v.is_floating_point() else v) for k, v in sd.items()}
    ref.load_state_dict(sd)
    ref.train()
    imgs, ml, cl = synthetic_batch(2, 256, seed=bseed)
    imgs = imgs.to(torch.bfloat16).float()
    draws = ForcedDecisions(2, max(len(c) for c in cl) + 1, seed=dseed)
    s = SolverConfig(optimizer="sgd", warmup_iters=0, lr=0.05)
    lr = lr_at(s, 0)

    def oracle_step(model, x, dtype):
        model.decoder.record = dtype == torch.float32
        masks, classes = model(x.to(dtype))
        masks, classes = [m.float() for m in masks], [c.float() for c in classes]
        loss, _ = RefCriterion(rcfg, point_source=draws)(masks, classes, [m.float() for m in ml], cl)
        loss.backward()
        ps = dict(model.named_parameters())
        grads = {n: p.grad.detach().float().clone() for n, p in ps.items()}
        # the reference's solver on an f32 copy (the update of the same weights)
        f32 = {n: torch.nn.Parameter(p.detach().float().clone()) for n, p in ps.items()}
        for n, p in f32.items():
            p.grad = grads[n].clone()
        before = {n: p.detach().clone() for n, p in f32.items()}
        ref_clip_per_parameter(list(f32.values()), s.clip_value)
        groups = ref_param_groups(model, lr, s.weight_decay, "sgd")
        for gr in groups:
            gr["params"] = [f32[gr["name"]]]
        ref_optimizer(groups, "sgd", s.momentum).step()
        upd = {n: f32[n].detach() - before[n] for n in f32}
        return float(loss), grads, upd

    # ---- oracle fp32 (records the decisions), then oracle bf16 (replays them)
    l32, g32, u32 = oracle_step(ref, imgs, torch.float32)
    forced = [rb for rb, _ in ref.decoder.trace]
    draws.replay = True
    ref16 = RefMask2Former(rcfg)
    ref16.load_state_dict(sd)
    ref16 = ref16.to(torch.bfloat16).train()
    ref16.decoder.mask_override = forced
    l16, g16, u16 = oracle_step(ref16, imgs, torch.bfloat16)

    # ---- product: one bf16 Trainer step on the GPU.  MIOpen's convolution solvers fixed
    # (deterministic choice, no Find): with Find the solver of a conv shape is picked by
    # timing, a different one in another process, and the step's bf16 rounding with it
    import dataclasses
    bench_state = (torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic)
    torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = False, True
    try:
        prod = Mask2Former(cfg)
        prod.load_state_dict(sd)
        tr = Trainer(prod, SetCriterion(cfg, matcher="device", point_source=draws),
                     dataclasses.replace(s, conv_find=False), device=DEV)
        assert tr.mode == "bf16"
        prod.decoder.mask_override = forced
        tr._set_lr()
        w0 = {n: m.detach().cpu().clone() for n, m in zip(tr.opt.names, tr.master_params())}
        loss, _ = tr.forward_backward(imgs.to(DEV), [m.to(DEV) for m in ml], [c.to(DEV) for c in cl])
        gp = {n: g.detach().float().cpu().clone() for n, g in zip(tr.opt.names, tr.opt.grad_views)}
        tr.apply_gradients()
        torch.cuda.synchronize()
    finally:
        torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = bench_state
    up = {n: m.detach().cpu() - w0[n] for n, m in zip(tr.opt.names, tr.master_params())}
    assert set(gp) == set(g32)
    names = sorted(g32)
    gfloor = 1e-2 * float(np.median([float(g32[n].norm()) for n in names]))
    ufloor = 1e-3 * float(np.median([float(u32[n].norm()) for n in names]))
    return dict(
        loss=(float(loss), l16, l32),
        eg={n: _rel_l2(gp[n], g32[n], gfloor) for n in names}, yg={n: _rel_l2(g16[n], g32[n], gfloor) for n in names},
        eu={n: _rel_l2(up[n], u32[n], ufloor) for n in names}, yu={n: _rel_l2(u16[n], u32[n], ufloor) for n in names},
        dist={n: float((gp[n].double() - g32[n].double()).norm()) / (gfloor / 1e-2) for n in names},
        ydist={n: float((g16[n].double() - g32[n].double()).norm()) / (gfloor / 1e-2) for n in names})


def _family(name):
    """decoder.layers.6.fc2.weight -> decoder.layers.*.fc2.weight"""
    return ".".join("*" if p.isdigit() else p for p in name.split("."))


def test_bf16_training_step_vs_oracle():
    """The PRODUCTION training step (bf16 Trainer: MFMA window attention fwd/bwd, the
    MFMA MSDA backward with grad_loc / grad_attn in its band walk, MFMA masked attention,
    the fused mask-head backward through the point-scatter kernel, the decoder Linears on
    csrc/small_linear.hip, bf16 GEMMs, the flat-buffer optimiser) vs the oracle
    (RefMask2Former + RefCriterion + the reference's solver, fp32 on CPU), Swin-T at
    256^2, on the same bf16-rounded weights and input and the same point draws
    (HF:m2f:726-779 losses, train_full.py:266-271 clip), for THREE weight / batch / draw
    seeds (SEEDS_BF16): one draw is one rounding realisation, so the gates are on the mean
    over seeds of the per-seed ratio to the yardstick.

    Decisions are forced from the fp32 oracle into the other runs: the decoder's attention
    masks (mask_override), the Hungarian matching of every decoder step and the
    importance-sampling top-k choice (tests/_draws.ForcedDecisions).

    Yardstick: the oracle ITSELF run in bf16 (torch CPU bf16 kernels, same weights,
    forced decisions).  Per parameter, the error is the relative L2 distance to the fp32
    oracle's gradient (norm floor 1e-2 of the median parameter gradient norm: gradients
    that are analytically ~0, e.g. the key bias of a softmax attention, are rounding
    noise on every path).  Bounds:
      * loss, per seed: |ours - fp32| <= 1.25 x |oracle-bf16 - fp32| + 2e-3 x loss;
      * gradients: mean over seeds of (median over parameters of ours / the yardstick's)
        <= 1.25, and the same for the 90th percentile;
      * weight updates of the step (per-parameter clip to norm 0.01, SGD): the same two
        bounds against the yardstick's update;
      * defects: no parameter whose error is above both 3 x its yardstick's and 2.5 x the
        yardstick's p90 (relative) and 5 % of the median gradient norm (absolute) on
        2 of the 3 seeds, and none above 10 x / 5 x p90 / 20 % on any one seed.
    The per-family mean ratios are printed (largest first) for a diagnosis."""
    runs = [_bf16_step_errors(*sd) for sd in SEEDS_BF16]
    q = lambda d, p: float(np.percentile(list(d.values()), p))          # noqa: E731
    rg50 = [q(r["eg"], 50) / q(r["yg"], 50) for r in runs]
    rg90 = [q(r["eg"], 90) / q(r["yg"], 90) for r in runs]
    ru50 = [q(r["eu"], 50) / q(r["yu"], 50) for r in runs]
    ru90 = [q(r["eu"], 90) / q(r["yu"], 90) for r in runs]
    names = sorted(runs[0]["eg"])
    fam = {}
    for n in names:
        fam.setdefault(_family(n), []).append(n)
    fam_ratio = {f: float(np.mean([np.mean([r["eg"][n] for n in ns]) / max(np.mean([r["yg"][n] for n in ns]), 1e-12)
                                   for r in runs])) for f, ns in fam.items()}
    top = sorted(fam_ratio.items(), key=lambda kv: -kv[1])[:8]
    for i, r in enumerate(runs):
        lp, l16, l32 = r["loss"]
        print(f"bf16 step seed {SEEDS_BF16[i]}: loss ours {lp:.5f} / oracle-bf16 {l16:.5f} / fp32 {l32:.5f}; grad "
              f"rel-L2 median {q(r['eg'], 50):.2e} (yard {q(r['yg'], 50):.2e}), p90 {q(r['eg'], 90):.2e} (yard "
              f"{q(r['yg'], 90):.2e}); update median {q(r['eu'], 50):.2e} (yard {q(r['yu'], 50):.2e}), p90 "
              f"{q(r['eu'], 90):.2e} (yard {q(r['yu'], 90):.2e})")
    print(f"bf16 step mean ratios over seeds: grad p50 {np.mean(rg50):.3f} p90 {np.mean(rg90):.3f}, update p50 "
          f"{np.mean(ru50):.3f} p90 {np.mean(ru90):.3f}; per-seed grad p90 {[round(v, 3) for v in rg90]}; "
          f"families (mean ratio to yardstick): {[(f, round(v, 2)) for f, v in top]}")
    if os.environ.get("VS_PARITY_DUMP"):                 # per-parameter errors for a diagnosis
        with open(os.environ["VS_PARITY_DUMP"], "w") as f:
            json.dump([{k: r[k] for k in ("eg", "yg", "eu", "yu", "loss")} for r in runs], f)
    for r in runs:
        lp, l16, l32 = r["loss"]
        assert abs(lp - l32) <= 1.25 * abs(l16 - l32) + 2e-3 * abs(l32), r["loss"]
    assert np.mean(rg50) <= 1.25 and np.mean(rg90) <= 1.25, (rg50, rg90)
    assert np.mean(ru50) <= 1.25 and np.mean(ru90) <= 1.25, (ru50, ru90)
    # a defect on 2 of the 3 seeds (a data-dependent kernel bug -- a tie, an edge shape --
    # need not show on every draw), or a gross one (10x the yardstick, 20 % of the median
    # gradient norm) on any single seed
    bad = [n for n in names if sum(
        r["eg"][n] > max(3.0 * r["yg"][n], 2.5 * q(r["yg"], 90)) and r["dist"][n] > 0.05 for r in runs) >= 2
        or any(r["eg"][n] > max(10.0 * r["yg"][n], 5.0 * q(r["yg"], 90)) and r["dist"][n] > 0.2 for r in runs)]
    assert not bad, [(n, [round(r["eg"][n], 3) for r in runs], [round(r["yg"][n], 3) for r in runs]) for n in bad[:5]]
