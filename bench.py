"""Training-throughput benchmark of the MI355X Swin + Mask2Former path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model swin_t] [--batch 4] [--size 1024]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Metric (BASELINE.json): images/sec at 1024^2, Swin-T Mask2Former, 1/2/4/8 GPUs.  A step
is one full training iteration (bf16 forward with bf16 parameters and f32 master weights,
set criterion with device Hungarian matching, backward, bucketed f32 RCCL gradient
all-reduce overlapped with backward when N>1, per-parameter grad clip, SGD momentum --
the reference's detectron2 solver)
on a synthetic COCO-format defect batch of `--batch` images per GPU, resident in HBM
before the timed region.  Weak scaling: per-GPU batch fixed.  Rank 0 prints ONE JSON
line; `roofline` covers the dominant hand-written kernel (`roofline_second` the next one) (HIP events on its launch
stream, algorithmic bytes/flops per launch), `step_roofline` the whole step against the
bf16 MFMA peak (algorithmic training FLOPs per image); `cpu_baseline`
times the oracle CPU restatement (fp32) on the host cores on a bounded sample
(BASELINE.md §3); `parity` is the mask-logit error vs the oracle in fp32 kernel mode and
on the production bf16 path.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# before HIP initialises (see visionseg/__init__.py)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "vision-instance-seg_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

# Vendor-GEMM solution table (PyTorch TunableOp over hipBLASLt/rocBLAS, incl. split-K for
# the tall-K weight-gradient GEMMs), tuned on MI355X for the bench configs and shipped
# in-tree: loaded read-only in main() (visionseg.linear.load_gemm_table).  --gemm-tuning
# tune re-tunes instead; that mode's environment must be set before torch loads.
_gt = "file"
for _i, _a in enumerate(sys.argv):
    if _a == "--gemm-tuning" and _i + 1 < len(sys.argv):
        _gt = sys.argv[_i + 1]
    elif _a.startswith("--gemm-tuning="):
        _gt = _a.split("=", 1)[1]
if _gt == "tune":
    os.environ.setdefault("PYTORCH_TUNABLEOP_ENABLED", "1")
    os.environ.setdefault("PYTORCH_TUNABLEOP_TUNING", "1")
    os.environ.setdefault("PYTORCH_TUNABLEOP_FILENAME", os.path.join(ROOT, "gpurun_out", "tunableop_results%d.csv"))
    os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS", "20")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

MODEL_NAMES = {"swin_t": "Swin-T", "swin_s": "Swin-S", "swin_b": "Swin-B", "swin_l": "Swin-L"}
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
MFMA_BF16_PEAK_TFS = 2500.0  # dense bf16 MFMA spec
VALU_F32_PEAK_TFS = 157.3    # f32 vector / f32 MFMA spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="swin_t")
    ap.add_argument("--batch", type=int, default=4, help="images per GPU")
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--queries", type=int, default=100)
    ap.add_argument("--matcher", default="device", choices=["device", "host"],
                    help="Hungarian matching on the device (csrc/match.hip) or scipy on the host")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-iters", type=int, default=3)
    ap.add_argument("--kernel-timing", type=int, default=1,
                    help="HIP-event per-kernel timing (graphs: over --timing-steps eager steps after the timed region)")
    ap.add_argument("--graphs", type=int, default=1, help="replay the step as HIP graphs (Trainer(graphs=True))")
    ap.add_argument("--timing-steps", type=int, default=2, help="eager steps for per-kernel timing in graph mode")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "amp"],
                    help="bf16: bf16 params/activations + f32 master weights; amp: f32 params + bf16 autocast")
    ap.add_argument("--optimizer", default="sgd", choices=["sgd", "adamw"],
                    help="sgd: the reference's detectron2 DefaultTrainer solver; adamw: upstream train_net")
    ap.add_argument("--attn-fp8", action="store_true",
                    help="C5: Swin window attention on fp8 (e4m3) MFMA (window^2 <= 160; bf16 elsewhere)")
    ap.add_argument("--linear-fp8", action="store_true",
                    help="C5: the Swin blocks' K-deep Linears on the block-scaled MX fp8 MFMA (csrc/token_gemm.hip)")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--arch", default="mask2former", choices=["mask2former", "maskdino"],
                    help="mask2former (C1-C3, C5) or maskdino (C4: 300 queries, 4-level encoder, DN; parity unpinned)")
    ap.add_argument("--gemm-tuning", default="file", choices=["file", "tune", "off"],
                    help="vendor GEMM solution table: in-tree TunableOp file (default), re-tune, or heuristics")
    return ap.parse_args()


# HBM traffic per op launch from rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; KiB,
# FETCH x2 on gfx950 -- tools/pmc_traffic.py), committed under profiles/ PER CONFIG
# (profiles/pmc_traffic_<model>_<size>.json); the kernels each timed op dispatches once
# per launch.  No file for the config -> traffic null.
PMC_DIR = os.path.join(ROOT, "profiles")


def pmc_file(model, size):
    return os.path.join(PMC_DIR, f"pmc_traffic_{model}_{size}.json")


OP_KERNELS = {   # op -> kernel-name substrings (template arguments included) whose dispatches make one launch
    # the pyramid-column kernel (default for encoder problems) or the 8 x 8 tile kernel
    "msda_bwd": ["msda_bwd_col_kernel<", "msda_bwd_mfma_wg_kernel<8, 8, true"],
    "msda_fwd": ["msda_fwd_kernel<"],
    "window_attn_fwd": ["win_attn_fwd_mfma(", "win_attn_fwd_mfma_big<3, false>", "win_attn_fwd_mfma_big<4, false>",
                        "win_attn_fwd_mfma_big<5, false>"],
    "window_attn_bwd": ["win_attn_bwd_fa<2, false>", "win_attn_bwd_fa<3, false>", "win_attn_bwd_fa<4, false>",
                        "win_attn_bwd_fa<5, false>"],
    "window_attn_fwd_fp8": [f"win_attn_fwd_mfma_big<{n}, true>" for n in (2, 3, 4, 5)],
    "window_attn_bwd_fp8": [f"win_attn_bwd_fa<{n}, true>" for n in (2, 3, 4, 5)],
    "mask_head_fwd": ["mask_head_fwd_bf16_kernel<"],
    "mask_head_bwd": ["mask_head_bwd_kernel<"],
    # one token_wgrad call = the weight-gradient kernel + (when split) its reduction
    "token_wgrad": ["token_wgrad_kernel<", "token_wgrad_reduce_kernel<"],
    # one bf16 token GEMM call = one tile-kernel or one streaming-kernel dispatch
    "token_gemm": ["token_gemm_kernel<false", "token_gemm_stream_kernel<"],
}
# ops whose one launch dispatches one kernel of EACH pattern (traffic summed over the
# patterns, per dispatch of the first) instead of one kernel of any of them
OP_MULTI = {"token_wgrad"}


def pmc_traffic(op, path):
    """(bytes per launch, kernels counted) of `op` from the committed PMC profile, or None:
    the mean per-dispatch bytes (FETCH + WRITE) of the kernels matching the op's patterns
    (one launch of the op = one dispatch of one of them)."""
    if op not in OP_KERNELS or not os.path.exists(path):
        return None, None
    rows = json.load(open(path))
    hits = [(k, v) for k, v in rows.items() if any(p in k for p in OP_KERNELS[op])]
    if not hits:
        return None, None
    if op in OP_MULTI:
        first = [v for k, v in hits if OP_KERNELS[op][0] in k]
        n = sum(v["dispatches"] for v in first)
    else:
        n = sum(v["dispatches"] for _, v in hits)
    tot = sum((v["fetch_bytes"] + v["write_bytes"]) * v["dispatches"] for _, v in hits) / max(1, n)
    return int(tot), sorted({p for p in OP_KERNELS[op] for k, _ in hits if p in k})


def kernel_roofline(summary, pmc_path, rank=0):
    """Pick the hand-written kernel with the largest total time (rank 1: the second largest)
    and price it against the roofline of its regime: HBM bytes for gather/copy kernels and
    for any kernel whose algorithmic intensity (FLOP per algorithmic byte) sits below the
    ridge point MFMA peak / HBM peak (312.5 FLOP/B for bf16), matrix FLOP/s otherwise.  The
    other ceiling's fraction is reported beside it (`frac_other`)."""
    if not summary or len(summary) <= rank:
        return None, {}
    name = sorted(summary, key=lambda k: -summary[k]["total_ms"])[rank]
    s = summary[name]
    t = s["mean_ms"] / 1e3
    hbm_kernels = {"msda_fwd", "msda_bwd", "window_partition", "window_reverse", "attn_bitmask", "mask_head_fwd"}
    ridge = MFMA_BF16_PEAK_TFS * 1e12 / (HBM_PEAK_GBS * 1e9)
    intensity = s["flops"] / s["bytes"] if s["bytes"] and s["flops"] else None
    if name in hbm_kernels or (intensity is not None and intensity < ridge):
        ach = s["bytes"] / t / 1e9
        traffic, kernels = pmc_traffic(name, pmc_path)
        roof = dict(bound="hbm", achieved=round(ach, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(ach / HBM_PEAK_GBS, 4), traffic=traffic, kernel=name,
                    intensity_flop_per_byte=round(intensity, 1) if intensity else None, ridge=ridge,
                    frac_other=dict(bound="mfma", achieved=round(s["flops"] / t / 1e12, 2),
                                    frac=round(s["flops"] / t / 1e12 / MFMA_BF16_PEAK_TFS, 5)) if s["flops"] else None,
                    traffic_source=(f"profiles/{os.path.basename(pmc_path)}: rocprofv3 --pmc FETCH_SIZE (x2, gfx950) "
                                    f"+ WRITE_SIZE per launch of {kernels}") if traffic else None,
                    algorithmic_bytes_per_launch=int(s["bytes"]), mean_launch_ms=round(s["mean_ms"], 4),
                    launches=s["launches"])
    else:
        ach = s["flops"] / t / 1e12
        traffic, kernels = pmc_traffic(name, pmc_path)
        roof = dict(bound="mfma", achieved=round(ach, 2), peak=MFMA_BF16_PEAK_TFS, unit="TFLOP/s",
                    frac=round(ach / MFMA_BF16_PEAK_TFS, 5), traffic=traffic, kernel=name,
                    intensity_flop_per_byte=round(intensity, 1) if intensity else None, ridge=ridge,
                    traffic_source=(f"profiles/{os.path.basename(pmc_path)}: rocprofv3 --pmc FETCH_SIZE (x2, gfx950) "
                                    f"+ WRITE_SIZE per launch of {kernels}") if traffic else None,
                    algorithmic_flops_per_launch=int(s["flops"]), mean_launch_ms=round(s["mean_ms"], 4),
                    launches=s["launches"])
    table = {k: dict(launches=v["launches"], total_ms=round(v["total_ms"], 3), mean_ms=round(v["mean_ms"], 4),
                     gbs=round(v["bytes"] / (v["mean_ms"] / 1e3) / 1e9, 1) if v["bytes"] else None,
                     tflops=round(v["flops"] / (v["mean_ms"] / 1e3) / 1e12, 2) if v["flops"] else None)
             for k, v in summary.items()}
    return roof, table


def _cpu_model_name():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(model_name, size, iters, queries):
    """the oracle CPU restatement (fp32) on this host's cores, median of
    `iters`, images/s, for (a) C1 = 2x512^2 forward+loss (after one warm-up) and (b) one
    `size`^2 image forward+loss+backward (the like-for-like training sample; its rate is
    `value`), about 30-40 s of CPU work in all.  Threads = the CPUs this process may run on
    (the box's CPU share), reported with os.cpu_count() and the CPU model."""
    from oracle.ref_model import RefConfig, RefMask2Former, RefCriterion
    from visionseg.model import M2FConfig
    from visionseg.data import synthetic_batch
    # the CPUs this process may use: the box's CPU share (OMP_NUM_THREADS, set there)
    # when given, else the affinity set (os.cpu_count() reports the whole machine)
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    threads = min(aff, int(os.environ.get("OMP_NUM_THREADS", aff)))
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    cfg = RefConfig.from_dict(M2FConfig.preset(model_name, num_queries=queries).to_dict())
    torch.manual_seed(0)
    m = RefMask2Former(cfg)
    crit = RefCriterion(cfg)

    def run(batch, sz, backward, warm):
        imgs, ml, cl = synthetic_batch(batch, sz, seed=42)
        ml = [x.float() for x in ml]
        ts = []
        for i in range(iters + warm):
            print(f"cpu baseline: {batch}x{sz}^2 {'fwd+loss+bwd' if backward else 'fwd+loss'} iter {i + 1}/"
                  f"{iters + warm}", file=sys.stderr, flush=True)
            t0 = time.perf_counter()
            if backward:
                masks, classes = m(imgs)
                loss, _ = crit(masks, classes, ml, cl)
                loss.backward()
                m.zero_grad(set_to_none=True)
            else:
                with torch.no_grad():
                    masks, classes = m(imgs)
                    crit(masks, classes, ml, cl)
            if i >= warm:
                ts.append(time.perf_counter() - t0)
        ts.sort()
        med = ts[len(ts) // 2]
        return batch / med, med

    c1, c1_t = run(2, 512, False, 1)
    v, t = run(1, size, True, 0)            # warmed up by the C1 runs (same model)
    torch.set_num_threads(prev)
    return dict(value=round(v, 4), unit="images/s", cores=threads, kind="port",
                sample=f"1x3x{size}^2 {model_name} Mask2Former fp32 forward+loss+backward (oracle CPU restatement), "
                       f"median of {iters} iters (after the C1 runs on the same model), {t:.2f} s/iter",
                c1_forward_loss=dict(value=round(c1, 4), unit="images/s",
                                     sample=f"C1: 2x3x512^2 forward+loss, median of {iters} after 1 warm-up, "
                                            f"{c1_t:.2f} s/iter"),
                host=dict(cpu_model=_cpu_model_name(), os_cpu_count=os.cpu_count(), threads_used=threads))


def _bf16_round_(model):
    with torch.no_grad():
        for p in model.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    return model


def parity_check(model_name, size, queries, dev):
    """BASELINE metric, second half: mask-logit max-abs-err vs the oracle CPU restatement
    on one `size`^2 image, every decoder step, weights = init_weights + perturbed
    tables/offsets (every path carries signal) rounded to bf16 so ONE oracle forward
    serves both checks:
      fp32: the GPU path in fp32 kernel mode, free-running (the decoder's attention masks
            are threshold decisions; the mask bits that differ from the oracle's, all at
            near-zero logits (tests/test_gpu_model.py), are counted);
      bf16: the production path (bf16 parameters and activations, MFMA window and masked
            attention, bf16 mask head) with the oracle's attention masks forced in (a
            near-zero logit flips freely in bf16), error absolute and relative to the
            step's max |logit|."""
    from oracle.ref_model import RefConfig, RefMask2Former
    from visionseg.model import M2FConfig, Mask2Former, unpack_bitmask_like
    cfg = M2FConfig.preset(model_name, num_queries=queries)
    m = Mask2Former(cfg).init_weights(0)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "rel_table" in n or "attention_weights" in n or "level_embed" in n:
                p.add_(0.3 * torch.randn(p.shape, generator=g))
    _bf16_round_(m)
    ref = RefMask2Former(RefConfig.from_dict(cfg.to_dict()))
    ref.load_state_dict({k: v.clone() for k, v in m.state_dict().items()})
    m = m.to(dev).eval()
    ref.eval()
    px = torch.randn(1, 3, size, size, generator=torch.Generator().manual_seed(5)).to(torch.bfloat16).float()
    with torch.no_grad():
        ref.decoder.record = True
        t0 = time.perf_counter()
        rmasks, _ = ref(px)
        t_ref = time.perf_counter() - t0
        m.decoder.record = True
        masks, _ = m(px.to(dev))
        err = max(float((a.cpu() - b).abs().max()) for a, b in zip(masks, rmasks))
        flips = sum(int((unpack_bitmask_like(w, rb.shape[-1]).cpu() != rb).sum())
                    for (rb, _), w in zip(ref.decoder.trace, m.decoder.trace))
        del masks
        m = m.to(torch.bfloat16)
        m.decoder.record = False
        m.decoder.mask_override = [rb for rb, _ in ref.decoder.trace]
        bmasks, _ = m(px.to(dev).to(torch.bfloat16))
        abs_err = [float((a.float().cpu() - b).abs().max()) for a, b in zip(bmasks, rmasks)]
        rel_err = [e / float(b.abs().max()) for e, b in zip(abs_err, rmasks)]
        mean_err = max(float((a.float().cpu() - b).abs().mean()) for a, b in zip(bmasks, rmasks))
        scale = max(float(b.abs().max()) for b in rmasks)
    del m, ref, bmasks
    torch.cuda.empty_cache()
    return dict(mask_logit_max_abs_err=float(f"{err:.3e}"), tolerance=1e-3, attention_mask_bit_flips=flips,
                bf16=dict(mask_logit_max_abs_err=float(f"{max(abs_err):.3e}"),
                          max_rel_to_logit_scale=float(f"{max(rel_err):.3e}"),
                          mean_abs_err=float(f"{mean_err:.3e}"), logit_scale=float(f"{scale:.3e}"),
                          tolerance="max abs err <= 0.02 x max|logit| of the step (bf16 activations, "
                                    "tests/test_gpu_model.py)", forced_attention_masks=True),
                oracle_forward_s=round(t_ref, 2),
                sample=f"1x3x{size}^2 {model_name} Mask2Former, {queries} queries, bf16-rounded weights and input, "
                       f"vs the oracle CPU restatement (fp32), all {cfg.dec_layers} decoder steps")


# Algorithmic training FLOPs per image (forward matmul/conv FLOPs x 3) for the BASELINE
# configs: Mask2Former forward counted with torch.utils.flop_counter on the HF oracle
# (BASELINE.md §2); MaskDINO (C4, no HF model exists) counted by the same method on the
# product's own training forward, denoising queries included, with the custom ops priced
# as the matmuls they replace (tools/flops.py --arch maskdino --model swin_l, measured on
# the box: 2198.3 GFLOP; profiles/r3_flops_c4.json)
TRAIN_FLOPS_PER_IMAGE = {("mask2former", "swin_t", 1024): 3 * 530.6e9,
                         ("mask2former", "swin_b", 1024): 3 * 1022.2e9,
                         ("mask2former", "swin_l", 1536): 3 * 3974.2e9,
                         ("maskdino", "swin_l", 1024): 3 * 2198.3e9}


def _config_tag(model, size, arch="mask2former", fp8=False):
    """BASELINE.json config the run corresponds to (C2 is the headline workload)."""
    if arch == "maskdino":
        return "C4 (per-GPU share)" if (model, size) == ("swin_l", 1024) else "custom"
    if (model, size) == ("swin_l", 1536):
        return "C5 (per-GPU share, fp8)" if fp8 else "C5 shape (per-GPU share, bf16)"
    return {("swin_t", 1024): "C2", ("swin_b", 1024): "C3 (per-GPU share)"}.get((model, size), "custom")


def main():
    a = parse()
    from visionseg.train import init_distributed, Trainer, SolverConfig
    from visionseg.model import M2FConfig, Mask2Former
    from visionseg.criterion import SetCriterion
    from visionseg.data import synthetic_batch
    from visionseg.profiling import KernelTimer

    rank, local, world = init_distributed()
    if world != a.gpus and rank == 0:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if a.gemm_tuning == "file":
        from visionseg.linear import load_gemm_table
        if not load_gemm_table():
            a.gemm_tuning = "file (not loaded)"
    if a.arch == "maskdino":
        from visionseg.maskdino import MaskDINO, MaskDINOConfig, MaskDINOCriterion
        if a.queries == 100:
            a.queries = 300
        cfg = MaskDINOConfig.preset(a.model, num_queries=a.queries)
        model = MaskDINO(cfg).init_weights(seed=0)
        crit = MaskDINOCriterion(cfg, matcher=a.matcher)
    else:
        cfg = M2FConfig.preset(a.model, num_queries=a.queries, attn_fp8=a.attn_fp8, linear_fp8=a.linear_fp8)
        model = Mask2Former(cfg).init_weights(seed=0)
        crit = SetCriterion(cfg, matcher=a.matcher)
    trainer = Trainer(model, crit, SolverConfig(precision=a.precision, optimizer=a.optimizer), device=dev,
                      graphs=bool(a.graphs))
    graphs = trainer.graphs
    images, ml, cl = synthetic_batch(a.batch, a.size, seed=42 + rank, device=dev)
    torch.cuda.synchronize()

    if graphs:    # the eager warm-ups of the trainer and the capture stay out of the timed region
        a.warmup = max(a.warmup, trainer.graph_warmup + 1)
    for _ in range(a.warmup):
        trainer.step(images, ml, cl)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    timer = KernelTimer() if a.kernel_timing else None
    if timer and not graphs:
        timer.__enter__()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = trainer.step(images, ml, cl)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if timer and graphs:
        # a graph replay carries no event timestamps: time the kernels over eager steps
        # of the same workload right after the timed region (outside it)
        timer.__enter__()
        for _ in range(max(1, a.timing_steps)):
            trainer.eager_step(images, ml, cl)
        torch.cuda.synchronize()
    if timer:
        timer.__exit__(None, None, None)
    t = torch.tensor([elapsed], device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms = elapsed / a.steps * 1e3
    value = a.batch * world * a.steps / elapsed
    if rank == 0:
        roof, table = kernel_roofline(timer.summary(), pmc_file(a.model, a.size)) if timer else (None, {})
        roof2, _ = kernel_roofline(timer.summary(), pmc_file(a.model, a.size), rank=1) if timer else (None, {})
        cpu, parity = None, None
        if a.arch == "maskdino":
            parity = {"unpinned": "no MaskDINO implementation exists in the container (SURVEY §8c); "
                                  "structural GPU tests only (tests/test_gpu_maskdino.py)"}
        if world == 1 and not a.no_cpu_baseline and a.arch == "mask2former":
            cpu = cpu_baseline(a.model, a.size, a.cpu_iters, a.queries)
        if world == 1 and not a.no_parity and a.arch == "mask2former":
            print("parity check vs the oracle ...", file=sys.stderr, flush=True)
            parity = parity_check(a.model, a.size, a.queries, dev)
        fl = TRAIN_FLOPS_PER_IMAGE.get((a.arch, a.model, a.size))
        step_roof = None
        if fl:
            ach = fl * value / 1e12
            step_roof = dict(bound="mfma", achieved=round(ach, 1), peak=MFMA_BF16_PEAK_TFS * world, unit="TFLOP/s",
                             frac=round(ach / (MFMA_BF16_PEAK_TFS * world), 4),
                             algorithmic_flops_per_image=fl,
                             note="whole training step: 3 x forward matmul/conv FLOPs (BASELINE.md §2; C4: tools/flops.py) x images/s "
                                  "/ (dense bf16 MFMA peak x GPUs)")
        prec = ("bf16 parameters and activations, f32 master weights, gradients reduced and applied in f32 "
                "(pure bf16, not autocast)" if a.precision == "bf16" else "f32 parameters + bf16 autocast")
        line = {
            "metric": f"images/sec @{a.size}^2 {MODEL_NAMES.get(a.model, a.model)} "
                      f"{'MaskDINO' if a.arch == 'maskdino' else 'Mask2Former'} training "
                      f"(fwd+loss+bwd+{a.optimizer.upper()})",
            "value": round(value, 3), "unit": "images/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms, 2), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16", "data": "synthetic COCO-format defect batches (random-init weights)",
            "config": {"workload": f"{_config_tag(a.model, a.size, a.arch, a.attn_fp8 or a.linear_fp8)}: {a.model} + {a.arch}, "
                                   f"{a.batch}x3x{a.size}^2 per GPU, {cfg.num_queries} queries, {prec}"
                                   f"{', fp8 (e4m3) window attention' if a.attn_fp8 else ''}"
                                   f"{', MX-fp8 (e4m3 + e8m0 per 32) Swin Linears with K >= 384' if a.linear_fp8 else ''}, 1 class",
                       "model": f"{a.model}_{a.arch}", "global_batch": a.batch * world, "image_size": a.size,
                       "parallelism": f"dp{world}"},
            "final_loss": round(float(loss.item()), 4),
            "gemm_tuning": a.gemm_tuning,
            "precision": a.precision,
            "optimizer": a.optimizer,
            "matcher": a.matcher,
            "graphs": graphs,
            "kernel_timing": ("HIP events over %d eager steps after the timed region" % max(1, a.timing_steps))
            if graphs else "HIP events over the timed region",
            "roofline": roof,
            "roofline_second": roof2,
            "step_roofline": step_roof,
            "cpu_baseline": cpu,
            "parity": parity,
            "kernels": table,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
