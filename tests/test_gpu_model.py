"""End-to-end parity of the MI355X model against the oracle (BASELINE metric:
mask-logit max-abs-err <= 1e-3 in fp32 kernel mode) and a bf16 training step."""
import json
import time

import numpy as np
import pytest
import torch

from oracle.detinit import det_init
from oracle.ref_model import RefConfig, RefMask2Former

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _product(cfg_dict, sd):
    from visionseg.model import M2FConfig, Mask2Former
    m = Mask2Former(M2FConfig.from_dict(cfg_dict))
    m.load_state_dict(sd)
    return m.to(DEV).eval()


@pytest.mark.parametrize("tag", ["a", "b"])
def test_tiny_model_vs_hf_golden(golden, tag):
    """fp32 kernels vs the HF-generated fixture (weights regenerated from the seed)."""
    d = golden("model_tiny.npz")
    cfg = json.loads(str(d["config"]))
    ref = RefMask2Former(RefConfig.from_dict(cfg))
    sd = det_init({k: v.shape for k, v in ref.state_dict().items()}, int(d["weight_seed"]))
    m = _product(cfg, sd)
    px = torch.from_numpy(d[f"{tag}_pixel_values"]).to(DEV)
    with torch.no_grad():
        masks, classes = m(px)
    got = torch.stack(masks).cpu().numpy()
    exp = d[f"{tag}_masks"]
    err = np.abs(got - exp).max()
    print(f"tiny[{tag}] mask-logit max|err| vs HF = {err:.3e}")
    assert err <= 1e-3
    np.testing.assert_allclose(torch.stack(classes).cpu().numpy(), d[f"{tag}_classes"], atol=1e-3, rtol=0)


def _swin_t_pair(size, queries=100, seed=0, preset="swin_t"):
    from visionseg.model import M2FConfig, Mask2Former
    cfg = M2FConfig.preset(preset, num_queries=queries)
    m = Mask2Former(cfg).init_weights(seed)
    # perturb the zero-initialised tables/offsets so every path carries signal
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "rel_table" in n or "attention_weights" in n or "level_embed" in n:
                p.add_(0.3 * torch.randn(p.shape, generator=g))
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    ref = RefMask2Former(RefConfig.from_dict(cfg.to_dict()))
    ref.load_state_dict(sd)
    return m.to(DEV).eval(), ref.eval(), cfg


@pytest.mark.parametrize("size", [256, 1024])
def test_swin_t_mask_logits_vs_oracle(size):
    """BASELINE metric: mask logits of the GPU path vs the CPU oracle, same weights and
    input, fp32 kernel mode, bound 1e-3 abs; 1024^2 is the C2 shape.

    The decoder's attention masks are threshold decisions (sigmoid(x) < 0.5, HF:m2f:2053):
    where an interpolated logit is within fp32 rounding of 0, the GPU and the CPU oracle
    (whose own rounding varies with its thread count) may decide differently, and the
    self-attention then carries that difference to every query of the image.  The test
    therefore checks (a) every differing mask bit sits at |oracle logit| < 1e-4, and (b)
    with the oracle's masks forced into the GPU decoder, all logits agree within 1e-3.
    It reports the free-running error too."""
    from visionseg.model import unpack_bitmask_like
    m, ref, cfg = _swin_t_pair(size)
    g = torch.Generator().manual_seed(5)
    px = torch.randn(1, 3, size, size, generator=g)
    with torch.no_grad():
        t0 = time.time()
        ref.decoder.record = True
        rmasks, rclasses = ref(px)
        tcpu = time.time() - t0
        m.decoder.record = True
        masks, classes = m(px.to(DEV))
        free = [float((a.cpu() - b).abs().max()) for a, b in zip(masks, rmasks)]
        flips, worst = 0, 0.0
        for (rb, ram), words in zip(ref.decoder.trace, m.decoder.trace):
            got = unpack_bitmask_like(words, rb.shape[-1]).cpu()
            diff = got != rb
            flips += int(diff.sum())
            if diff.any() and worst == 0.0:
                worst = float(ram[diff].abs().max())
        # a flip is a threshold decision on a logit within rounding of 0 (the oracle's own
        # rounding varies with the CPU thread count of the box): |logit| < 5e-4 against
        # logits of magnitude ~10 (measured flips: 1e-6 .. 1.1e-4).  Checked in the FIRST
        # decoder step that has any: once a bit differs, the self-attention carries the
        # difference into every later step's logits, whose flips then sit further from 0
        # (a 3.7e-3 flip seen downstream of a 1e-5 one; the GPU side's last bits vary from
        # run to run -- 0 or 5 flips over three runs of this test)
        assert worst < 5e-4, f"first mask-bit flip where the oracle logit is {worst:.2e} from the threshold"
        m.decoder.mask_override = [rb for rb, _ in ref.decoder.trace]
        fmasks, fclasses = m(px.to(DEV))
        m.decoder.mask_override = None
    forced = [float((a.cpu() - b).abs().max()) for a, b in zip(fmasks, rmasks)]
    print(f"swin_t@{size}: mask-logit max|err| free-running {max(free):.2e} ({flips} threshold flips, "
          f"max |logit| at a flip {worst:.1e}); forced-mask {max(forced):.2e}; oracle {tcpu:.1f}s")
    assert max(forced) <= 1e-3, forced
    cerr = max(float((a.cpu() - b).abs().max()) for a, b in zip(fclasses, rclasses))
    assert cerr <= 1e-3
    if flips == 0:
        assert max(free) <= 1e-3


def _rel_errors(got, exp):
    """(max over decoder steps of max|err| / max|exp|, same with mean|err|)."""
    wmax, wmean = 0.0, 0.0
    for a, b in zip(got, exp):
        d = (a.float().cpu() - b).abs()
        sc = float(b.abs().max())
        wmax = max(wmax, float(d.max()) / sc)
        wmean = max(wmean, float(d.mean()) / sc)
    return wmax, wmean


@pytest.mark.parametrize("size", [256, 1024])
def test_swin_t_bf16_production_path_vs_oracle(size):
    """The PRODUCTION path (bf16 parameters and activations: MFMA window attention, MFMA
    masked attention, bf16 mask head, bf16 GEMMs) vs the fp32 oracle on the same
    bf16-rounded weights and input; 1024^2 is the benchmarked C2 shape.  The oracle's
    attention-mask decisions are forced into both (a logit near 0 flips freely at bf16
    resolution).

    Tolerance: bf16 storage of every activation through ~70 layers has no analytic bound,
    so the yardstick is the oracle ITSELF run in bf16 (same weights, torch CPU bf16
    kernels): the production path must be as close to the fp32 oracle as that, within a
    factor 1.25, in max and in mean error per decoder step (relative to the step's max
    |logit|), and within the absolute caps max 0.03 / mean 0.004 (measured round 2:
    ours 0.015 / 0.0024 at 256^2, 0.016 / 0.0022 at 1024^2; oracle-in-bf16 0.016 / 0.0025
    and 0.027 / 0.0030 on the build container's CPU)."""
    import copy
    m, ref, cfg = _swin_t_pair(size)
    with torch.no_grad():
        for p in list(m.parameters()) + list(ref.parameters()):
            p.copy_(p.to(torch.bfloat16).float())
    g = torch.Generator().manual_seed(5)
    px = torch.randn(1, 3, size, size, generator=g).to(torch.bfloat16).float()
    with torch.no_grad():
        ref.decoder.record = True
        rmasks, rclasses = ref(px)
        forced = [rb for rb, _ in ref.decoder.trace]
        ref16 = copy.deepcopy(ref).to(torch.bfloat16)
        ref16.decoder.record = False
        ref16.decoder.mask_override = forced
        t0 = time.time()
        omasks, _ = ref16(px.to(torch.bfloat16))
        t16 = time.time() - t0
        m = m.to(torch.bfloat16)
        m.decoder.mask_override = forced
        masks, classes = m(px.to(DEV).to(torch.bfloat16))
    ours = _rel_errors(masks, rmasks)
    yard = _rel_errors(omasks, rmasks)
    cerr = max(float((a.float().cpu() - b).abs().max()) for a, b in zip(classes, rclasses))
    print(f"swin_t@{size} bf16 production path: max|err|/max|logit| {ours[0]:.2e}, mean {ours[1]:.2e}; "
          f"oracle-in-bf16 {yard[0]:.2e} / {yard[1]:.2e} ({t16:.1f}s); class-logit max|err| {cerr:.2e}")
    assert ours[0] <= 1.25 * yard[0] and ours[1] <= 1.25 * yard[1]
    assert ours[0] <= 0.03 and ours[1] <= 0.004
    assert cerr <= 0.05


def test_swin_b_c3_model_vs_oracle():
    """Config C3's model (Swin-B + Mask2Former, ws 12: the 64 < N <= 160 window-attention
    kernels in every block) vs the oracle at 512^2, oracle attention masks forced in:
    fp32 kernel mode within the BASELINE bound 1e-3; the bf16 production path within
    max 0.05 / mean 0.006 of the step's max |logit| (Swin-T at the same settings: 0.015 /
    0.0024)."""
    m, ref, cfg = _swin_t_pair(512, preset="swin_b")
    with torch.no_grad():
        for p in list(m.parameters()) + list(ref.parameters()):
            p.copy_(p.to(torch.bfloat16).float())
    px = torch.randn(1, 3, 512, 512, generator=torch.Generator().manual_seed(5)).to(torch.bfloat16).float()
    with torch.no_grad():
        ref.decoder.record = True
        rmasks, rclasses = ref(px)
        forced = [rb for rb, _ in ref.decoder.trace]
        m.decoder.mask_override = forced
        fmasks, fclasses = m(px.to(DEV))
        f32err = max(float((a.cpu() - b).abs().max()) for a, b in zip(fmasks, rmasks))
        m = m.to(torch.bfloat16)
        bmasks, _ = m(px.to(DEV).to(torch.bfloat16))
    ours = _rel_errors(bmasks, rmasks)
    print(f"swin_b@512: fp32-mode mask-logit max|err| {f32err:.2e}; bf16 production max|err|/max|logit| "
          f"{ours[0]:.2e}, mean {ours[1]:.2e}")
    assert f32err <= 1e-3
    assert ours[0] <= 0.05 and ours[1] <= 0.006


def test_bf16_training_step():
    from visionseg.model import M2FConfig, Mask2Former
    from visionseg.criterion import SetCriterion
    from visionseg.train import Trainer, SolverConfig
    from visionseg.data import synthetic_batch
    cfg = M2FConfig.preset("swin_t", train_num_points=1024)
    m = Mask2Former(cfg).init_weights(0)
    tr = Trainer(m, SetCriterion(cfg), SolverConfig(warmup_iters=0), device=DEV)
    imgs, ml, cl = synthetic_batch(2, 512, seed=3, device=DEV)
    losses = [float(tr.step(imgs, ml, cl)) for _ in range(3)]
    assert all(np.isfinite(losses)), losses
    for p in m.parameters():
        assert torch.isfinite(p).all()
    print("bf16 losses", losses)


@pytest.mark.parametrize("arch", ["maskdino", "mask2former"])
def test_train_template_seam_and_inference_seam(tmp_path, arch):
    """train_template.train_maskdino(...) contract (metrics dict, results, checkpoint; the
    MaskDINO model) and the `--model mask2former` branch, through the prefetching loader
    (2 worker processes), and the ai_segmentation init_detector / inference_detector
    contract on the trained model (MaskDINO recognised from its checkpoint)."""
    from visionseg import adapters
    from visionseg.data import write_coco_dataset
    from visionseg.inference import init_detector, inference_detector
    train_maskdino = adapters.train_maskdino if arch == "maskdino" else adapters.train_mask2former
    write_coco_dataset(str(tmp_path / "train"), 4, 128, seed=1)
    write_coco_dataset(str(tmp_path / "val"), 2, 128, seed=2)
    hp = dict(epochs=2, batch_size=2, img_size=128, save_period=1, warmup_epochs=0, workers=2)
    r = train_maskdino("exp_test", tmp_path / "train", tmp_path / "val", tmp_path / "out", hp)
    assert set(r) == {"mAP50", "mAP75", "mAP", "precision", "recall"}
    assert all(0.0 <= v <= 1.0 for v in r.values())
    assert (tmp_path / "out" / "model_final.pth").exists() and (tmp_path / "out" / "model_epoch0002.pth").exists()
    assert train_maskdino("missing", tmp_path / "nope", tmp_path / "val", tmp_path / "out2", hp) is None
    det = init_detector("swin_t", str(tmp_path / "out" / "model_final.pth"), device="cuda:0")
    img = (np.random.default_rng(0).integers(0, 256, (100, 140, 3))).astype(np.uint8)
    res = inference_detector(det, img)
    pi = res.pred_instances
    assert len(pi) == 100 and pi.masks.shape == (100, 100, 140) and pi.masks.dtype == torch.bool
    best = int(pi.scores.cpu().numpy().argmax())                  # the caller's selection (ai_segmentation.py:83-88)
    mask = pi.masks[best].cpu().numpy()
    assert mask.shape == img.shape[:2] and int(pi.labels[best]) == 0


def test_predictor_graph_replay_matches_eager():
    """The inference Predictor (labeling_server seam): the pure-bf16 forward replayed as a
    HIP graph per padded input shape, for more shapes than the LRU keeps (graphs are
    evicted and recaptured).

    (1) A shape replayed after its graph was evicted and recaptured gives bit-identical
    instances (the stale-argument / freed-constant failure modes of graph reuse).
    (2) Graph replay vs the eager forward: same labels, scores within 2e-2, at most 3 % of
    mask pixels flipped.  Not bit-exact: inside a long test process the vendor libraries
    (hipBLASLt, MIOpen) occasionally ran another solver for a captured launch than for the
    eager one; with bf16 activations that moves logits in the last bits, a decoder
    attention-mask bit near the threshold flips, and the self-attention carries the flip
    on (scores moved up to 7.7e-3 in 2 of 6 full-file runs; in a fresh process, 16 shape
    passes were bit-identical, tools/pred_debug.py)."""
    from visionseg.inference import Predictor
    from visionseg.model import M2FConfig, Mask2Former
    cfg = M2FConfig.preset("swin_t")
    m = Mask2Former(cfg).init_weights(0)
    pg = Predictor(m, device=DEV, min_size=256, max_size=320, graphs=True, max_graphs=2)
    pe = Predictor(m, device=DEV, min_size=256, max_size=320, graphs=False)
    assert pg.graphs and next(pg.model.parameters()).dtype == torch.bfloat16
    assert next(m.parameters()).dtype == torch.float32           # the caller's model is left as it is
    rng = np.random.default_rng(0)
    imgs = [rng.integers(0, 256, (*shape, 3)).astype(np.uint8) for shape in ((200, 260), (256, 256), (300, 180))]
    first = None
    for img in imgs + [imgs[0]]:                                   # the last one: (200, 260) after eviction
        a, b = pg(img).pred_instances, pe(img).pred_instances
        if first is None:
            first = a
        assert torch.equal(a.labels, b.labels)
        assert float((a.scores - b.scores).abs().max()) <= 2e-2
        assert float((a.masks != b.masks).float().mean()) <= 3e-2
    assert torch.equal(a.masks, first.masks) and torch.equal(a.scores, first.scores)   # recaptured == first capture
    assert len(pg._graphs) == 2


@pytest.mark.gpu
def test_predictor_bf16_vs_f32_model():
    """The default Predictor (amp: a pure-bf16 copy of the model, bf16 activations, the
    production MFMA kernels) against the same model run in f32 (amp=False: f32 parameters
    and the f32 kernel mode), on the same preprocessed images, free-running (the decoder's
    attention masks are each path's own, so a bf16 flip of a near-zero mask logit changes
    what later layers attend to).  Bounds: class probabilities within 8e-2, at least 98 % of
    the binary-mask pixels equal, the post-processed top-20 scores (sorted, so near-tie
    reorderings between equal scores do not count) within 2e-2, and the mask logits within
    1e-2 of the max |logit| on average (box, both shapes: class probabilities 1.8e-2 and
    3.5e-2, mean logit difference 3.8e-3 and 4.7e-3, 99.1-99.3 % of the mask pixels equal,
    top-20 scores within 3.3e-3).  The largest mask-logit difference is only bounded
    loosely (0.5 of max): free-running, it sits where a flipped attention-mask bit changed a
    later layer's input, and which bits flip depends on the convolution solver MIOpen's Find
    picks in the process (box runs, 200 x 260: 8.8e-2 and 2.2e-1 of max, with 99.3 % of the
    mask pixels equal, class probabilities within 2.3e-2, top-20 scores within 3.1e-3).  With
    the attention masks forced, the same kernels stay within 1.4 % of max |logit|
    (test_swin_t_bf16_production_path_vs_oracle)."""
    from visionseg.inference import Predictor, instance_inference
    from visionseg.model import M2FConfig, Mask2Former
    m = Mask2Former(M2FConfig.preset("swin_t")).init_weights(0)
    pb = Predictor(m, device=DEV, min_size=256, max_size=320, graphs=False)
    pf = Predictor(m, device=DEV, min_size=256, max_size=320, amp=False, graphs=False)
    assert next(pb.model.parameters()).dtype == torch.bfloat16
    assert next(pf.model.parameters()).dtype == torch.float32
    rng = np.random.default_rng(1)
    for shape in ((200, 260), (300, 180)):
        img = rng.integers(0, 256, (*shape, 3)).astype(np.uint8)
        x, valid, orig = pf._preprocess(img)
        with torch.no_grad():
            ob, of = pb._forward(x.to(torch.bfloat16)), pf._forward(x)
        mb, cb = ob[0][-1][0].float(), ob[1][-1][0].float()
        mf, cf = of[0][-1][0].float(), of[1][-1][0].float()
        dprob = float((cb.softmax(-1) - cf.softmax(-1)).abs().max())
        scale = float(mf.abs().max())
        dm = float((mb - mf).abs().max()) / scale
        agree = float(((mb > 0) == (mf > 0)).float().mean())
        sb = instance_inference(mb, cb, orig, valid_hw=valid, pad_hw=tuple(x.shape[-2:]), top_k=20)[0]
        sf = instance_inference(mf, cf, orig, valid_hw=valid, pad_hw=tuple(x.shape[-2:]), top_k=20)[0]
        ds = float((sb.sort().values - sf.sort().values).abs().max())
        dmean = float((mb - mf).abs().mean()) / scale
        print(f"predictor bf16 vs f32 {shape}: class prob {dprob:.2e}, mask logit {dm:.2e} of max "
              f"(mean {dmean:.2e}), mask agreement {agree:.4f}, top-20 scores {ds:.2e}")
        assert dprob <= 8e-2 and dmean <= 1e-2 and dm <= 0.5 and agree >= 0.98 and ds <= 2e-2, \
            (dprob, dmean, dm, agree, ds)
        # the full seam agrees too (bf16 path end to end, post-processing included)
        res = pb(img).pred_instances
        assert res.masks.shape[1:] == shape and len(res) == 100
