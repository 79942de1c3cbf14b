"""The fused flat-buffer optimiser step (csrc/optim.hip through visionseg.optim.FlatOptimizer)
vs the reference's solver restated in oracle/ref_solver.py (detectron2 parameter groups,
clip_grad_norm_ per parameter / global, torch's own CPU SGD / AdamW), and the in-graph
external-event mechanism the overlapped gradient all-reduce relies on."""
import copy

import pytest
import torch

from oracle.ref_solver import ref_clip_full_model, ref_clip_per_parameter, ref_optimizer, ref_param_groups

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _tiny_model():
    from visionseg.model import M2FConfig, Mask2Former
    cfg = M2FConfig(embed_dim=32, depths=(2, 2, 2, 2), num_heads=(1, 2, 4, 8), feature_size=64,
                    mask_feature_size=64, hidden_dim=64, enc_ffn=128, dec_ffn=128, dec_heads=2, enc_layers=2,
                    dec_layers=4, num_queries=10)
    return Mask2Former(cfg).init_weights(3)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("optimizer,clip", [("sgd", "norm"), ("sgd", "none"), ("adamw", "norm"),
                                            ("adamw", "full_model"), ("sgd", "full_model")])
def test_flat_step_vs_oracle_solver(dtype, optimizer, clip):
    from visionseg.optim import FlatOptimizer
    from visionseg.train import SolverConfig
    s = SolverConfig(optimizer=optimizer, clip_type=clip, clip_value=0.01, lr=0.02)
    ref = _tiny_model()
    prod = copy.deepcopy(ref).to(DEV).to(dtype)
    with torch.no_grad():                       # both start from the same (dtype-rounded) weights
        for p, q in zip(ref.parameters(), prod.parameters()):
            p.copy_(q.float().cpu())
    groups = ref_param_groups(ref, s.lr, s.weight_decay, optimizer, s.backbone_multiplier)
    ropt = ref_optimizer(groups, optimizer, s.momentum, s.betas, s.eps)
    opt = FlatOptimizer(prod, s, DEV)
    byname = dict(zip(opt.names, opt.grad_views))
    rparams = dict(ref.named_parameters())
    bases = [grp["lr"] for grp in ropt.param_groups]
    g = torch.Generator().manual_seed(11)
    flag = dict(zip(opt.names, opt.flag_views))
    for it in range(4):
        with torch.no_grad():
            opt.flags.fill_(1.0)
            for k, (name, p) in enumerate(rparams.items()):
                # gradient magnitudes on both sides of the clip threshold
                gr = torch.randn(p.shape, generator=g) * (10 ** float(torch.empty(()).uniform_(-5, 0, generator=g)))
                gr = gr.to(dtype).float()
                if it < 2 and k % 4 == it:
                    # no gradient this step (torch.optim skips .grad None: no decay, no
                    # momentum; AdamW's bias correction counts the parameter's own steps)
                    p.grad = None
                    byname[name].zero_()
                    flag[name].zero_()
                    continue
                p.grad = gr.clone()
                byname[name].copy_(gr.to(dtype))
        if clip == "norm":
            ref_clip_per_parameter(list(rparams.values()), s.clip_value)
        elif clip == "full_model":
            ref_clip_full_model(list(rparams.values()), s.clip_value)
        factor = 0.5 + 0.25 * it                 # a changing schedule
        for grp, base in zip(ropt.param_groups, bases):
            grp["lr"] = base * factor
        opt.set_lr(s.lr * factor)
        ropt.step()
        opt.step()
    torch.cuda.synchronize()
    assert float(opt.step_count) == 4
    steps = opt.param_steps.cpu().tolist()
    assert min(steps) == 3 and max(steps) == 4
    worst = 0.0
    for name, m in zip(opt.names, opt.layout.views(opt.master)):
        r = rparams[name].detach()
        err = float((m.cpu() - r).abs().max())
        worst = max(worst, err / (float(r.abs().max()) + s.lr))
    print(f"{optimizer}/{clip}/{dtype}: worst master-weight error {worst:.2e} (relative to max|p| + lr)")
    # f32 arithmetic in another order (the global norm of "full_model" is one block's sum
    # over the chunk partials): a few f32 ulps of the weight scale
    assert worst <= 4e-6
    if dtype == torch.bfloat16:                 # working weights = bf16 rounding of the master
        assert torch.equal(opt.weights, opt.master.to(torch.bfloat16))
        for p, w in zip(opt.params, opt.layout.views(opt.weights)):
            assert p.data_ptr() == w.data_ptr()


def test_external_event_orders_side_stream():
    """A side-stream copy issued AFTER a graph launch, waiting on an external event the
    graph records mid-way, sees what the graph wrote before the event and runs before
    the graph's tail (what GradReducer.replay_collectives relies on)."""
    a = torch.zeros(1 << 20, device=DEV)
    out = torch.zeros_like(a)
    x = torch.randn(2048, 2048, device=DEV)
    from visionseg.optim import ExternalEvent
    ev = ExternalEvent()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        y = x
        for _ in range(3):
            y = y @ x
        a.fill_(1.0)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = x
        for _ in range(20):                      # slow head: a no-op wait would copy zeros
            y = (y @ x) * 1e-3
        a.fill_(7.0)
        ev.record()
        for _ in range(40):                      # long tail the side stream may overlap
            y = (y @ x) * 1e-3
    side = torch.cuda.Stream(priority=-1)           # as GradReducer's collective stream
    main = torch.cuda.current_stream()
    overlapped = []
    for _ in range(3):
        a.zero_()
        out.zero_()
        torch.cuda.synchronize()
        t0, t1, t2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        t0.record(main)
        g.replay()
        t2.record(main)
        with torch.cuda.stream(side):
            ev.wait(side)
            out.copy_(a)
            t1.record(side)
        main.wait_stream(side)
        torch.cuda.synchronize()
        assert float(out.min()) == 7.0 and float(out.max()) == 7.0   # ordering: always
        overlapped.append(t0.elapsed_time(t1) < t0.elapsed_time(t2))
    # the side copy finished before the graph's tail did (it overlapped the replay); the
    # hardware-queue placement of streams is the runtime's, so once in three replays
    assert any(overlapped), overlapped
