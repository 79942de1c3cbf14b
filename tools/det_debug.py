"""Run-to-run determinism of the bf16 inference forward: the same input twice through the
same model, module outputs compared in call order; prints the first modules that differ."""
import os
import sys
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vision-instance-seg_amd")]
import torch
import visionseg  # noqa: F401
from visionseg.model import M2FConfig, Mask2Former

if len(sys.argv) > 1 and sys.argv[1] == "bench":
    torch.backends.cudnn.benchmark = True
cfg = M2FConfig.preset("swin_t")
m = Mask2Former(cfg).init_weights(0).to("cuda").to(torch.bfloat16).eval()
outs = []
def hook(name):
    def f(mod, inp, out):
        t = out[0] if isinstance(out, (tuple, list)) else out
        if isinstance(t, (tuple, list)):
            t = t[0]
        if torch.is_tensor(t):
            outs.append((name, t.detach().float().clone()))
    return f
for n, mod in m.named_modules():
    if n:
        mod.register_forward_hook(hook(n))
x = torch.randn(1, 3, 320, 224, device="cuda").to(torch.bfloat16)
res = []
NR = int(os.environ.get("DET_RUNS", "4"))
with torch.no_grad():
    for it in range(NR):
        outs.clear()
        m(x)
        torch.cuda.synchronize()
        res.append(list(outs))
for it in range(1, NR):
    bad = [(a[0], float((a[1] - b[1]).abs().max())) for a, b in zip(res[0], res[it]) if not torch.equal(a[1], b[1])]
    if bad or it == NR - 1:
        print(f"run {it} vs 0: {len(bad)} of {len(res[0])} module outputs differ; first: {bad[:4]}")
