"""C2 pixel-decoder tail timings: the 3x3 output conv (4 x 256 x 256 x 256, bf16) as MIOpen
(NCHW input, channels-last input; Find off / on) vs csrc/conv3x3.hip (forward, input
gradient, weight gradient separately), and the FPN merge NCHW vs NHWC.  HIP events,
median of 20."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, "vision-instance-seg_amd")
from visionseg import ops  # noqa: E402

DEV = "cuda"


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[n // 2]


def main():
    B, C, H, W = 4, 256, 256, 256
    fl = 2.0 * B * H * W * C * C * 9
    x = torch.randn(B, C, H, W, device=DEV).to(torch.bfloat16)
    w = (torch.randn(C, C, 3, 3, device=DEV) * 0.02).to(torch.bfloat16)
    gy = torch.randn(B, C, H, W, device=DEV).to(torch.bfloat16)
    xl, gyl = x.contiguous(memory_format=torch.channels_last), gy.contiguous(memory_format=torch.channels_last)
    for bench in (False, True):
        torch.backends.cudnn.benchmark = bench
        for name, xi, gi in (("nchw", x, gy), ("nhwc", xl, gyl)):
            xs, ws = xi.clone().requires_grad_(), w.clone().requires_grad_()
            tf = timeit(lambda: F.conv2d(xs, ws, padding=1))
            y = F.conv2d(xs, ws, padding=1)
            tb = timeit(lambda: torch.autograd.grad(y, (xs, ws), gi, retain_graph=True))
            print(f"miopen {name} find={int(bench)}: fwd {tf:.3f} ms ({fl / tf / 1e9:.0f} TF/s)  "
                  f"bwd {tb:.3f} ms ({2 * fl / tb / 1e9:.0f} TF/s)", flush=True)
    torch.backends.cudnn.benchmark = False
    xt = xl.permute(0, 2, 3, 1)
    gt = gyl.permute(0, 2, 3, 1)
    wf, wb = ops.conv3x3_layouts(w, True, True)
    t1 = timeit(lambda: ops.conv3x3_raw(xt, wf))
    t2 = timeit(lambda: ops.conv3x3_raw(gt, wb))
    t3 = timeit(lambda: ops.conv3x3_wgrad(gt, xt, torch.bfloat16))
    t4 = timeit(lambda: ops.conv3x3_layouts(w, True, True))
    print(f"conv3x3.hip: fwd {t1:.3f} ms ({fl / t1 / 1e9:.0f} TF/s)  dgrad {t2:.3f} ms ({fl / t2 / 1e9:.0f} TF/s)  "
          f"wgrad {t3:.3f} ms ({fl / t3 / 1e9:.0f} TF/s)  layouts {t4:.3f} ms", flush=True)
    # numerics spot check vs MIOpen
    y0 = F.conv2d(xl, w, padding=1)
    y1 = ops.conv3x3_raw(xt, wf).permute(0, 3, 1, 2)
    print("fwd rel vs miopen", float((y1.float() - y0.float()).norm() / y0.float().norm()), flush=True)
    # FPN merge
    Hs, Ws = 128, 128
    src = torch.randn(B, Hs * Ws, C, device=DEV).to(torch.bfloat16)
    ta = timeit(lambda: ops.upsample_add(x, src, Hs, Ws))
    tb_ = timeit(lambda: ops.upsample_add_nhwc(xl, src, Hs, Ws))
    from visionseg import _lib as L
    gs = torch.empty(B, Hs * Ws, C, device=DEV, dtype=torch.bfloat16)
    tc = timeit(lambda: L.lib().vs_upsample_backward(L.dtype_code(gy), L.ptr(gy), L.ptr(gs), B, C, H, W, Hs, Ws,
                                                     L.stream(gy)))
    td = timeit(lambda: L.lib().vs_upsample_backward_nhwc(L.dtype_code(gy), L.ptr(gyl), L.ptr(gs), B, C, H, W, Hs,
                                                          Ws, L.stream(gy)))
    print(f"upsample_add fwd nchw {ta:.3f} nhwc {tb_:.3f} ms; bwd nchw {tc:.3f} nhwc {td:.3f} ms", flush=True)
    # GroupNorm NCHW vs NHWC (fwd + bwd, relu)
    gw_, gb_ = torch.ones(C, device=DEV, dtype=torch.bfloat16), torch.zeros(C, device=DEV, dtype=torch.bfloat16)
    xa = x.clone().requires_grad_()
    xb = xl.clone().requires_grad_()
    te = timeit(lambda: ops.group_norm_nchw(xa, gw_, gb_, 32, 1e-5, True).backward(gy))
    tf_ = timeit(lambda: ops.group_norm_nhwc(xb, gw_, gb_, 32, 1e-5, True).backward(gyl))
    print(f"group_norm fwd+bwd nchw {te:.3f} nhwc {tf_:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
