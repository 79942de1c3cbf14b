"""Time ops.topk_rows (csrc/topk.hip) against torch.topk on the importance-sampling shapes:
rows x 37 632 uncertainties (-|logit|), k = 9 408, with continuous values and with heavy
duplication (a coarse grid of values, many equal keys per digit)."""
import sys
import time

import torch

sys.path.insert(0, "vision-instance-seg_amd")
from visionseg import ops  # noqa: E402


def bench(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    n, k = 37632, 9408
    g = torch.Generator(device=dev).manual_seed(0)
    for rows in (160, 400, 4000):
        cont = -torch.abs(torch.randn(rows, n, device=dev, generator=g))
        dup = -torch.abs(torch.round(torch.randn(rows, n, device=dev, generator=g) * 8) / 8)
        tiny = -torch.abs(torch.randn(rows, n, device=dev, generator=g) * 1e-3 + 1e-2)
        for name, x in (("continuous", cont), ("dup1/8", dup), ("narrow", tiny)):
            a = bench(lambda: ops.topk_rows(x, k))
            b = bench(lambda: torch.topk(x, k, dim=1))
            print(f"rows {rows:5d} {name:10s} topk_rows {a:7.3f} ms  torch.topk {b:7.3f} ms", flush=True)


if __name__ == "__main__":
    main()
