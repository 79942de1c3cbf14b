"""Per-step kernel breakdown from a rocprofv3 --kernel-trace CSV of bench.py.

A step is delimited by the flat optimiser step launches (flat_step_kernel): the
last complete step is the span after the second-to-last optimizer burst up to the end
of the last one.  Prints busy time by category and the top kernels of that step.
Usage: python tools/step_breakdown.py <kernel_trace.csv> [top] [step]
step counts back from the end (-1 = last, -3 = the last graph-replayed step of a bench
run whose final 2 steps are the eager kernel-timing steps).  The timing steps' device
spin kernels (bench.py keeps the host enqueue out of the measured window) are dropped.
"""
import csv
import sys
from collections import defaultdict


def category(name):
    n = name
    if n.startswith("Cijk_") or "gemm" in n.lower() or n.startswith("igemm"):
        return "gemm"
    if "vs::" in n:
        return "hip_kernels"
    if "layer_norm" in n or "GammaBeta" in n or "cuComputeGradInput" in n:
        return "layernorm"
    if "reduce_kernel" in n or "Moments" in n:
        return "reductions"
    if "copy" in n.lower() or "fillBuffer" in n:
        return "copies"
    if "elementwise" in n:
        return "elementwise"
    return "other"


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    which = int(sys.argv[3]) if len(sys.argv) > 3 else -1
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if "spin_kernel" not in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    opt = [i for i, r in enumerate(rows) if "flat_step_kernel" in r[2]]
    # group optimizer launches into bursts
    # bursts separated by the forward/backward: split at gaps above half the largest gap
    thr = max(b - a for a, b in zip(opt, opt[1:])) // 2
    bursts, cur = [], [opt[0]]
    for i in opt[1:]:
        if i - cur[-1] <= thr:
            cur.append(i)
        else:
            bursts.append(cur)
            cur = [i]
    bursts.append(cur)
    a, b = bursts[which - 1][-1] + 1, bursts[which][-1]
    step = rows[a:b + 1]
    window = (step[-1][1] - step[0][0]) / 1e6
    busy = sum(e - s for s, e, _ in step) / 1e6
    cat, per = defaultdict(float), defaultdict(lambda: [0.0, 0])
    for s, e, n in step:
        cat[category(n)] += (e - s) / 1e6
        per[n][0] += (e - s) / 1e6
        per[n][1] += 1
    print(f"# step {which} window {window:.1f} ms under the profiler; kernel busy {busy:.1f} ms, {len(step)} launches")
    for k, v in sorted(cat.items(), key=lambda x: -x[1]):
        print(f"#   {k:12s} {v:7.2f} ms")
    for n, (t, c) in sorted(per.items(), key=lambda x: -x[1][0])[:top]:
        print(f"{t:8.3f} ms {c:5d}  {n[:150]}")
    # idle gaps between consecutive kernels (host-side waits: syncs, launch overhead)
    gaps = []
    end = step[0][1]
    for i in range(1, len(step)):
        s_, e_, n_ = step[i]
        if s_ > end:
            gaps.append(((s_ - end) / 1e6, i))
        end = max(end, e_)
    idle = sum(g for g, _ in gaps)
    small = sum(g for g, _ in gaps if g < 0.05)
    print(f"# idle {idle:.1f} ms in {len(gaps)} gaps ({small:.1f} ms in gaps < 50 us); largest:")
    for g, i in sorted(gaps, reverse=True)[:12]:
        print(f"#   {g:7.3f} ms at launch {i}: after {step[i - 1][2][:60]}  ->  {step[i][2][:60]}")


if __name__ == "__main__":
    main()
