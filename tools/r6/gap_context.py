"""Kernels around the largest idle gaps of one graph-replayed step (rocprofv3 kernel-trace CSV of
bench.py; the step as in tools/step_breakdown.py).  Usage: gap_context.py <csv> [step] [ngaps]"""
import csv
import sys


def main():
    path = sys.argv[1]
    which = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    ngaps = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if "spin_kernel" not in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                             r.get("Stream_Id", r.get("Queue_Id", "?"))))
    rows.sort()
    opt = [i for i, r in enumerate(rows) if "flat_step_kernel" in r[2]]
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
    gaps = sorted(((step[i + 1][0] - max(r[1] for r in step[:i + 1]), i) for i in range(len(step) - 1)), reverse=True)
    for g, i in gaps[:ngaps]:
        print(f"== gap {g / 1e3:.1f} us after launch {i}")
        for j in range(max(0, i - 4), min(len(step), i + 5)):
            s, e, n, q = step[j]
            print(f"   {j:5d} q{q} {(e - s) / 1e3:8.1f} us  {n[:120]}")


if __name__ == "__main__":
    main()
