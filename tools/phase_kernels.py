"""Per-phase kernel listing of one graph-replayed step (rocprofv3 kernel-trace CSV).
Usage: python tools/phase_kernels.py <kernel_trace.csv> <phase> [top]
phase: crit | dec_fwd | dec_bwd | pix_bwd"""
import csv
import sys
from collections import defaultdict

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
              for r in csv.DictReader(open(sys.argv[1])))
opt = [i for i, r in enumerate(rows) if "flat_step_kernel" in r[2]]
step = rows[opt[-2] + 1:opt[-1] + 1]


def first(key):
    return next(i for i, r in enumerate(step) if key in r[2])


last_x = max(i for i, r in enumerate(step) if "xattn_bwd" in r[2] or "mask_head_bwd" in r[2])
bwd0 = first("grid_sampler_2d_backward")
span = {"dec_fwd": (first("mask_head_fwd"), first("match_cost")),
        "crit": (first("match_cost"), bwd0),
        "dec_bwd": (bwd0, last_x + 1),
        "pix_bwd": (last_x + 1, first("win_attn_bwd"))}[sys.argv[2]]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
seg = step[span[0]:span[1]]
print(f"# {sys.argv[2]}: {len(seg)} launches, {sum(e - s for s, e, _ in seg) / 1e6:.2f} ms busy")
per = defaultdict(lambda: [0, 0.0])
for s, e, n in step[span[0]:span[1]]:
    per[n[:110]][0] += 1
    per[n[:110]][1] += (e - s) / 1e3
for n, (c, t) in sorted(per.items(), key=lambda x: -x[1][1])[:top]:
    print(f"{t / 1e3:7.3f} ms {c:4d}  {n}")
