"""Runs of one (kernel, grid) in a rocprofv3 kernel trace of tools/lnbench.py, in launch
order, with the median duration of each run: python3 tools/r5/ln_shapes.py <kernel_trace.csv>"""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "ln_" not in n and "colsum" not in n:
        continue
    n = n.replace("void vs::(anonymous namespace)::", "").split("(")[0]
    rows.append((int(r["Start_Timestamp"]), n, r.get("Grid_Size_X", r.get("Grid_Size")),
                 (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
rows.sort()
# lnbench: per shape, backward calls (ln_bwd + colsum) then forward calls; a new shape starts
# where a backward follows a forward
stats, order, phase, prev = {}, [], 0, ""
for t, n, g, d in rows:
    if n.startswith("ln_bwd") and prev.startswith("ln_fwd"):
        phase += 1
    prev = n
    k = (phase, n, g)
    if k not in stats:
        stats[k] = []
        order.append(k)
    stats[k].append(d)
for k in order:
    v = sorted(stats[k])
    print(f"shape {k[0]}  {k[1]:55s} grid {k[2]:>8}  n {len(v):4d}  median {v[len(v) // 2]:8.2f} us")
