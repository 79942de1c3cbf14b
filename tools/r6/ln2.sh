#!/bin/bash
# LayerNorm backward: per-kernel durations (ln_bwd vs the partial-row reduction) by rocprofv3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6l
mkdir -p $O
for p in 512 128; do
  VS_LN_BWD_PARTS=$p timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/p$p -o ln -- python3 tools/r6/ln_bench.py > $O/p$p.log 2>&1 || exit 1
  python3 - $O/p$p/ln_kernel_trace.csv $p <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
seq = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows]
# group consecutive launches per shape: the bench runs 33 fwd then 33 (bwd + reduce) per shape
agg = collections.OrderedDict()
shape = -1
prev = None
for name, us in seq:
    short = name.replace("(anonymous namespace)", "").split("(")[0].split("<")[0].split("::")[-1]
    if short == "ln_fwd_kernel" and prev != "ln_fwd_kernel":
        shape += 1
    prev = short
    a = agg.setdefault((shape, short), [0, 0.0])
    a[0] += 1
    a[1] += us
print("PARTS", sys.argv[2])
for (sh, k), (n, t) in agg.items():
    print(f"  shape {sh} {k:28s} n={n:3d} mean {t / n:7.2f} us")
PY
  rm -rf $O/p$p
done
