#!/bin/bash
# token_wgrad time split under rocprofv3 (kernel time only): normal / no MFMA / no DMA / loop skeleton / epilogue only
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5i
mkdir -p $O
for d in 0 1 2 3 4; do
  VS_WGRAD_DEBUG=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$d -o w -- python3 -u tools/r5/wg_pmc.py 16384 1536 384 > $O/d$d.log 2>&1 || exit $?
  python3 - $O/t$d/w_kernel_stats.csv $d <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "wgrad" in r["Name"]:
        print("dbg", sys.argv[2], f'{float(r["AverageNs"])/1e3:8.1f} us', r["Name"][:60])
PY
done
