#!/bin/bash
# MSDA forward HBM reads: query order vs pyramid-column order (FETCH_SIZE pass each)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6f
mkdir -p $O
A="--no-cpu-baseline --no-parity --graphs 0 --steps 3 --warmup 2"
for c in 1 0; do
  VS_MSDA_FWD_COL=$c timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f$c -o b -- python3 bench.py $A > $O/f$c.log 2>&1 || exit $?
  python3 - <<PY
import sys
sys.path.insert(0, "tools")
from pmc_traffic import load
f = load("$O/f$c/b_counter_collection.csv", "FETCH_SIZE")
for k, v in f.items():
    if "msda_fwd" in k or "msda_bwd_col" in k:
        print("col=$c", k[:40], "fetch MB per dispatch", round(2.0 * sum(v) / len(v) / 1e6, 1), len(v))
PY
  rm -rf $O/f$c
done
