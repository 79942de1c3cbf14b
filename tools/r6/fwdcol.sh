#!/bin/bash
# op tests of the touched kernels, then the MSDA forward column order A/B (kbench + bench kernels table)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6e
mkdir -p $O
for c in 1 0 1 0; do
  VS_MSDA_FWD_COL=$c timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity > $O/bench_col$c.log 2>&1 || exit $?
  python3 -c "
import json,sys
d=json.loads([l for l in open('$O/bench_col$c.log') if l.startswith('{')][-1])
k=d.get('kernels',{})
print('col=$c', d['value'], d['ms_per_step'], {n: k[n] for n in k if n.startswith('msda')})"
done
