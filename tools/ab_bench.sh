#!/bin/bash
# Same-box C2 bench A/B: ab_old/ (tools/mk_ab_old.sh) vs the working tree, interleaved.
#   tools/ab_bench.sh <out dir under gpurun_out> [rounds]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-ab}
R=${2:-3}
mkdir -p $O
for i in $(seq 1 $R); do
  for side in old new; do
    b=bench.py
    [ $side = old ] && b=ab_old/bench.py
    timeout -k 10 300 python3 $b --no-cpu-baseline --no-parity > $O/$side$i.log 2>&1 || exit $?
    python3 -c "
import json
d=json.loads([l for l in open('$O/$side$i.log') if l.startswith('{')][-1])
print('$side', d['value'], d['ms_per_step'])"
  done
done
