#!/bin/bash
# MSDA forward variants, one box interleaved: T=2 (default, 115 VGPR, 4 waves/SIMD), T=1 (78 VGPR, 6 waves),
# T=2 capped at 5 waves (96 VGPR, spills)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6i
mkdir -p $O
for t in 0 1 5 0 1 5; do
  VS_MSDA_FWD_T=$t timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity > $O/b$t.log 2>&1 || exit $?
  python3 -c "
import json
d=json.loads([l for l in open('$O/b$t.log') if l.startswith('{')][-1])
k=d.get('kernels',{})
print('T=$t', d['value'], d['ms_per_step'], {n: (k[n]['mean_ms'], k[n]['gbs']) for n in k if n.startswith('msda_fwd')})"
done
