#!/bin/bash
# MSDA forward tap-batching A/B after the T=1 selection fix: parity for both T, then interleaved benches
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6j
mkdir -p $O
for t in 2 1; do
  VS_MSDA_FWD_T=$t timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k msda > $O/t$t.log 2>&1 || { tail -30 $O/t$t.log; exit 1; }
  tail -2 $O/t$t.log
done
for t in 2 1 2 1; do
  VS_MSDA_FWD_T=$t timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity > $O/b$t.log 2>&1 || exit $?
  python3 -c "
import json
d=json.loads([l for l in open('$O/b$t.log') if l.startswith('{')][-1])
k=d.get('kernels',{})
print('T=$t', d['value'], d['ms_per_step'], {n: (k[n]['mean_ms'], k[n]['gbs']) for n in k if n.startswith('msda_fwd')})"
done
