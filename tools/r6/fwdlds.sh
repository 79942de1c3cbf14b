#!/bin/bash
# MSDA forward: LDS-staged column kernel vs fwd4 (column order) -- bit-equality test, then bench A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6h
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "msda" > $O/tests.log 2>&1 || { grep -E "^FAILED|Error|assert" $O/tests.log | cut -c1-300 | head -20; tail -2 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in 1 0 1 0; do
  VS_MSDA_FWD_LDS=$c timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity > $O/bench_lds$c.log 2>&1 || exit $?
  python3 -c "
import json
d=json.loads([l for l in open('$O/bench_lds$c.log') if l.startswith('{')][-1])
k=d.get('kernels',{})
print('lds=$c', d['value'], d['ms_per_step'], {n: (k[n]['mean_ms'], k[n]['gbs']) for n in k if n.startswith('msda_fwd')})"
done
