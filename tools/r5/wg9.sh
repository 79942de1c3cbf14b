#!/bin/bash
# token_wgrad reduction: 16 split groups per block (default below 1024 blocks) vs 4
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5w9
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tgemm.py -k "wgrad or deferred" > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
for g in 4 0; do
  VS_WGRAD_REDUCE_GROUPS=$g timeout -k 10 200 python3 -u tools/r5/wgrad_ab.py --quick > $O/wg$g.log 2>&1 || exit $?
done
paste <(grep token_wgrad $O/wg4.log | cut -c1-62) <(grep token_wgrad $O/wg0.log | cut -c49-62)
grep total $O/wg4.log $O/wg0.log
for g in 0 4 0; do
  VS_WGRAD_REDUCE_GROUPS=$g timeout -k 10 500 python3 bench.py --no-cpu-baseline --no-parity > $O/bench_$g.log 2>&1 || exit $?
  echo "$g $(tail -1 $O/bench_$g.log | cut -c1-160)"
done
