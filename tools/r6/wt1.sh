#!/bin/bash
# batched weight transposes: tgemm tests + C2 bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6m
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_tgemm.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity > $O/bench$i.log 2>&1 || exit $?
  tail -1 $O/bench$i.log | cut -c1-190
done
