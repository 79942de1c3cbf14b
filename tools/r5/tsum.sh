#!/bin/bash
# window table-gradient partial sums: column-sum kernel vs the ATen dim-0 sum (VS_TABLE_SUM_ATEN=1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ts
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "window" > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
for a in 0 1 0 1; do
  VS_TABLE_SUM_ATEN=$a timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-parity > $O/bench$a.log 2>&1 || exit $?
  echo "aten=$a $(tail -1 $O/bench$a.log | cut -c90-160)"
done
