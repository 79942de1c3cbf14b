#!/bin/bash
# glue batch 2 (colsum record popped, rel-table gradient in 2 launches, batched table casts):
# window / table / tgemm / model tests, then same-box A/B bench vs ab_old
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6o
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "table or window or win" tests/test_gpu_tgemm.py tests/test_gpu_model.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_bench.sh r6o/ab 3
