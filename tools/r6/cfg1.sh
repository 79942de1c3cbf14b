#!/bin/bash
# configs at their per-GPU shapes + model/tgemm tests + C2 bench (token path from 4096 tokens)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_model.py tests/test_gpu_tgemm.py > $O/tests.log 2>&1
rc=$?
grep -E "C3 |C4 |C5 |passed|failed|FAILED" $O/tests.log | cut -c1-300
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 500 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-250
exit $rc
