#!/bin/bash
# after the second prune (dst backward, two-pass window forward, wgrad / table-sum switches):
# op tests of the touched kernels + a bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6j
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_tgemm.py tests/test_gpu_fp8.py tests/test_gpu_self_attn.py > $O/tests.log 2>&1
rc=$?
tail -1 $O/tests.log
grep -E "^FAILED|Error" $O/tests.log | cut -c1-300 | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-200
