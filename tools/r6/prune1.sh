#!/bin/bash
# after the prune + msda adaptive quantum + point-gather XCD order: op tests of the touched kernels
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_tgemm.py tests/test_gpu_point_loss.py tests/test_gpu_self_attn.py > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
grep -E "^FAILED|Error" $O/tests.log | cut -c1-300 | head -20
exit $rc
