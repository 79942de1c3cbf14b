#!/bin/bash
# glue batch 3 (input projections as token Linears, one level-row add): model / parity tests,
# small-Linear microbenchmark, same-box A/B bench vs ab_old
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6q
mkdir -p $O
timeout -k 10 120 python3 -u tools/r6/small_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_train_parity.py tests/test_gpu_conv3x3.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_bench.sh r6q/ab 3
