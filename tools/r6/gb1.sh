#!/bin/bash
# MLP GELU backward in fc2's dX epilogue: tgemm tests, model / training-parity tests, A/B bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${OUT:-r6s}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_tgemm.py > $O/tgemm.log 2>&1 || { tail -30 $O/tgemm.log; exit 1; }
tail -1 $O/tgemm.log
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_train_parity.py tests/test_gpu_fp8.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_bench.sh ${AB_DIR:-r6s/ab} 3
