#!/bin/bash
# decoder small Linears with several K chunks in flight: microbenchmark, op tests, training parity, A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6u
mkdir -p $O
timeout -k 10 120 python3 -u tools/r6/small_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "small or decoder or qkv or linear" > $O/ops.log 2>&1 || { tail -30 $O/ops.log; exit 1; }
tail -1 $O/ops.log
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_train_parity.py tests/test_gpu_maskdino.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_bench.sh r6u/ab 3
