#!/bin/bash
# small_linear token-split weight-gradient kernel: parity tests, then a C2 bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/wg
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -k "small_linear" tests/test_gpu_ops.py > gpurun_out/wg/tests.log 2>&1 || exit $?
for s in 1 0 1; do
  VS_SMALL_WGRAD_SPLIT=$s timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity --steps 20 > gpurun_out/wg/bench_$s.log 2>&1 || exit $?
  echo "split=$s $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/wg/bench_$s.log)"
done
