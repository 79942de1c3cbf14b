#!/bin/bash
# small_linear forward / fused backward: parity tests, C2 bench A/B (VS_SMALL_LINEAR_FUSED),
# data-path throughput (tools/loader_bench.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/sl
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -k "small_linear" tests/test_gpu_ops.py > $O/tests.log 2>&1 || exit $?
for s in 1 0 1; do
  VS_SMALL_LINEAR_FUSED=$s timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity --steps 20 > $O/bench_$s.log 2>&1 || exit $?
  echo "fused=$s $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$s.log)"
done
timeout -k 10 300 python3 tools/loader_bench.py --images 64 --iters 24 --workers 4,8,16 > $O/loader.log 2>&1 || exit $?
cat $O/loader.log
