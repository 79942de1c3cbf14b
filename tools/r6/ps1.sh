#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_point_loss.py tests/test_gpu_maskdino.py tests/test_gpu_train_parity.py > $O/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tests.log | cut -c1-300 | head; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/graph -o bench -- python3 bench.py --no-cpu-baseline --no-parity --kernel-timing 0 --steps 4 --warmup 3 > $O/graph.log 2>&1 || exit $?
python3 tools/step_breakdown.py $O/graph/bench_kernel_trace.csv 200 > $O/breakdown.txt || exit $?
rm -f $O/graph/bench_kernel_trace.csv
head -8 $O/breakdown.txt
