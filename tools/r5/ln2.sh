#!/bin/bash
# colsum_partials 32 x 32 slices: norm / column-sum tests, kernel stats of a short bench, bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ln2
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_tgemm.py -k "norm or colsum or column or bias or linear" > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o b -- python3 bench.py --no-cpu-baseline --no-parity --steps 5 > $O/trace.log 2>&1 || exit $?
grep -h "colsum_partials\|ln_bwd_kernel" $O/trace/b_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
rm -f $O/trace/b_kernel_trace.csv
timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-parity > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-200
