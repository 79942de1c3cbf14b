#!/bin/bash
# graph-replayed C2 step trace -> the kernels around the largest idle gaps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${OUT:-gaps}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/graph -o bench -- python3 bench.py --no-cpu-baseline --no-parity --kernel-timing 0 --steps 4 --warmup 3 > $O/graph.log 2>&1 || exit $?
python3 tools/r6/gap_context.py $O/graph/bench_kernel_trace.csv -1 8 > $O/gaps.txt || exit $?
python3 tools/step_breakdown.py $O/graph/bench_kernel_trace.csv 90 > $O/breakdown.txt || exit $?
gzip -f $O/graph/bench_kernel_trace.csv
