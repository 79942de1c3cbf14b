#!/bin/bash
# C2 bench line + graph-replayed step trace with per-category breakdown
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6p
mkdir -p $O
timeout -k 10 500 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/graph -o bench -- python3 bench.py --no-cpu-baseline --no-parity --kernel-timing 0 --steps 4 --warmup 3 > $O/graph.log 2>&1 || exit $?
python3 tools/step_breakdown.py $O/graph/bench_kernel_trace.csv 80 > $O/breakdown.txt || exit $?
rm -f $O/graph/bench_kernel_trace.csv
head -60 $O/breakdown.txt
