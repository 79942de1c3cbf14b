#!/bin/bash
# Kernel trace of graph-replayed bench steps + per-step breakdown (idle gaps inside the replay).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pg
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/graph -o bench -- python3 bench.py --no-cpu-baseline --no-parity --kernel-timing 0 --steps 4 --warmup 3 "$@" > $O/graph.log 2>&1 || exit $?
python3 tools/step_breakdown.py $O/graph/bench_kernel_trace.csv 80 > $O/breakdown.txt || exit $?
echo done
