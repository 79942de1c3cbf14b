#!/bin/bash
# final-tree C2 graph-step breakdown + eager call-site attribution of the glue kernels
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6k
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/graph -o bench -- python3 bench.py --no-cpu-baseline --no-parity --kernel-timing 0 --steps 4 --warmup 3 > $O/graph.log 2>&1 || exit $?
python3 tools/step_breakdown.py $O/graph/bench_kernel_trace.csv 90 > $O/breakdown.txt || exit $?
rm -f $O/graph/bench_kernel_trace.csv
head -8 $O/breakdown.txt
timeout -k 10 500 python3 -u tools/torch_prof.py > $O/tprof.txt 2>&1 || exit $?
grep -A40 "glue ops by call site" $O/tprof.txt | cut -c1-250
