#!/bin/bash
# maskdino factor test, then the C2 profile set: rocprofv3 kernel trace + stats of the
# default bench command (graph-replayed steps) and SQ counters of the hand-written kernels.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -q tests/test_gpu_maskdino.py -k factor_mask --timeout 200 > $O/maskdino_factor.log 2>&1
tail -2 $O/maskdino_factor.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py --no-cpu-baseline --no-parity > $O/trace.log 2>&1 || exit $?
tail -1 $O/trace.log | cut -c1-300
python3 tools/step_breakdown.py $O/trace/bench_kernel_trace.csv 70 -3 > $O/step_graph.txt 2>&1 || true
head -60 $O/step_graph.txt | cut -c1-200
bash tools/r5/pmc_sq.sh
