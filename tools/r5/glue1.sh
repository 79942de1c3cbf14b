#!/bin/bash
# C2 glue changes: targeted GPU tests (projections, model, train parity, decoder), the default
# bench line, then a kernel trace of the bench command and its per-step breakdown.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5g
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_tgemm.py tests/test_gpu_model.py tests/test_gpu_train_parity.py tests/test_host_logic.py \
    tests/test_gpu_graphs.py > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head -20 | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py --no-cpu-baseline --no-parity > $O/trace.log 2>&1 || exit $?
python3 tools/step_breakdown.py $O/trace/bench_kernel_trace.csv 70 -3 > $O/step_graph.txt 2>&1 || true
head -45 $O/step_graph.txt | cut -c1-200
