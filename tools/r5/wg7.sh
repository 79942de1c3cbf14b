#!/bin/bash
# grouped / deferred weight gradients: tests (op, trainer parity, graphs), bench, step breakdown
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5l
mkdir -p $O
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tgemm.py tests/test_gpu_train_parity.py tests/test_gpu_graphs.py tests/test_gpu_conv3x3.py > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head -20 | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-250
python3 -c "import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); print(json.dumps(d['roofline']))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py --no-cpu-baseline --no-parity > $O/trace.log 2>&1 || exit $?
python3 tools/step_breakdown.py $O/trace/bench_kernel_trace.csv 30 -3 > $O/step_graph.txt 2>&1 || true
head -30 $O/step_graph.txt | cut -c1-160
