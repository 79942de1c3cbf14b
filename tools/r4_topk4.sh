#!/bin/bash
# Round-4 GPU call: top-k with the row loads issued up front and a one-scan compaction --
# tests, microbenchmark, C4 line.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py -m gpu -q --timeout 120 --timeout-method thread > $O/topk4_tests.log 2>&1
rc=$?; tail -2 $O/topk4_tests.log; grep -E "^FAILED|Error" $O/topk4_tests.log | head -20 | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/topk_bench.py > $O/topk_bench4.txt 2>&1 || exit $?
cat $O/topk_bench4.txt
timeout -k 10 300 python3 bench.py --arch maskdino --model swin_l --no-cpu-baseline --no-parity --steps 5 > $O/c4_topk4.log 2>&1 || exit $?
tail -1 $O/c4_topk4.log | cut -c1-200
