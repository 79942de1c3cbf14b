#!/bin/bash
# Round-4 GPU call: top-k variant 1 (aggregated digit counts in every pass, 4 keys per thread
# in the compaction) vs variant 0 -- tests for both, a microbenchmark, the C4 line.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py -m gpu -q --timeout 120 --timeout-method thread > $O/topk3_tests.log 2>&1
rc=$?; tail -2 $O/topk3_tests.log; grep -E "^FAILED|Error" $O/topk3_tests.log | head -20 | cut -c1-300
[ $rc -ne 0 ] && exit $rc
VS_TOPK_VARIANT=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py -m gpu -q --timeout 120 --timeout-method thread > $O/topk3_tests_v0.log 2>&1
rc=$?; tail -1 $O/topk3_tests_v0.log
[ $rc -ne 0 ] && exit $rc
echo "== variant 1" > $O/topk_bench.txt
timeout -k 10 200 python -u tools/topk_bench.py >> $O/topk_bench.txt 2>&1 || exit $?
echo "== variant 0" >> $O/topk_bench.txt
VS_TOPK_VARIANT=0 timeout -k 10 200 python -u tools/topk_bench.py >> $O/topk_bench.txt 2>&1 || exit $?
cat $O/topk_bench.txt
timeout -k 10 300 python3 bench.py --arch maskdino --model swin_l --no-cpu-baseline --no-parity --steps 5 > $O/c4_topk3.log 2>&1 || exit $?
tail -1 $O/c4_topk3.log | cut -c1-200
