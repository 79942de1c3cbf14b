#!/bin/bash
# Round-4 GPU call: LDS-resident top-k -- kernel tests, criterion / MaskDINO tests, C4 and C2 lines.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py -m gpu -v --timeout 120 --timeout-method thread > $O/topk2_tests.log 2>&1
rc=$?; tail -3 $O/topk2_tests.log; grep -E "^FAILED|Error" $O/topk2_tests.log | head -20 | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_point_loss.py tests/test_gpu_maskdino.py tests/test_gpu_train_parity.py -m gpu -q \
    --timeout 300 --timeout-method thread > $O/topk2_crit_tests.log 2>&1
rc=$?; tail -2 $O/topk2_crit_tests.log; grep -E "^FAILED" $O/topk2_crit_tests.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --arch maskdino --model swin_l --no-cpu-baseline --no-parity --steps 5 > $O/c4_topk2.log 2>&1 || exit $?
tail -1 $O/c4_topk2.log | cut -c1-200
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity --steps 10 > $O/c2_topk2.log 2>&1 || exit $?
tail -1 $O/c2_topk2.log | cut -c1-200
