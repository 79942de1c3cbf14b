#!/bin/bash
# Round-4 GPU call: MaskDINO tests (incl. the point-sample-rows kernel), then the C4 line.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_maskdino.py -m gpu -q --timeout 300 --timeout-method thread \
    > $O/maskdino_tests.log 2>&1
rc=$?
tail -2 $O/maskdino_tests.log
grep -E "^FAILED" $O/maskdino_tests.log | head
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --arch maskdino --model swin_l --no-cpu-baseline --no-parity --steps 5 > $O/c4_psr.log 2>&1 || exit $?
tail -1 $O/c4_psr.log | cut -c1-200
