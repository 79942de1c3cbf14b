#!/bin/bash
# Round-4 GPU call: the fp8 tests (incl. the fp8-Linear model vs oracle + training step),
# then the C5 lines and the C2 fused-GELU A/B (tools/r4_c5.sh).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp8.py -m gpu -q -s --timeout 300 --timeout-method thread \
    > $O/fp8_tests.log 2>&1
rc=$?
tail -2 $O/fp8_tests.log
grep -E "^FAILED|swin_l@384" $O/fp8_tests.log | cut -c1-300
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/r4_c5.sh
