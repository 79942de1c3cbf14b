#!/bin/bash
# Round-4 msda backward: pyramid-column kernel tests vs the oracle / tile kernel, then the
# kernel bench (column 8x16 / 16x16 / 8x8 vs the 8 x 8 tile kernel) on smooth and iid offsets.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -k "msda" --timeout 200 \
    --timeout-method thread > gpurun_out/r4/msda_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4/msda_tests.log
grep -E "^FAILED|Error|assert" gpurun_out/r4/msda_tests.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python tools/kbench.py --only msda --msda-modes col,prod,col16,col8,taps4,col,prod --iters 20 \
    > gpurun_out/r4/msda_kbench.txt 2>&1
rc2=$?
grep msda gpurun_out/r4/msda_kbench.txt
exit $rc2
