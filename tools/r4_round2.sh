#!/bin/bash
# Round-4 GPU call: the full -m gpu suite at the current tree, then C2 bench lines with the
# pyramid-column msda backward (default) and the 8 x 8 tile kernel (VS_MSDA_COL=0).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread \
    --durations=40 > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
grep -E "bf16 step mean|FAILED" $O/gpu_tests.log | cut -c1-400
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
B="python3 bench.py --no-cpu-baseline --no-parity"
timeout -k 10 300 $B > $O/c2_col.log 2>&1 || exit $?
tail -1 $O/c2_col.log | cut -c1-200
VS_MSDA_COL=0 timeout -k 10 300 $B > $O/c2_tile.log 2>&1 || exit $?
tail -1 $O/c2_tile.log | cut -c1-200
