#!/bin/bash
# Round-4 GPU call: the full -m gpu suite at this tree (+ smoke).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread \
    --durations=25 > $O/gpu_tests_full.log 2>&1
rc=$?
tail -3 $O/gpu_tests_full.log
grep -E "bf16 step mean|FAILED" $O/gpu_tests_full.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?
tail -2 $O/smoke.log
exit $rc
