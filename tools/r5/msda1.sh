#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -v tests/test_gpu_ops.py -k "msda" -s --timeout 250 -x > $O/msda_tests.log 2>&1
rc=$?
tail -2 $O/msda_tests.log
grep -E "FAILED|Error|assert" $O/msda_tests.log | head -20 | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/kbench.py --only msda --msda-modes dst,col --iters 10 > $O/msda_kbench.log 2>&1
cat $O/msda_kbench.log | grep -v amdgpu.ids
