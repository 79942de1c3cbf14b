#!/bin/bash
# conv3x3.hip first GPU run: its tests, the timing A/B, then the default bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_conv3x3.py \
    > $O/tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert" $O/tests.log | head -40 | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/r5/conv_ab.py > $O/conv_ab.log 2>&1 || exit $?
cat $O/conv_ab.log
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-300
