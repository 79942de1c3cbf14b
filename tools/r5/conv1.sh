#!/bin/bash
# conv3x3.hip + token_wgrad.hip first GPU run: their tests, the timing A/Bs, then the default bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_conv3x3.py \
    tests/test_gpu_tgemm.py -k "conv3x3 or upsample or pixel_decoder or wgrad or plane_projection" > $O/tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert" $O/tests.log | head -50 | cut -c1-300
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python3 -u tools/r5/conv_ab.py > $O/conv_ab.log 2>&1 || exit $?
cat $O/conv_ab.log
timeout -k 10 300 python3 -u tools/r5/wgrad_ab.py > $O/wgrad_ab.log 2>&1 || exit $?
cat $O/wgrad_ab.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-300
