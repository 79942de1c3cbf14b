#!/bin/bash
# token_wgrad: one-round plan; DMA spread A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5m
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tgemm.py -k "wgrad or deferred" > $O/tests.log 2>&1
rc=$?
tail -1 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head | cut -c1-200; [ $rc -ne 0 ] && exit $rc
for sp in 0 1; do
  VS_WGRAD_SPREAD=$sp timeout -k 10 200 python3 -u tools/r5/wgrad_ab.py --quick > $O/wg$sp.log 2>&1 || exit $?
done
paste <(grep token_wgrad $O/wg0.log | cut -c1-62) <(grep token_wgrad $O/wg1.log | cut -c49-62)
grep total $O/wg0.log $O/wg1.log
