#!/bin/bash
# token_wgrad tile A/B: BI = 128 vs 256 (32-token chunks), and 64-token chunks at BI = 128
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5g2
mkdir -p $O
timeout -k 10 200 python -u -m pytest -q --timeout 100 --timeout-method thread -m gpu tests/test_gpu_tgemm.py -k "wgrad" > $O/tests.log 2>&1
rc=$?
tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
VS_WGRAD_BI=128 VS_WGRAD_CFG=1 timeout -k 10 200 python3 -u tools/r5/wgrad_ab.py --quick > $O/wg_a.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/r5/wgrad_ab.py --quick > $O/wg_b.log 2>&1 || exit $?
VS_WGRAD_BI=128 VS_WGRAD_CFG=0 timeout -k 10 200 python3 -u tools/r5/wgrad_ab.py --quick > $O/wg_c.log 2>&1 || exit $?
paste <(grep token_wgrad $O/wg_a.log | cut -c1-70) <(grep token_wgrad $O/wg_b.log | cut -c36-70) <(grep token_wgrad $O/wg_c.log | cut -c36-70)
grep total $O/wg_a.log $O/wg_b.log $O/wg_c.log
