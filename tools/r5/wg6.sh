#!/bin/bash
# token_wgrad: WG order (split-major / tile-major) x tile (256x128 / 128x128 two-per-CU)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5k
mkdir -p $O
timeout -k 10 200 python -u -m pytest -q --timeout 100 --timeout-method thread -m gpu tests/test_gpu_tgemm.py -k "wgrad" > $O/tests.log 2>&1
rc=$?
tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
VS_WGRAD_SMALL=1 timeout -k 10 200 python -u -m pytest -q --timeout 100 --timeout-method thread -m gpu tests/test_gpu_tgemm.py -k "wgrad" > $O/tests2.log 2>&1 || exit $?
tail -1 $O/tests2.log
for cfg in "0 0" "1 0" "0 1" "1 1"; do
  set -- $cfg
  VS_WGRAD_ORDER=$1 VS_WGRAD_SMALL=$2 timeout -k 10 200 python3 -u tools/r5/wgrad_ab.py --quick > $O/wg_$1$2.log 2>&1 || exit $?
done
paste <(grep token_wgrad $O/wg_00.log | cut -c1-62) <(grep token_wgrad $O/wg_10.log | cut -c49-62) <(grep token_wgrad $O/wg_01.log | cut -c49-62) <(grep token_wgrad $O/wg_11.log | cut -c49-62)
grep total $O/wg_*.log
