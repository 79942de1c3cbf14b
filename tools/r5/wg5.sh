#!/bin/bash
# fragment-order partials: wgrad / conv tests, timings, kernel split at stage-3 fc1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tgemm.py tests/test_gpu_conv3x3.py -k "wgrad or conv3x3 or pixel_decoder or linear_backward" > $O/tests.log 2>&1
rc=$?
tail -1 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head | cut -c1-200; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 -u tools/r5/wgrad_ab.py --quick > $O/wg.log 2>&1 || exit $?
grep -E "token_wgrad" $O/wg.log | cut -c1-75
timeout -k 10 300 python3 -u tools/r5/conv_ab.py > $O/conv_ab.log 2>&1 || exit $?
grep conv3x3 $O/conv_ab.log
for d in 0 4; do
  VS_WGRAD_DEBUG=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$d -o w -- python3 -u tools/r5/wg_pmc.py 16384 1536 384 > $O/d$d.log 2>&1 || exit $?
  python3 - $O/t$d/w_kernel_stats.csv $d <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "wgrad" in r["Name"]:
        print("dbg", sys.argv[2], f'{float(r["AverageNs"])/1e3:8.1f} us', r["Name"][:60])
PY
done
