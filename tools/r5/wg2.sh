#!/bin/bash
# token_wgrad ring + parallel reduce: tests, kernel-trace of the A/B script, bench + step breakdown.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_conv3x3.py \
    tests/test_gpu_tgemm.py -k "conv3x3 or upsample or pixel_decoder or wgrad or plane_projection or dgrad or linear" > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head -20 | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/r5/conv_ab.py > $O/conv_ab.log 2>&1 || exit $?
grep conv3x3 $O/conv_ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/wtrace -o wg -- python3 -u tools/r5/wgrad_ab.py > $O/wgrad_ab.log 2>&1 || exit $?
grep -E "total|s1 qkv|s3 fc1|enc fc1" $O/wgrad_ab.log
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r5e/wtrace/wg_kernel_stats.csv")))
for r in rows:
    n = r["Name"]
    if "wgrad" in n or "splitk" in n or "colsum" in n or "token_gemm" in n:
        print(f'{float(r["AverageNs"])/1e3:9.1f} us avg {int(r["Calls"]):5d} calls  {n[:110]}')
PY
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py --no-cpu-baseline --no-parity > $O/trace.log 2>&1 || exit $?
python3 tools/step_breakdown.py $O/trace/bench_kernel_trace.csv 50 -3 > $O/step_graph.txt 2>&1 || true
head -40 $O/step_graph.txt | cut -c1-180
