#!/bin/bash
# round-5 evidence: wgrad tests + timings, PMC traffic of the C2 bench (FETCH / WRITE passes),
# kernel-trace stats of the default bench command, the default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5p
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tgemm.py -k "wgrad or deferred" > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
timeout -k 10 200 python3 -u tools/r5/wgrad_ab.py --quick > $O/wg.log 2>&1 || exit $?
grep total $O/wg.log
A="--no-cpu-baseline --no-parity"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/c2_$c -o b -- python3 bench.py $A --graphs 0 --steps 3 --warmup 2 > $O/c2_$c.log 2>&1 || exit $?
done
python3 tools/pmc_traffic.py $O/c2_FETCH_SIZE/b_counter_collection.csv $O/c2_WRITE_SIZE/b_counter_collection.csv $O/pmc_traffic_swin_t_1024.json > $O/c2_top.txt || exit 1
rm -rf $O/c2_FETCH_SIZE $O/c2_WRITE_SIZE
head -8 $O/c2_top.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py --no-cpu-baseline > $O/trace.log 2>&1 || exit $?
cp $O/trace/bench_kernel_stats.csv $O/kernel_stats.csv
rm -f $O/trace/bench_kernel_trace.csv
cp $O/pmc_traffic_swin_t_1024.json profiles/pmc_traffic_swin_t_1024.json
timeout -k 10 500 python3 bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-400
python3 -c "import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); print(json.dumps(d['roofline'])); print(json.dumps(d.get('cpu_baseline')))"
