#!/bin/bash
# Round-6 profile set from the repo root: graph-replayed C2 step trace + breakdown, rocprofv3
# kernel stats of the default bench command, PMC FETCH_SIZE / WRITE_SIZE passes of eager steps
# (each pass its own run) summarised per kernel into profiles/pmc_traffic_swin_t_1024.json's format
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${OUT:-r6w}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/graph -o bench -- python3 bench.py --no-cpu-baseline --no-parity --kernel-timing 0 --steps 4 --warmup 3 > $O/graph.log 2>&1 || exit $?
python3 tools/step_breakdown.py $O/graph/bench_kernel_trace.csv 90 > $O/breakdown.txt || exit $?
rm -f $O/graph/bench_kernel_trace.csv
head -8 $O/breakdown.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o bench -- python3 bench.py --no-cpu-baseline > $O/stats.log 2>&1 || exit $?
tail -1 $O/stats.log | cut -c1-300
rm -f $O/stats/bench_kernel_trace.csv
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/$c -o b -- python3 bench.py --no-cpu-baseline --no-parity --graphs 0 --steps 3 --warmup 2 > $O/$c.log 2>&1 || exit $?
done
python3 tools/pmc_traffic.py $O/FETCH_SIZE/b_counter_collection.csv $O/WRITE_SIZE/b_counter_collection.csv $O/pmc_traffic_swin_t_1024.json > $O/pmc_top.txt || exit 1
rm -rf $O/FETCH_SIZE $O/WRITE_SIZE
head -12 $O/pmc_top.txt
