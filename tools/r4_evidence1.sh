#!/bin/bash
# Round-4 evidence, call 1 of 2: tools/profile_round.sh (the full default C2 bench line,
# kernel trace + stats of the graph run and of an eager run, FETCH_SIZE / WRITE_SIZE
# passes), summarised on the box (kernel stats, step breakdowns, PMC JSON).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
R=gpurun_out/round
bash tools/profile_round.sh || exit $?
python tools/pmc_traffic.py $R/fetch/b_counter_collection.csv $R/write/b_counter_collection.csv $R/pmc.json > $R/pmc_top.txt || exit 1
python tools/step_breakdown.py $R/trace/bench_kernel_trace.csv 60 -3 > $R/step_graph.txt || exit 1
python tools/step_breakdown.py $R/eager/bench_kernel_trace.csv 60 -3 > $R/step_eager.txt || exit 1
cp $R/trace/bench_kernel_stats.csv $R/kernel_stats.csv || exit 1
rm -rf $R/trace $R/eager $R/fetch $R/write
tail -1 $R/bench.log | cut -c1-300
head -12 $R/pmc_top.txt
echo done
