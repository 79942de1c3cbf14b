#!/bin/bash
# Round evidence in one GPU call, summarised ON THE BOX so gpurun_out stays under the
# 64 MiB copy-back cap: tools/profile_round.sh (C2 bench line, kernel trace of the graph
# run and of an eager run, FETCH_SIZE / WRITE_SIZE passes), the C5 PMC pair, and the
# C3 / C4 / C5 bench lines.  Raw rocprof CSVs are reduced to the kernel stats, step
# breakdowns and PMC JSON, then deleted.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
R=gpurun_out/round
O=gpurun_out/all
mkdir -p $O
bash tools/profile_round.sh || exit $?
python tools/pmc_traffic.py $R/fetch/b_counter_collection.csv $R/write/b_counter_collection.csv $R/pmc.json > $R/pmc_top.txt || exit 1
python tools/step_breakdown.py $R/trace/bench_kernel_trace.csv 60 -3 > $R/step_graph.txt || exit 1
python tools/step_breakdown.py $R/eager/bench_kernel_trace.csv 60 -3 > $R/step_eager.txt || exit 1
cp $R/trace/bench_kernel_stats.csv $R/kernel_stats.csv || exit 1
rm -rf $R/trace $R/eager $R/fetch $R/write
# C5 warm-up run first: MIOpen's convolution Find results land in the user find-db, so
# the PMC passes below replay the chosen solvers instead of profiling the Find search
timeout -k 10 300 python3 bench.py --model swin_l --size 1536 --no-cpu-baseline --no-parity --graphs 0 --steps 1 --warmup 1 > $O/warm5.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch5 -o b -- python3 bench.py --model swin_l --size 1536 --no-cpu-baseline --no-parity --graphs 0 --steps 2 --warmup 1 > $O/fetch5.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write5 -o b -- python3 bench.py --model swin_l --size 1536 --no-cpu-baseline --no-parity --graphs 0 --steps 2 --warmup 1 > $O/write5.log 2>&1 || exit $?
python tools/pmc_traffic.py $O/fetch5/b_counter_collection.csv $O/write5/b_counter_collection.csv $O/pmc_swin_l_1536.json > $O/pmc5_top.txt || exit 1
rm -rf $O/fetch5 $O/write5
timeout -k 10 120 python3 tools/flops.py --arch maskdino --model swin_l > $O/flops_c4.json 2> $O/flops.err || exit $?
timeout -k 10 120 python3 tools/flops.py --arch mask2former --model swin_t > $O/flops_c2.json 2>> $O/flops.err || exit $?
timeout -k 10 300 python3 bench.py --model swin_b --no-cpu-baseline --no-parity --steps 5 > $O/c3.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --arch maskdino --model swin_l --no-cpu-baseline --steps 5 > $O/c4.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --model swin_l --size 1536 --no-cpu-baseline --no-parity --steps 5 > $O/c5_bf16.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --model swin_l --size 1536 --attn-fp8 --no-cpu-baseline --no-parity --steps 5 > $O/c5_fp8.log 2>&1 || exit $?
# C5 step breakdown (graph-replayed steps under the kernel trace)
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace5 -o b -- python3 bench.py --model swin_l --size 1536 --no-cpu-baseline --no-parity --steps 3 > $O/trace5.log 2>&1 || exit $?
python tools/step_breakdown.py $O/trace5/b_kernel_trace.csv 60 -3 > $O/step_c5.txt || exit 1
rm -rf $O/trace5
du -sh gpurun_out
echo done
