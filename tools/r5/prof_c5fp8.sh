#!/bin/bash
# kernel trace of the C5 step with fp8 Linears (rowwise vendor GEMM) + the C2 op census
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5f8 -o b -- python3 bench.py --model swin_l --size 1536 --no-cpu-baseline --no-parity --steps 4 --warmup 3 --linear-fp8 > $O/trace_c5f8.log 2>&1 || exit $?
python3 tools/step_breakdown.py $O/trace_c5f8/b_kernel_trace.csv 60 -3 > $O/step_c5_fp8.txt 2>&1
head -50 $O/step_c5_fp8.txt | cut -c1-180
rm -rf $O/trace_c5f8
timeout -k 10 300 python3 tools/op_census.py > $O/op_census_c2.txt 2>&1
head -100 $O/op_census_c2.txt | cut -c1-150
