#!/bin/bash
# Round-4 GPU call: kernel traces of the C5 bf16 and fp8-Linear steps (graph-replayed),
# per-kernel sums of the last step of each (tools/step_breakdown.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4/c5p
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-parity --model swin_l --size 1536 --kernel-timing 0 --steps 3 --warmup 3"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/bf16 -o b -- $B > $O/bf16.log 2>&1 || exit $?
python3 tools/step_breakdown.py $O/bf16/b_kernel_trace.csv 400 > $O/step_bf16.txt || exit $?
rm -rf $O/bf16
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/lfp8 -o b -- $B --linear-fp8 > $O/lfp8.log 2>&1 || exit $?
python3 tools/step_breakdown.py $O/lfp8/b_kernel_trace.csv 400 > $O/step_lfp8.txt || exit $?
rm -rf $O/lfp8
head -8 $O/step_bf16.txt; head -8 $O/step_lfp8.txt
