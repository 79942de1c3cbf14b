#!/bin/bash
# C4 (MaskDINO Swin-L 1024^2) graph-replayed step breakdown.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4/c4p
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/t -o b -- python3 bench.py --arch maskdino --model swin_l --no-cpu-baseline --no-parity --kernel-timing 0 --steps 3 --warmup 3 > $O/t.log 2>&1 || exit $?
python3 tools/step_breakdown.py $O/t/b_kernel_trace.csv 70 > $O/step_c4.txt || exit $?
rm -rf $O/t
head -60 $O/step_c4.txt | cut -c1-170
