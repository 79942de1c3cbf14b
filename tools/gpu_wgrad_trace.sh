#!/bin/bash
# kernel-trace stats of the C2 bench with the token-split small_linear wgrad kernel on / off
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/wgt
for s in 1 0; do
  VS_SMALL_WGRAD_SPLIT=$s timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wgt/t$s -o b -- python3 bench.py --no-cpu-baseline --no-parity --steps 5 > gpurun_out/wgt/b$s.log 2>&1 || exit $?
  grep -i "small_wgrad" gpurun_out/wgt/t$s/b_kernel_stats.csv > gpurun_out/wgt/stats_$s.txt
  rm -f gpurun_out/wgt/t$s/b_kernel_trace.csv
done
