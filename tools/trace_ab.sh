#!/bin/bash
# Kernel traces of the bench step for two environment settings (AB_A / AB_B), for
# tools/step_breakdown.py comparisons.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/trace_ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
env $AB_A timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/A -o t -- python3 $R/bench.py --no-cpu-baseline --steps 6 --warmup 3 > $O/A.log 2>&1 || exit 1
env $AB_B timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/B -o t -- python3 $R/bench.py --no-cpu-baseline --steps 6 --warmup 3 > $O/B.log 2>&1 || exit 1
