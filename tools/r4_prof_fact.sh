#!/bin/bash
# Graph-replayed C2 step breakdowns with the factored masks (default) and without.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4/pf
mkdir -p $O
for m in 1 0; do
  VS_FACTORED_MASKS=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/f$m -o bench -- python3 bench.py --no-cpu-baseline --no-parity --kernel-timing 0 --steps 4 --warmup 3 > $O/f$m.log 2>&1 || exit $?
  python3 tools/step_breakdown.py $O/f$m/bench_kernel_trace.csv 60 > $O/breakdown_f$m.txt || exit $?
done
echo done
