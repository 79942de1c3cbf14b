#!/bin/bash
# Round profile set (run on the GPU box from the repo root): the full bench line (CPU
# baseline + parity), rocprofv3 kernel trace + stats of the bench command, then
# FETCH_SIZE and WRITE_SIZE passes (eager steps: PMC is collected per dispatch), each
# pass its own run.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/round
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench.log 2> $O/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py --no-cpu-baseline > $O/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/eager -o bench -- python3 bench.py --no-cpu-baseline --graphs 0 > $O/eager.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o b -- python3 bench.py --no-cpu-baseline --graphs 0 --steps 3 --warmup 2 > $O/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o b -- python3 bench.py --no-cpu-baseline --graphs 0 --steps 3 --warmup 2 > $O/write.log 2>&1 || exit $?
echo done
