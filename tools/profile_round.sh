#!/bin/bash
# Round profile set (run on the GPU box from the repo root): unprofiled bench line,
# rocprofv3 kernel trace + stats of the same command, FETCH_SIZE and WRITE_SIZE passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/round
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py > $O/trace.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o b -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 2 > $O/fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o b -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 2 > $O/write.log 2>&1 || exit $?
echo done
