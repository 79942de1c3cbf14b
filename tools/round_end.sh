#!/bin/bash
# Round-end evidence in one GPU call: full -m gpu suite, smoke(), then the C2 profile set
# (default bench line, kernel trace + stats, eager trace, FETCH / WRITE PMC passes).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 660 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -2 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
bash tools/profile_round.sh || exit $?
tail -1 gpurun_out/round/bench.log | cut -c1-300
