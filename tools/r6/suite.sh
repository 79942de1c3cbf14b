#!/bin/bash
# Round-6 GPU call: the full -m gpu suite (no -x: every failure listed), smoke, default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${OUT:-r6v}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
    --durations=30 > $O/gpu_tests_full.log 2>&1
rc=$?
tail -3 $O/gpu_tests_full.log
grep -E "bf16 step mean|FAILED|maskdino bf16" $O/gpu_tests_full.log | cut -c1-400
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-400
exit $rc
