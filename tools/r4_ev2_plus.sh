#!/bin/bash
# matcher tests after the finalise change, then the C3-C5 evidence set.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gpu_match_factors.py tests/test_gpu_match.py -m gpu -q --timeout 200 \
    --timeout-method thread > gpurun_out/r4/match_tests2.log 2>&1
rc=$?
tail -2 gpurun_out/r4/match_tests2.log
[ $rc -ne 0 ] && exit $rc
bash tools/r4_evidence2.sh
