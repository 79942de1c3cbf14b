#!/bin/bash
# Round-4 GPU call: the full -m gpu suite (-s: the parity tests' printed ratios land in the
# log) with per-test durations, then the default bench line without the CPU legs.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread \
    --durations=40 > gpurun_out/r4/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4/gpu_tests.log
grep -E "bf16 step|FAILED" gpurun_out/r4/gpu_tests.log | cut -c1-400
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-parity > gpurun_out/r4/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r4/bench.log | cut -c1-300
