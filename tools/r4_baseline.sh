#!/bin/bash
# Round-4 first GPU call: the full -m gpu suite with per-test durations, then the bf16
# training-step parity test verbose (its printed ratios), then the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
    --durations=40 > gpurun_out/r4/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4/gpu_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_parity.py -m gpu -q -s --timeout 250 \
    --timeout-method thread -k bf16 > gpurun_out/r4/bf16_parity.log 2>&1 || exit $?
grep "bf16 step" gpurun_out/r4/bf16_parity.log
timeout -k 10 400 python bench.py --no-cpu-baseline --no-parity > gpurun_out/r4/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r4/bench.log | cut -c1-300
