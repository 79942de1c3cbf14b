#!/bin/bash
# Round-6: decoder self-attention kernel tests, training-step parity, C2 bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -s -m gpu tests/test_gpu_self_attn.py > $O/sa_tests.log 2>&1 || { grep -E "self_attn \(|Error|assert" $O/sa_tests.log | cut -c1-400 | head -30; exit 1; }
grep -E "self_attn \(|passed|failed" $O/sa_tests.log | cut -c1-300
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread -m gpu tests/test_gpu_train_parity.py > $O/tp.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tp.log | head -20; tail -5 $O/tp.log; exit 1; }
grep -E "passed|failed|self_attn|mean ratio|p90" $O/tp.log | cut -c1-300 | head -40
timeout -k 10 500 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-300
