#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread -m gpu tests/test_gpu_train_parity.py > $O/tp.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tp.log | cut -c1-600 | head -20; exit 1; }
grep -E "passed|failed|self_attn|mean ratio|p90" $O/tp.log | cut -c1-600 | head -40
