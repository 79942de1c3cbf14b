#!/bin/bash
# Quick GPU check of one area: pytest -k "$1" over the op tests, then the C2 bench step time.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q -k "$1" --timeout 120 --timeout-method thread > gpurun_out/t_q.log 2>&1
tail -2 gpurun_out/t_q.log
grep -E "^E |FAILED" gpurun_out/t_q.log | head -5
timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/b1.log 2>&1 || exit $?
tail -1 gpurun_out/b1.log | grep -o '"ms_per_step": [0-9.]*'
