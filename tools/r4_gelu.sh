#!/bin/bash
# Round-4 GPU call: GELU backward with the one-exp erf (act_bwd_colsum) -- op tests, C2 and C5 lines.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -k "activation or gelu" --timeout 120 --timeout-method thread > $O/gelu_tests.log 2>&1
rc=$?; tail -2 $O/gelu_tests.log; grep -E "^FAILED" $O/gelu_tests.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity --steps 10 > $O/c2_gelu.log 2>&1 || exit $?
tail -1 $O/c2_gelu.log | cut -c1-200
timeout -k 10 400 python3 bench.py --model swin_l --size 1536 --no-cpu-baseline --no-parity --steps 5 > $O/c5_gelu.log 2>&1 || exit $?
tail -1 $O/c5_gelu.log | cut -c1-200
