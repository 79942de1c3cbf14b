#!/bin/bash
# C4 line with graph capture (the batched factored mask losses), then the graph-replay test.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 300 python3 bench.py --arch maskdino --model swin_l --no-cpu-baseline --no-parity --steps 5 > $O/c4_fac3.log 2>&1 || { tail -5 $O/c4_fac3.log; exit 1; }
tail -1 $O/c4_fac3.log | cut -c1-200
timeout -k 10 500 python -u -m pytest tests/test_gpu_maskdino.py tests/test_gpu_configs.py -m gpu -q --timeout 300 \
    --timeout-method thread -k "maskdino or c4 or C4 or graph" > $O/maskdino_tests5.log 2>&1
rc=$?
tail -2 $O/maskdino_tests5.log
exit $rc
