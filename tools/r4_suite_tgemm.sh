#!/bin/bash
# Round-4 GPU call: token GEMM microbench at the current kernel (C2 / C5 shapes), then the
# full -m gpu suite at this tree.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 300 python3 -u tools/tgemm_bench.py --configs C2,C5 --iters 20 > $O/tgemm_bench3.txt 2>&1 || exit $?
grep "per step" $O/tgemm_bench3.txt | cut -c1-300
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread \
    --durations=30 > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
grep -E "bf16 step mean|FAILED" $O/gpu_tests.log | cut -c1-300
exit $rc
