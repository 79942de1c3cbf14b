#!/bin/bash
# Round-4 token GEMM: correctness tests, then the microbenchmark at the C2 / C5 shapes.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gpu_tgemm.py -m gpu -q -s --timeout 120 --timeout-method thread \
    > gpurun_out/r4/tgemm_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4/tgemm_tests.log
grep -E "^FAILED|Error" gpurun_out/r4/tgemm_tests.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u tools/tgemm_bench.py --configs C2,C5 --iters 20 > gpurun_out/r4/tgemm_bench.txt 2>&1
rc=$?
cat gpurun_out/r4/tgemm_bench.txt | cut -c1-330
exit $rc
