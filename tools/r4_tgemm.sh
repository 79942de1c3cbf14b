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
[ $rc -ne 0 ] && exit $rc
# window attention: XCD-grouped (window, head) mapping (default) vs the 2-D grid
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fp8.py -m gpu -q \
    -k "window" --timeout 200 --timeout-method thread > gpurun_out/r4/win_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4/win_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for x in 1 0; do
  VS_WIN_XCD=$x timeout -k 10 150 python tools/winbench.py --configs C2,C5 --iters 10 > gpurun_out/r4/wb_xcd$x.txt 2>&1 || exit $?
  echo "== VS_WIN_XCD=$x"; grep -E "window_attn" gpurun_out/r4/wb_xcd$x.txt | cut -c1-160
done
