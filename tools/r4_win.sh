#!/bin/bash
# Round-4 window-attention backward: the window / fp8 tests, then winbench attribution of
# the multi-window backward (VS_WIN_BWD_DBG bits: 1 no phase-1 math, 2 no phase-2 math,
# 4 no global loads, 8 no bin updates) and the round-3 kernel (VS_WIN_BWD_MW=0).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fp8.py -m gpu -q \
    -k "window" --timeout 200 --timeout-method thread > gpurun_out/r4/win_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4/win_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for d in 0 1 2 3 4 8; do
  VS_WIN_BWD_DBG=$d timeout -k 10 120 python tools/winbench.py --configs C5 --iters 10 > gpurun_out/r4/wb_dbg$d.txt 2>&1 || exit $?
  echo "dbg $d: $(grep 'stage1.*bf16.*window_attn_bwd ' gpurun_out/r4/wb_dbg$d.txt | awk '{print $7}') ms (C5 stage1 bwd)"
done
VS_WIN_BWD_MW=0 timeout -k 10 120 python tools/winbench.py --configs C5 --iters 10 > gpurun_out/r4/wb_fa.txt 2>&1 || exit $?
echo "fa: $(grep 'stage1.*bf16.*window_attn_bwd ' gpurun_out/r4/wb_fa.txt | awk '{print $7}') ms"
