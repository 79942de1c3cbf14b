#!/bin/bash
# Round-4 GPU call: window-attention tests + winbench at C2 after the per-half bias bins of
# the ws-7 backward.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fp8.py -m gpu -q -k "window" --timeout 200 \
    --timeout-method thread > $O/win_tests2.log 2>&1
rc=$?
tail -2 $O/win_tests2.log
grep -E "^FAILED" $O/win_tests2.log | head
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 150 python tools/winbench.py --configs C2 --iters 20 > $O/wb_halfbins.txt 2>&1 || exit $?
grep -E "bf16.*window_attn_bwd" $O/wb_halfbins.txt | cut -c1-160
exit $rc
