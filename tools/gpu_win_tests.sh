# window-attention kernel change: op tests (bf16 / fp8 / fp32, small and large windows, shifted),
# model-level tests through the Swin backbone, then the C5 / C2 stage-sum microbench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -s -k "window or fp8 or swin_t_bf16 or swin_b_c3" tests/test_gpu_ops.py tests/test_gpu_fp8.py tests/test_gpu_model.py > gpurun_out/win_tests.log 2>&1 || { tail -30 gpurun_out/win_tests.log; exit 1; }
tail -2 gpurun_out/win_tests.log
timeout -k 10 300 python tools/winbench.py --configs C2,C3,C5 > gpurun_out/winbench.txt 2>&1 || exit $?
grep "sum over" gpurun_out/winbench.txt
