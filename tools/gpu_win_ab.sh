# window-attention op tests with the default kernels, then the stage-sum microbench for
# the online forward (default) and the two-pass forward (VS_WIN_FWD_ONLINE=0)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -k "window or fp8 or column_sum or activation_backward" tests/test_gpu_ops.py tests/test_gpu_fp8.py > gpurun_out/win_quick.log 2>&1 || { tail -30 gpurun_out/win_quick.log; exit 1; }
tail -1 gpurun_out/win_quick.log
timeout -k 10 300 python tools/winbench.py --configs ${WIN_CFG:-C2,C3,C5} > gpurun_out/winbench_online.txt 2>&1 || exit $?
VS_WIN_FWD_ONLINE=0 timeout -k 10 300 python tools/winbench.py --configs ${WIN_CFG:-C2,C3,C5} > gpurun_out/winbench_twopass.txt 2>&1 || exit $?
grep "sum over" gpurun_out/winbench_online.txt | grep fwd
grep "sum over" gpurun_out/winbench_twopass.txt | grep fwd
grep "sum over" gpurun_out/winbench_online.txt | grep bwd
