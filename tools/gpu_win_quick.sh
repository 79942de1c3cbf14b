# window-attention op tests + stage-sum microbench (quick A/B after a kernel change)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -k "window or fp8" tests/test_gpu_ops.py tests/test_gpu_fp8.py > gpurun_out/win_quick.log 2>&1 || { tail -30 gpurun_out/win_quick.log; exit 1; }
tail -1 gpurun_out/win_quick.log
timeout -k 10 300 python tools/winbench.py --configs ${WIN_CFG:-C2,C3,C5} > gpurun_out/winbench.txt 2>&1 || exit $?
grep "sum over" gpurun_out/winbench.txt
