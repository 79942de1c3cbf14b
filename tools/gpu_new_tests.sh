cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 60 ./tools/micro/mfma_scale_probe > gpurun_out/r3_mfma_scale_probe.txt 2>&1
timeout -k 10 300 python tools/msda_bar_bisect.py > gpurun_out/r3_msda_bar_bisect.txt 2>&1 || exit $?
cat gpurun_out/r3_msda_bar_bisect.txt
timeout -k 10 200 python tools/lnbench.py > gpurun_out/r3_lnbench.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -s tests/test_gpu_fp8.py tests/test_gpu_train_parity.py tests/test_gpu_optim.py tests/test_gpu_model.py tests/test_gpu_configs.py > gpurun_out/r3_new_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3_new_tests.log; exit $rc
