cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python tools/fp8_debug.py > gpurun_out/r3_fp8_debug.txt 2>&1; cat gpurun_out/r3_fp8_debug.txt
timeout -k 10 300 python tools/msda_bar_bisect.py > gpurun_out/r3_msda_bar_bisect.txt 2>&1 || exit $?
cat gpurun_out/r3_msda_bar_bisect.txt
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -s "tests/test_gpu_ops.py::test_msda_mfma_backward_vs_binned_and_oracle" "tests/test_gpu_ops.py::test_msda_encoder_shapes_backward_vs_oracle" "tests/test_gpu_ops.py::test_msda_destination_backward_vs_oracle" tests/test_gpu_train_parity.py tests/test_gpu_configs.py > gpurun_out/r3_new_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3_new_tests.log; exit $rc
