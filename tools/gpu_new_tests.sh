cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 60 ./tools/micro/mfma_scale_probe > gpurun_out/r3_mfma_scale_probe.txt 2>&1; cat gpurun_out/r3_mfma_scale_probe.txt
timeout -k 10 300 python tools/kbench.py --only msda --msda-modes mfma,syncbar --iters 20 > gpurun_out/r3_kbench_msda.txt 2>&1 || exit $?
grep msda_bwd gpurun_out/r3_kbench_msda.txt
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -s tests/test_gpu_train_parity.py tests/test_gpu_optim.py "tests/test_gpu_ops.py::test_msda_mfma_backward_vs_binned_and_oracle" "tests/test_gpu_ops.py::test_msda_encoder_shapes_backward_vs_oracle" "tests/test_gpu_ops.py::test_msda_destination_backward_vs_oracle" "tests/test_gpu_ops.py::test_msda_carry_backward_vs_oracle" tests/test_gpu_model.py > gpurun_out/r3_new_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3_new_tests.log; exit $rc
