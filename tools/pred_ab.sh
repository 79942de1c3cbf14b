# one test, repeated in separate processes (run-to-run stability; debug aid)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${AB_TEST:-tests/test_gpu_train_parity.py::test_bf16_training_step_vs_oracle}
for i in $(seq 1 ${AB_N:-3}); do
  timeout -k 10 300 python -u -m pytest -q -s --timeout 250 --timeout-method thread $T > gpurun_out/ab_$i.log 2>&1; echo "run $i rc=$?"; grep "${AB_GREP:-bf16 step}" gpurun_out/ab_$i.log | cut -c1-330
done
