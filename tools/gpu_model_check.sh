# model-level GPU checks after a model-graph change: model / training-parity / graph tests,
# then the default bench line
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_train_parity.py tests/test_gpu_graphs.py ${EXTRA_TESTS} > gpurun_out/model_check.log 2>&1 || { tail -40 gpurun_out/model_check.log; exit 1; }
tail -1 gpurun_out/model_check.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_check.log 2>&1 || { tail -5 gpurun_out/bench_check.log; exit 1; }
tail -1 gpurun_out/bench_check.log | cut -c1-200
