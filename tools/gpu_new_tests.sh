cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python tools/fp8_debug.py > gpurun_out/r3_fp8_debug.txt 2>&1; cat gpurun_out/r3_fp8_debug.txt | grep -v "by query"
timeout -k 10 1100 python -u -m pytest -v --timeout 300 --timeout-method thread -s tests -m gpu > gpurun_out/r3_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3_gpu_tests.log; exit $rc
