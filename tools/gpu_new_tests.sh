cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -s tests/test_gpu_fp8.py tests/test_gpu_configs.py::test_c5_swin_l_1536_fp8_step_and_logits > gpurun_out/r3_fp8_tests.log 2>&1 || { tail -5 gpurun_out/r3_fp8_tests.log; exit 1; }
tail -2 gpurun_out/r3_fp8_tests.log
timeout -k 10 300 python tools/winbench.py --configs C5 > gpurun_out/r3_winbench_c5.txt 2>&1 || exit $?
grep "sum over" gpurun_out/r3_winbench_c5.txt
timeout -k 10 300 python bench.py --model swin_l --size 1536 --attn-fp8 --no-cpu-baseline --no-parity --steps 5 > gpurun_out/r3_bench_c5_fp8.log 2>&1 || exit $?
tail -1 gpurun_out/r3_bench_c5_fp8.log | cut -c1-200
timeout -k 10 300 python bench.py --model swin_l --size 1536 --no-cpu-baseline --no-parity --steps 5 > gpurun_out/r3_bench_c5_bf16.log 2>&1 || exit $?
tail -1 gpurun_out/r3_bench_c5_bf16.log | cut -c1-200
