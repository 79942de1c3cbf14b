#!/bin/bash
# Round-4 GPU call: token GEMM tests + microbench (LDS-staged epilogue), the Predictor
# bf16-vs-f32 test, then the C5 lines (bf16 / fp8 Linears / fp8 Linears + fp8 attention)
# and C2 with the fused fc1 + GELU (VS_TGEMM_GELU=1) vs without.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tgemm.py tests/test_gpu_model.py -m gpu -q -s --timeout 200 \
    --timeout-method thread -k "tgemm or token_gemm or mx_ or gelu or fp8 or predictor_bf16" > $O/tgemm_tests.log 2>&1
rc=$?
tail -2 $O/tgemm_tests.log
grep -E "^FAILED|predictor bf16" $O/tgemm_tests.log | head
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u tools/tgemm_bench.py --configs C2,C5 --iters 20 > $O/tgemm_bench2.txt 2>&1 || exit $?
grep "per step" $O/tgemm_bench2.txt | cut -c1-300
bash tools/r4_c5.sh
