#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -v tests/test_gpu_tgemm.py tests/test_gpu_fp8.py -k "row or mlp_fp8 or dgrad or linears" -s --timeout 250 > $O/fp8b_tests.log 2>&1
tail -2 $O/fp8b_tests.log
grep -E "FAILED|Error" $O/fp8b_tests.log | head -20 | cut -c1-300
bash tools/r5/c5ab.sh
