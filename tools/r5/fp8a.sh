#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -v tests/test_gpu_tgemm.py tests/test_gpu_maskdino.py -k "row or mlp_fp8 or dgrad or factor_mask" -s --timeout 200 > $O/fp8a_tests.log 2>&1
tail -3 $O/fp8a_tests.log
grep -E "fp8 rows|FAILED|mlp fp8" $O/fp8a_tests.log | cut -c1-300
timeout -k 10 300 python3 tools/r5/scaled_mm_probe.py > $O/scaled_mm_probe2.log 2>&1
cat $O/scaled_mm_probe2.log | cut -c1-330
