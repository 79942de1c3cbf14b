#!/bin/bash
# Round-4 GPU call: smoke, the factored-path tests, MaskDINO tests (batched factored mask
# losses), then the C4 line.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_match_factors.py tests/test_gpu_maskdino.py tests/test_gpu_configs.py -m gpu -q -s \
    --timeout 300 --timeout-method thread -k "tiny or maskdino or c4 or C4 or factor" > $O/maskdino_tests4.log 2>&1
rc=$?
tail -2 $O/maskdino_tests4.log
grep -E "^FAILED|maskdino (fp32|bf16)" $O/maskdino_tests4.log | cut -c1-200
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --arch maskdino --model swin_l --no-cpu-baseline --no-parity --steps 5 > $O/c4_fac3.log 2>&1 || exit $?
tail -1 $O/c4_fac3.log | cut -c1-200
