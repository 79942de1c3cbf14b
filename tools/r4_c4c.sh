#!/bin/bash
# Round-4 GPU call: MaskDINO tests (factored matcher + mask losses), the C4 line, profile.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_maskdino.py tests/test_gpu_configs.py -m gpu -q -s --timeout 300 \
    --timeout-method thread -k "maskdino or c4 or C4 or factor" > $O/maskdino_tests3.log 2>&1
rc=$?
tail -2 $O/maskdino_tests3.log
grep -E "^FAILED|maskdino (fp32|bf16)" $O/maskdino_tests3.log | cut -c1-200
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --arch maskdino --model swin_l --no-cpu-baseline --no-parity --steps 5 > $O/c4_fac2.log 2>&1 || exit $?
tail -1 $O/c4_fac2.log | cut -c1-200
bash tools/r4_c4_prof.sh > /dev/null 2>&1 || exit $?
head -40 $O/c4p/step_c4.txt | cut -c1-150
