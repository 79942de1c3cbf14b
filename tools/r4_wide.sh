#!/bin/bash
# Round-4 GPU call: the 4-wave 128 x 128-per-wave token GEMM layout (VS_TGEMM_WIDE=1) --
# token GEMM tests with it, then the microbench at C5 with and without it.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tgemm.py -m gpu -q -s --timeout 200 --timeout-method thread \
    -k "mlp_fp8 or dgrad_modes" > $O/tgemm_mlp_tests.log 2>&1 || { tail -5 $O/tgemm_mlp_tests.log; exit 1; }
tail -1 $O/tgemm_mlp_tests.log
VS_TGEMM_WIDE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_tgemm.py -m gpu -q --timeout 200 --timeout-method thread \
    > $O/tgemm_wide_tests.log 2>&1
rc=$?
tail -2 $O/tgemm_wide_tests.log
grep -E "^FAILED" $O/tgemm_wide_tests.log | head
[ $rc -ne 0 ] && exit $rc
for w in 1 0; do
  VS_TGEMM_WIDE=$w timeout -k 10 300 python3 -u tools/tgemm_bench.py --configs C5 --iters 20 > $O/tgemm_wide$w.txt 2>&1 || exit $?
  echo "== wide=$w"; grep -E "C5 stage[234] (qkv|fc1|fc2)|per step" $O/tgemm_wide$w.txt | sed 's/ TF\/s)/)/g' | cut -c1-200
done
# C4 (MaskDINO Swin-L 1024^2) A/B of this round's switches
B="python3 bench.py --arch maskdino --model swin_l --no-cpu-baseline --no-parity --steps 5"
for v in "" "VS_TGEMM_FWD=0" "VS_MSDA_COL=0" "VS_WIN_XCD=0"; do
  env $v timeout -k 10 300 $B > $O/c4_ab.log 2>&1 || exit $?
  echo "C4 [$v] $(tail -1 $O/c4_ab.log | cut -c1-140)"
done
B="python3 bench.py --no-cpu-baseline --no-parity --model swin_l --size 1536 --steps 5"
for v in "" "VS_TGEMM_WIDE=1"; do
  env $v timeout -k 10 300 $B --linear-fp8 > $O/c5_lfp8_ab.log 2>&1 || exit $?
  echo "C5 linear-fp8 [$v] $(tail -1 $O/c5_lfp8_ab.log | cut -c1-140)"
done
