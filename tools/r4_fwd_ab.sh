#!/bin/bash
# Round-4 GPU call: per-shape token-GEMM forward dispatch -- its tests, the predictor test,
# then C2 bench lines with the dispatch (default) and without (VS_TGEMM_FWD=0), twice
# interleaved, then the profiled step breakdown.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O/pf
timeout -k 10 400 python -u -m pytest tests/test_gpu_tgemm.py tests/test_gpu_model.py -m gpu -q -s --timeout 300 \
    --timeout-method thread -k "dispatch or predictor_bf16 or bf16_vs_f64 or graph" > $O/fwd_tests.log 2>&1
rc=$?
tail -2 $O/fwd_tests.log
grep -E "^FAILED|predictor bf16" $O/fwd_tests.log | cut -c1-300
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
B="python3 bench.py --no-cpu-baseline --no-parity"
for i in 1 2; do
  timeout -k 10 300 $B > $O/c2_fwd1_$i.log 2>&1 || exit $?
  tail -1 $O/c2_fwd1_$i.log | cut -c1-200
  VS_TGEMM_FWD=0 timeout -k 10 300 $B > $O/c2_fwd0_$i.log 2>&1 || exit $?
  tail -1 $O/c2_fwd0_$i.log | cut -c1-200
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pf/f1 -o bench -- python3 bench.py --no-cpu-baseline --no-parity --kernel-timing 0 --steps 4 --warmup 3 > $O/pf/f1.log 2>&1 || exit $?
python3 tools/step_breakdown.py $O/pf/f1/bench_kernel_trace.csv 70 > $O/pf/breakdown_f1.txt || exit $?
head -8 $O/pf/breakdown_f1.txt
