#!/bin/bash
# Round-4 GPU call: matcher / attention masks from the mask head's factors -- the new
# tests, the criterion / model / training-step parity tests that run through the path,
# then C2 bench lines with the factored masks (default) and without (VS_FACTORED_MASKS=0),
# then the profiled step breakdown of the factored path.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_match_factors.py tests/test_gpu_match.py tests/test_gpu_point_loss.py \
    tests/test_gpu_train_parity.py tests/test_gpu_graphs.py -m gpu -q -s --timeout 300 --timeout-method thread \
    > $O/factors_tests.log 2>&1
rc=$?
tail -3 $O/factors_tests.log
grep -E "^FAILED|match_cost_factors|level mask|bf16 step mean" $O/factors_tests.log | cut -c1-300
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
B="python3 bench.py --no-cpu-baseline --no-parity"
timeout -k 10 300 $B > $O/c2_fact.log 2>&1 || exit $?
tail -1 $O/c2_fact.log | cut -c1-200
VS_FACTORED_MASKS=0 timeout -k 10 300 $B > $O/c2_nofact.log 2>&1 || exit $?
tail -1 $O/c2_nofact.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $O/pf
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/pf/f1 -o bench -- python3 bench.py --no-cpu-baseline --no-parity --kernel-timing 0 --steps 4 --warmup 3 > $O/pf/f1.log 2>&1 || exit $?
python3 tools/step_breakdown.py $O/pf/f1/bench_kernel_trace.csv 70 > $O/pf/breakdown_f1.txt || exit $?
