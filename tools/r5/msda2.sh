#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -q tests/test_gpu_ops.py -k "msda" --timeout 250 -x > $O/msda_tests.log 2>&1
rc=$?
tail -2 $O/msda_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/kbench.py --only msda --msda-modes col,dst --iters 10 > $O/msda_kbench.log 2>&1
grep -v amdgpu.ids $O/msda_kbench.log | grep bwd
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench_msda2.log 2>&1 || exit $?
tail -1 $O/bench_msda2.log | cut -c1-200
python3 -c "import json;d=json.loads(open('$O/bench_msda2.log').read().strip().splitlines()[-1]);print(d['roofline'])"
