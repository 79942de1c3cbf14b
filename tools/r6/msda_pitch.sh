#!/bin/bash
# MSDA column backward W pitch: kbench (old tree / new tree, interleaved twice), msda tests, C2 step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-msda_pitch}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k msda > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  VS_ROOT=$PWD/ab_old timeout -k 10 200 python3 tools/kbench.py --only msda --msda-modes col --iters 30 > $O/old$i.log 2>&1 || exit $?
  timeout -k 10 200 python3 tools/kbench.py --only msda --msda-modes col --iters 30 > $O/new$i.log 2>&1 || exit $?
done
grep -h msda_bwd $O/old1.log $O/new1.log $O/old2.log $O/new2.log
bash tools/ab_bench.sh ${1:-msda_pitch}/ab 3
