#!/bin/bash
# tile-kernel activation-backward epilogue with the pre-activation loads one K-step earlier:
# token GEMM tests, the act-bwd dX microbench (old tree vs new), C2 step A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${OUT:-pre_early}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_tgemm.py > $O/tgemm.log 2>&1 || { tail -30 $O/tgemm.log; exit 1; }
tail -1 $O/tgemm.log
VS_ROOT=$PWD/ab_old timeout -k 10 200 python3 tools/r6/gb_bench.py > $O/gb_old.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/r6/gb_bench.py > $O/gb_new.log 2>&1 || exit 1
bash tools/ab_bench.sh ${OUT:-pre_early}/ab 3
