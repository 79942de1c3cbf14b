#!/bin/bash
# LayerNorm backward partial count at small M: ln_bench old / new twice, then the C2 step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-ln_parts}
mkdir -p $O
for i in 1 2; do
  VS_ROOT=$PWD/ab_old timeout -k 10 200 python3 tools/r6/ln_bench.py > $O/old$i.log 2>&1 || exit $?
  timeout -k 10 200 python3 tools/r6/ln_bench.py > $O/new$i.log 2>&1 || exit $?
done
bash tools/ab_bench.sh ${1:-ln_parts}/ab 3
