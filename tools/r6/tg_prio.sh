#!/bin/bash
# token GEMM per-shape times (tools/tgemm_bench.py --configs C2): ab_old/ vs the working tree, twice; step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-tg_prio}
mkdir -p $O
for i in 1 2; do
  VS_ROOT=$PWD/ab_old timeout -k 10 200 python3 tools/tgemm_bench.py --configs C2 > $O/old$i.log 2>&1 || exit $?
  timeout -k 10 200 python3 tools/tgemm_bench.py --configs C2 > $O/new$i.log 2>&1 || exit $?
done
bash tools/ab_bench.sh ${1:-tg_prio}/ab 2
