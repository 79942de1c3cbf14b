#!/bin/bash
# token_wgrad per-shape times (tools/r5/wgrad_ab.py --quick): ab_old/ vs the working tree, twice
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-wg_prio}
mkdir -p $O
for i in 1 2; do
  (cd ab_old && timeout -k 10 200 python3 ../tools/r5/wgrad_ab.py --quick > ../$O/old$i.log 2>&1) || exit $?
  timeout -k 10 200 python3 tools/r5/wgrad_ab.py --quick > $O/new$i.log 2>&1 || exit $?
done
