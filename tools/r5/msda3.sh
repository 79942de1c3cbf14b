#!/bin/bash
# msda_bwd column size with the integer W build: 8 x 16 (default) vs 16 x 16 vs 8 x 8
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5m3
mkdir -p $O
timeout -k 10 300 python3 -u tools/kbench.py --only msda --iters 20 --msda-modes col,col16,col8 > $O/kb.log 2>&1 || exit $?
grep -i "bwd" $O/kb.log | cut -c1-200
