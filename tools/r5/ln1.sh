#!/bin/bash
# LayerNorm backward workgroup-cap A/B at the Swin stage shapes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ln
mkdir -p $O
LNB_PARTS=256,512,1024,2048 timeout -k 10 300 python3 -u tools/lnbench.py > $O/ln.log 2>&1 || exit $?
cat $O/ln.log
