#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6t
mkdir -p $O
timeout -k 10 400 python3 tools/op_census.py > $O/census.txt 2>&1 || { tail -20 $O/census.txt; exit 1; }
echo ok
