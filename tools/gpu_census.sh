#!/bin/bash
# op census of one eager C2 step + graph-replay kernel breakdown of the current tree
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pg
timeout -k 10 300 python3 tools/op_census.py > gpurun_out/op_census.txt 2>&1 || exit $?
bash tools/prof_graph.sh && rm -rf gpurun_out/pg/graph
