#!/bin/bash
# Round-4 GPU call: the default bench line (as the driver runs it) at the final tree.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/c2_final_default.log 2>&1 || exit $?
tail -1 $O/c2_final_default.log | cut -c1-300
