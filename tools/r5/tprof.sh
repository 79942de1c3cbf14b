#!/bin/bash
# call sites of the step's copies / fills (torch.profiler over 2 eager C2 steps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5tp
mkdir -p $O
timeout -k 10 500 python3 -u tools/torch_prof.py > $O/tprof.txt 2>&1 || exit $?
grep -A46 "by input shape" $O/tprof.txt | cut -c1-330
