#!/bin/bash
# eager call-site attribution of the glue kernels (forward frames / backward autograd nodes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6n
mkdir -p $O
timeout -k 10 500 python3 -u tools/torch_prof.py > $O/tprof.txt 2>&1 || exit $?
grep -A70 "glue ops by call site" $O/tprof.txt | cut -c1-230
