#!/bin/bash
# LayerNorm kernels per shape (kernel trace of tools/lnbench.py at the default workgroup cap)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ln3
mkdir -p $O
LNB_PARTS=512 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o ln -- python3 -u tools/lnbench.py > $O/ln.log 2>&1 || exit $?
python3 tools/r5/ln_shapes.py $O/tr/ln_kernel_trace.csv > $O/shapes.txt || exit 1
rm -f $O/tr/ln_kernel_trace.csv
cat $O/shapes.txt
