#!/bin/bash
# HBM traffic of the msda backward kernels (column vs tile) at the C2 encoder shape:
# separate FETCH_SIZE / WRITE_SIZE passes over tools/kbench.py (each kernel's last half of
# dispatches = the "smooth" offset set), summarised by tools/pmc_traffic.py.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4/msda_pmc
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o k -- python3 tools/kbench.py --only msda --msda-modes col,prod --iters 4 > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o k -- python3 tools/kbench.py --only msda --msda-modes col,prod --iters 4 > $O/write.log 2>&1 || exit $?
F=$(find $O/fetch -name "*counter_collection.csv" | head -1)
W=$(find $O/write -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py "$F" "$W" $O/traffic.json | grep -i msda
