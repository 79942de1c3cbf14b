#!/bin/bash
# Round-4 GPU call: op census of one C2 training step (aten copies / casts / adds / sums by
# call site), then the training-seam throughput on mixed-aspect COCO-format data.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 300 python3 tools/op_census.py > $O/op_census.txt 2>&1 || exit $?
tail -5 $O/op_census.txt
bash tools/r4_seam.sh
