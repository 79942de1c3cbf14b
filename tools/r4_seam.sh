#!/bin/bash
# Round-4 training-seam throughput on mixed-aspect COCO-format data (tools/seam_bench.py).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/seam_bench.py --images 96 --iters 160 --timed 60 --workers 12 \
    --modes auto,exact > gpurun_out/r4/seam_bench.log 2>&1
rc=$?
grep '"tool"' gpurun_out/r4/seam_bench.log | cut -c1-600
tail -3 gpurun_out/r4/seam_bench.log
exit $rc
