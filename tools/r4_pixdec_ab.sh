#!/bin/bash
# Round-4 GPU call: C2 with the 1/4-resolution FPN blocks NCHW (default) vs channels-last
# (VS_PIXDEC_NCHW=0), then the conv kernels of each in a profiled step.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O/pd
B="python3 bench.py --no-cpu-baseline --no-parity"
timeout -k 10 300 $B > $O/c2_pd1.log 2>&1 || exit $?
tail -1 $O/c2_pd1.log | cut -c1-200
VS_PIXDEC_NCHW=0 timeout -k 10 300 $B > $O/c2_pd0.log 2>&1 || exit $?
tail -1 $O/c2_pd0.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
VS_PIXDEC_NCHW=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/pd/p0 -o bench -- python3 bench.py --no-cpu-baseline --no-parity --kernel-timing 0 --steps 4 --warmup 3 > $O/pd/p0.log 2>&1 || exit $?
python3 tools/step_breakdown.py $O/pd/p0/bench_kernel_trace.csv 200 > $O/pd/breakdown_p0.txt || exit $?
grep -iE "conv|igemm|transpose|group_norm|upsample|naive" $O/pd/breakdown_p0.txt | cut -c1-150
