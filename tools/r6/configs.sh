#!/bin/bash
# C3 / C4 / C5 per-GPU bench lines on the round-6 tree (one GPU call, each run time-limited)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${OUT:-r6cfg}
mkdir -p $O
timeout -k 10 300 python3 bench.py --model swin_b --no-cpu-baseline --no-parity --steps 5 > $O/c3.log 2>&1 || exit $?
grep '^{' $O/c3.log | tail -1 | cut -c1-120
timeout -k 10 300 python3 bench.py --arch maskdino --model swin_l --queries 300 --no-cpu-baseline --no-parity --steps 5 > $O/c4.log 2>&1 || exit $?
grep '^{' $O/c4.log | tail -1 | cut -c1-120
timeout -k 10 300 python3 bench.py --model swin_l --size 1536 --no-cpu-baseline --no-parity --steps 5 > $O/c5_bf16.log 2>&1 || exit $?
grep '^{' $O/c5_bf16.log | tail -1 | cut -c1-120
timeout -k 10 300 python3 bench.py --model swin_l --size 1536 --linear-fp8 --no-cpu-baseline --no-parity --steps 5 > $O/c5_lfp8.log 2>&1 || exit $?
grep '^{' $O/c5_lfp8.log | tail -1 | cut -c1-120
