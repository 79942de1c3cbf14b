#!/bin/bash
# C3 / C4 / C5 per-GPU bench lines at the current tree (one GPU call, each run time-limited).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/cfg
mkdir -p $O
timeout -k 10 300 python3 bench.py --model swin_b --no-cpu-baseline --no-parity --steps 5 > $O/c3.log 2>&1 || exit $?
tail -1 $O/c3.log | cut -c1-160
timeout -k 10 300 python3 bench.py --arch maskdino --model swin_l --no-cpu-baseline --steps 5 > $O/c4.log 2>&1 || exit $?
tail -1 $O/c4.log | cut -c1-160
timeout -k 10 300 python3 bench.py --model swin_l --size 1536 --no-cpu-baseline --no-parity --steps 5 > $O/c5_bf16.log 2>&1 || exit $?
tail -1 $O/c5_bf16.log | cut -c1-160
timeout -k 10 300 python3 bench.py --model swin_l --size 1536 --attn-fp8 --no-cpu-baseline --no-parity --steps 5 > $O/c5_fp8.log 2>&1 || exit $?
tail -1 $O/c5_fp8.log | cut -c1-160
