#!/bin/bash
# Round-4 GPU call: C5 bf16 vs fp8 Linears with the dX GEMM on bf16 (VS_FP8_DGRAD=0) and on
# MX fp8 (default), and fp8 Linears + fp8 window attention with the bf16 dX.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-parity --model swin_l --size 1536 --steps 5"
timeout -k 10 300 $B > $O/c5b_bf16.log 2>&1 || exit $?
tail -1 $O/c5b_bf16.log | cut -c1-200
VS_FP8_DGRAD=0 timeout -k 10 300 $B --linear-fp8 > $O/c5b_lfp8_nodg.log 2>&1 || exit $?
tail -1 $O/c5b_lfp8_nodg.log | cut -c1-200
timeout -k 10 300 $B --linear-fp8 > $O/c5b_lfp8.log 2>&1 || exit $?
tail -1 $O/c5b_lfp8.log | cut -c1-200
VS_FP8_DGRAD=0 timeout -k 10 300 $B --linear-fp8 --attn-fp8 > $O/c5b_fp8_nodg.log 2>&1 || exit $?
tail -1 $O/c5b_fp8_nodg.log | cut -c1-200
