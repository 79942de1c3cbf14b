#!/bin/bash
# Round-4 C5 lines: bf16, fp8 Linears (MX token GEMM), fp8 Linears + fp8 window attention,
# then C2 with the fc1+GELU token GEMM vs without (VS_TGEMM_GELU A/B).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-parity"
timeout -k 10 300 $B --model swin_l --size 1536 --steps 5 > $O/c5_bf16.log 2>&1 || exit $?
tail -1 $O/c5_bf16.log | cut -c1-200
timeout -k 10 300 $B --model swin_l --size 1536 --steps 5 --linear-fp8 > $O/c5_lfp8.log 2>&1 || exit $?
tail -1 $O/c5_lfp8.log | cut -c1-200
timeout -k 10 300 $B --model swin_l --size 1536 --steps 5 --linear-fp8 --attn-fp8 > $O/c5_fp8.log 2>&1 || exit $?
tail -1 $O/c5_fp8.log | cut -c1-200
timeout -k 10 300 $B > $O/c2_base.log 2>&1 || exit $?
tail -1 $O/c2_base.log | cut -c1-200
VS_TGEMM_GELU=1 timeout -k 10 300 $B > $O/c2_gelu.log 2>&1 || exit $?
tail -1 $O/c2_gelu.log | cut -c1-200
