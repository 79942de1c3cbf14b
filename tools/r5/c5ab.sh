#!/bin/bash
# C5 (Swin-L 1536^2 bf16) per-GPU step: bf16 vs fp8 Linears (rowwise vendor GEMM) vs + fp8 attention
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5
mkdir -p $O
A="--model swin_l --size 1536 --no-cpu-baseline --no-parity --steps 8 --warmup 3"
for v in "" "--linear-fp8" "--linear-fp8 --attn-fp8"; do
  timeout -k 10 400 python3 bench.py $A $v > $O/c5ab.log 2>&1 || { tail -5 $O/c5ab.log; exit 1; }
  echo "$v $(tail -1 $O/c5ab.log)" | cut -c1-260 | tee -a $O/c5ab.jsonl
done
