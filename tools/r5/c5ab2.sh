#!/bin/bash
# C5 on the round-5 tree: bf16 vs fp8 Linears vs fp8 Linears + fp8 attention, interleaved twice
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5c5
mkdir -p $O
A="--model swin_l --size 1536 --no-cpu-baseline --no-parity --steps 5 --warmup 3"
for r in 1 2; do
  for v in "" "--linear-fp8" "--linear-fp8 --attn-fp8"; do
    timeout -k 10 500 python3 bench.py $A $v > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "[$v] $(grep '^{' $O/b.log | tail -1)" >> $O/c5ab.txt
    echo "[$v] $(grep '^{' $O/b.log | tail -1 | cut -c60-130)"
  done
done
