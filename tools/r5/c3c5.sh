#!/bin/bash
# round-5 tree: C3 (swin_b), C4 (swin_l maskdino, 300 queries), C5 (swin_l 1536^2) bf16, C5 fp8 Linears + attention
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5c
mkdir -p $O
A="--no-cpu-baseline --no-parity --steps 5 --warmup 3"
run() {
  timeout -k 10 500 python3 bench.py $A "$@" > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  grep '^{' $O/b.log | tail -1 >> $O/c3c5.jsonl
  echo "$* $(grep '^{' $O/b.log | tail -1 | cut -c1-140)"
}
run --model swin_b
run --model swin_l --arch maskdino --queries 300
run --model swin_l --size 1536
run --model swin_l --size 1536 --linear-fp8 --attn-fp8
