#!/bin/bash
# Interleaved A/B of two environment settings on one box (box-to-box variance is larger
# than most single changes): AB_A / AB_B hold space-separated VAR=value lists, AB_ROUNDS
# rounds of A then B, each bench run under its own time limit; stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab
mkdir -p $O
ROUNDS=${AB_ROUNDS:-3}
STEPS=${AB_STEPS:-20}
run() { # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 $R/bench.py --steps $STEPS --warmup 5 --no-cpu-baseline > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/$name.log)" | tee -a $O/summary.txt
  return $rc
}
for i in $(seq 1 $ROUNDS); do
  run A$i $AB_A VS_AB_SIDE=A || exit 1
  run B$i $AB_B VS_AB_SIDE=B || exit 1
done
