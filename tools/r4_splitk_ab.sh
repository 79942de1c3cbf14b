#!/bin/bash
# C2 A/B: manual split-K weight gradients (default) vs the library GEMM over the whole
# token axis (VS_SPLITK_MIN_TOKENS huge: hipBLASLt's own stream-K kernels), twice each.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-parity"
for i in 1 2; do
  timeout -k 10 300 $B > $O/c2_sk1.log 2>&1 || exit $?
  echo "split-K   $(tail -1 $O/c2_sk1.log | cut -c1-150)"
  VS_SPLITK_MIN_TOKENS=1000000000 timeout -k 10 300 $B > $O/c2_sk0.log 2>&1 || exit $?
  echo "library   $(tail -1 $O/c2_sk0.log | cut -c1-150)"
done
