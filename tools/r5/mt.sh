#!/bin/bash
# token-Linear threshold A/B: VS_SPLITK_MIN_TOKENS 16384 (default) vs 4096 (Swin stage 4 and 4900-token windows on the token path)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5mt
mkdir -p $O
for m in 4096 16384 4096 16384; do
  VS_SPLITK_MIN_TOKENS=$m timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-parity > $O/bench$m.log 2>&1 || exit $?
  echo "min_tokens=$m $(tail -1 $O/bench$m.log | cut -c90-160)"
done
