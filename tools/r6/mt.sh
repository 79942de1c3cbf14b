#!/bin/bash
# token-path threshold A/B on one box, interleaved: VS_SPLITK_MIN_TOKENS 4096 (default) vs 16384
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6g
mkdir -p $O
for t in 4096 16384 4096 16384 4096 16384; do
  VS_SPLITK_MIN_TOKENS=$t timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity --kernel-timing 0 --steps 20 > $O/b_$t.log 2>&1 || exit $?
  echo "min_tokens=$t $(tail -1 $O/b_$t.log | cut -c1-150)"
done
