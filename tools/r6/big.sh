#!/bin/bash
# token GEMM 256 x 256 tile on/off for the plain (EPI 0) products: forward shapes + step A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6y
mkdir -p $O
for v in 1 0; do
  echo "== VS_TGEMM_BIG=$v"
  VS_TGEMM_BIG=$v timeout -k 10 300 python3 -u tools/tgemm_bench.py --configs C2 --iters 20 2>&1 | grep -v amdgpu.ids | grep "stage3\|stage4\|forward" | cut -c1-150 || exit 1
done
for i in 1 2 3; do
  for v in 1 0; do
    VS_TGEMM_BIG=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity > $O/b$v$i.log 2>&1 || exit $?
    python3 -c "
import json
d=json.loads([l for l in open('$O/b$v$i.log') if l.startswith('{')][-1]); print('big=$v', d['value'], d['ms_per_step'])"
  done
done
