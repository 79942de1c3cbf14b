#!/bin/bash
# LayerNorm fwd/bwd microbenchmark at the C2 shapes: backward variants (VS_LN_BWD2: 0 = one-pass,
# 1/2 = two-pass packed, U = 1/2) x max chunks per lane (VS_LN_BWD_KMAX) x workgroups
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in 0 1 2; do
  for k in 4 2 1; do
    for p in 512 1024; do
      echo "== VS_LN_BWD2=$v KMAX=$k PARTS=$p"
      VS_LN_BWD2=$v VS_LN_BWD_KMAX=$k VS_LN_BWD_PARTS=$p timeout -k 10 200 python3 -u tools/r6/ln_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done
