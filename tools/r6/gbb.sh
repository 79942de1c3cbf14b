#!/bin/bash
# activation-backward dX epilogue: 256 x 256 tile (default) vs 128 x 128 tile for those modes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in 1 0; do
  echo "== VS_TGEMM_GB_BIG=$v"
  VS_TGEMM_GB_BIG=$v timeout -k 10 200 python3 -u tools/r6/gb_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
