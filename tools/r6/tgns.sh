#!/bin/bash
# token GEMM K-step ring depth (VS_TGEMM_NS = 2: two stages, 2 workgroups / CU; 3 / 4: deeper ring, 1 / CU)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6r
mkdir -p $O
for ns in 2 3 4; do
  echo "== VS_TGEMM_NS=$ns"
  VS_TGEMM_NS=$ns timeout -k 10 300 python3 -u tools/tgemm_bench.py --configs C2 --iters 20 2>&1 | grep -v amdgpu.ids | sed 's/tgemm_fp8.*//' || exit 1
done
