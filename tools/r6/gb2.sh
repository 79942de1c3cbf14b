#!/bin/bash
# activation-backward epilogue on the 128 x 128 tile with early pre loads: tgemm tests + A/B bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6x
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_tgemm.py > $O/tgemm.log 2>&1 || { tail -30 $O/tgemm.log; exit 1; }
tail -1 $O/tgemm.log
timeout -k 10 200 python3 -u tools/r6/gb_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/ab_bench.sh r6x/ab 3
