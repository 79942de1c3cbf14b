#!/bin/bash
# LayerNorm backward next-row prefetch A/B (VS_LN_BWD_PF): tests, per-shape kernel trace, C2 bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ln4
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "norm" > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
VS_LN_BWD_PF=0 timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "norm" > $O/tests0.log 2>&1 || exit $?
tail -1 $O/tests0.log
for pf in 1 0; do
  VS_LN_BWD_PF=$pf LNB_PARTS=512 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr$pf -o ln -- python3 -u tools/lnbench.py > $O/ln$pf.log 2>&1 || exit $?
  python3 tools/r5/ln_shapes.py $O/tr$pf/ln_kernel_trace.csv > $O/shapes$pf.txt || exit 1
  rm -f $O/tr$pf/ln_kernel_trace.csv
done
paste <(grep ln_bwd $O/shapes1.txt | cut -c1-110) <(grep ln_bwd $O/shapes0.txt | cut -c95-110)
for pf in 1 0 1; do
  VS_LN_BWD_PF=$pf timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-parity > $O/bench$pf.log 2>&1 || exit $?
  echo "pf=$pf $(tail -1 $O/bench$pf.log | cut -c90-200)"
done
