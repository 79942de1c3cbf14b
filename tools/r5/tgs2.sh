# streaming token GEMM up to K = 384 (one slice): tests + fwd shapes + dgrad A/B at C2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5tgs2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_tgemm.py -k "token_gemm" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/tgemm_bench.py --configs C2 --iters 20 > $O/stream.log 2>&1 || exit $?
grep "stage1" $O/stream.log | cut -c1-200
timeout -k 10 300 python3 -u tools/r5/wgrad_ab.py --quick > $O/wg.log 2>&1 || exit $?
grep "dgrad s1\|dgrad total" $O/wg.log
VS_TGEMM_STREAM_ROWS=0 timeout -k 10 300 python3 -u tools/r5/wgrad_ab.py --quick > $O/wg_tile.log 2>&1 || exit $?
grep "dgrad s1\|dgrad total" $O/wg_tile.log
