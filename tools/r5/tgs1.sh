# streaming token GEMM: parity tests + C2 shapes (tile kernel vs streaming)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5tgs
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_tgemm.py -k "token_gemm" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
VS_TGEMM_STREAM_ROWS=0 timeout -k 10 300 python3 -u tools/tgemm_bench.py --configs C2 --iters 20 > $O/tile.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/tgemm_bench.py --configs C2 --iters 20 > $O/stream.log 2>&1 || exit $?
grep "stage1\|stage2" $O/tile.log | cut -c1-260
echo ---
grep "stage1\|stage2" $O/stream.log | cut -c1-260
