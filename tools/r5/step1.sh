# Linear / GEMM tests, then the default C2 bench line and an A/B without the streaming GEMM
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s1
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tgemm.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 bench.py --no-cpu-baseline --no-parity > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-200
VS_TGEMM_STREAM_ROWS=0 VS_TGEMM_STREAM_GELU=0 timeout -k 10 500 python3 bench.py --no-cpu-baseline --no-parity > $O/bench_nostream.log 2>&1 || exit $?
tail -1 $O/bench_nostream.log | cut -c1-200
