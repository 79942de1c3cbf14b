# default dispatch (fb for bf16 N > 64) vs the round-4 backward: tests + winbench C2/C3/C5
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5w5
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "window_attention" tests/test_gpu_fp8.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for fb in 0 1; do
  VS_WIN_BWD_FB=$fb timeout -k 10 300 python3 -u tools/winbench.py --configs C2,C3,C5 --iters 10 > $O/bench_fb$fb.log 2>&1 || exit $?
done
( echo "# tools/winbench.py, VS_WIN_BWD_FB=0 (round-4 backward) then 1 (default: fb for bf16 N > 64)"; grep bwd $O/bench_fb0.log; echo; grep bwd $O/bench_fb1.log ) > $O/ab.txt
grep "sum over" $O/ab.txt
