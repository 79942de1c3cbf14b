# win_attn_bwd_fb: parity tests + C5 / C2 A/B against the round-4 backward
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5w2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "window_attention" tests/test_gpu_fp8.py > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for fb in 0 1; do
  VS_WIN_BWD_FB=$fb timeout -k 10 300 python3 -u tools/winbench.py --configs C5,C2 --iters 10 > $O/bench_fb$fb.log 2>&1 || exit $?
done
grep "bwd" $O/bench_fb0.log | grep -v sum > $O/a.txt; grep "bwd" $O/bench_fb1.log | grep -v sum > $O/b.txt
paste -d'\n' $O/a.txt $O/b.txt
grep "sum over" $O/bench_fb0.log $O/bench_fb1.log | grep bwd
