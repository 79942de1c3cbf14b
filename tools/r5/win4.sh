# fb backward at C5: timing split (debug instances) and the waves-per-EU A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5w4
mkdir -p $O
timeout -k 10 300 python3 -u tools/winbench.py --configs C5 --iters 10 --variants 0,1,2,4,6,3 > $O/split_fb.log 2>&1 || exit $?
grep "stage1" $O/split_fb.log | grep bwd
VS_WIN_BWD_WPE=3 timeout -k 10 300 python3 -u tools/winbench.py --configs C5 --iters 10 > $O/wpe3.log 2>&1 || exit $?
grep "stage1\|stage2\|sum" $O/wpe3.log | grep bwd
