# window-attention backward at C5: timing split (VS_WIN_BWD_VAR debug instances) + SQ counters
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5w
mkdir -p $O
timeout -k 10 300 python3 -u tools/winbench.py --configs C5 --iters 10 --variants 0,1,2,4,8,9,6,3 > $O/split.log 2>&1 || exit $?
grep "stage1\|stage2" $O/split.log | grep bwd
WIN_CFG=C5 O2=$O timeout -k 10 600 bash tools/win_pmc.sh > $O/pmc.log 2>&1 || exit $?
cp gpurun_out/winpmc/summary.txt $O/sq_c5.txt
