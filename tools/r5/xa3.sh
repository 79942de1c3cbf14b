# window / masked attention tests after the WinGeom division change + xattn blocks-per-workgroup sweep
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5x3
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "window or masked_attention" tests/test_gpu_fp8.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for nb in 2 4 8; do
  VS_XATTN_BLOCKS=$nb timeout -k 10 300 python3 -u tools/kbench.py --only xattn --iters 20 > $O/kb_b$nb.log 2>&1 || exit $?
  echo "blocks $nb: $(grep 'S=16384.*bwd' $O/kb_b$nb.log)"
done
timeout -k 10 300 python3 -u tools/winbench.py --configs C2,C5 --iters 10 > $O/win.log 2>&1 || exit $?
grep "sum over" $O/win.log
