# msda_bwd column kernel: integer W build vs f32 turns -- tests + kbench A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5m1
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "msda" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for w in 0 1 0 1; do
  VS_MSDA_WINT=$w timeout -k 10 300 python3 -u tools/kbench.py --only msda --iters 20 > $O/kb_w$w.log 2>&1 || exit $?
  echo "wint=$w: $(grep -i 'bwd' $O/kb_w$w.log | head -3 | tr '\n' ' ' | cut -c1-300)"
done
