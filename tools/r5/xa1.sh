# masked cross-attention backward v2 vs v1: parity tests + kbench timings at the decoder shapes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5x1
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "masked_attention" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for ver in 1 2; do
  VS_XATTN_BWD=$ver timeout -k 10 300 python3 -u tools/kbench.py --only xattn --iters 20 > $O/kb_v$ver.log 2>&1 || exit $?
  echo "v$ver"; grep -i "xattn" $O/kb_v$ver.log
done
