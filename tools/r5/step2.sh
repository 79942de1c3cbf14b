# C2 step A/B on one box: dgrad rule r5a (earlier) vs r5b (default)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tgemm.py > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
for r in r5b r5a r5b; do
  VS_TGEMM_DGRAD_RULE=$r timeout -k 10 500 python3 bench.py --no-cpu-baseline --no-parity > $O/bench_$r.log 2>&1 || exit $?
  echo "$r $(tail -1 $O/bench_$r.log | cut -c1-160)"
done
