# msda_bwd column kernel timing split (VS_MSDA_DBG instances; results not checked)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5m2
mkdir -p $O
for d in 0 1 2 4 8 15; do
  VS_MSDA_DBG=$d timeout -k 10 300 python3 -u tools/kbench.py --only msda --iters 20 > $O/kb_d$d.log 2>&1 || exit $?
  echo "dbg=$d: $(grep -i 'init col.*bwd\|iid4px col.*bwd' $O/kb_d$d.log | tr '\n' ' ' | cut -c1-250)"
done
