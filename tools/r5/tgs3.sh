# input-gradient GEMMs at the C2 shapes: streaming kernel allowed (default) vs tile kernel only
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5tgs3
mkdir -p $O
timeout -k 10 300 python3 -u tools/r5/wgrad_ab.py --dgrad-only > $O/dg.log 2>&1 || exit $?
VS_TGEMM_STREAM_ROWS=0 timeout -k 10 300 python3 -u tools/r5/wgrad_ab.py --dgrad-only > $O/dg_tile.log 2>&1 || exit $?
paste -d'\n' <(grep dgrad $O/dg_tile.log) <(grep dgrad $O/dg.log)
