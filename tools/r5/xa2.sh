# per-kernel times of the masked cross-attention ops at the decoder shapes (kbench --only xattn)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5x2
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o x -- python3 tools/kbench.py --only xattn --iters 20 > $O/kb.log 2>&1 || exit $?
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r5x2/tr/x_kernel_trace.csv')))
from collections import defaultdict
d=defaultdict(list)
for r in rows:
    n=r['Kernel_Name']
    if 'xattn' not in n: continue
    key=(n.split('(')[0][-40:], r.get('Grid_Size_X', r.get('Grid_Size','')))
    d[key].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
for k,v in sorted(d.items()):
    v=sorted(v)
    print(f"{k[0]:42s} grid={k[1]:>8s} n={len(v):4d} median={v[len(v)//2]:8.2f} us")
PY
rm -f $O/tr/x_kernel_trace.csv
