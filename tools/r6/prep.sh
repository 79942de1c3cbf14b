#!/bin/bash
# vectorised MSDA prologue (P = 4): op tests, model / parity tests, A/B bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6z
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "prep or msda" > $O/ops.log 2>&1 || { tail -30 $O/ops.log; exit 1; }
tail -1 $O/ops.log
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_train_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_bench.sh r6z/ab 3
python3 - <<'PY'
import json
for s in ("old", "new"):
    d = json.loads([l for l in open(f"gpurun_out/r6z/ab/{s}1.log") if l.startswith("{")][-1])
    k = d["kernels"]
    print(s, {n: (k[n]["mean_ms"], k[n]["gbs"]) for n in k if "prep" in n})
PY
