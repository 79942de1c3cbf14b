#!/bin/bash
# C2 bench A/B on one box: deferred grouped weight gradients on/off, DMA spread on/off
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5n
mkdir -p $O
for cfg in "0 0" "1 0" "1 1" "0 1" "1 0"; do
  set -- $cfg
  VS_DEFER_WGRAD=$1 VS_WGRAD_SPREAD=$2 timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-parity > $O/b_$1$2.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads([l for l in open('$O/b_$1$2.log') if l.startswith('{')][-1]); print('defer=$1 spread=$2', d['ms_per_step'], d['value'])"
done
