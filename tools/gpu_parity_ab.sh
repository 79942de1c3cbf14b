#!/bin/bash
# bf16 training-step parity statistics with the small-token kernels on / off (per-parameter dumps)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pab
mkdir -p $O
for s in 1 0; do
  VS_PARITY_DUMP=$O/dump_$s.json VS_SMALL_LINEAR_FUSED=$s timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -k "bf16_training_step_vs_oracle" tests/test_gpu_train_parity.py > $O/p_$s.log 2>&1
  echo "fused=$s rc=$?"
done
