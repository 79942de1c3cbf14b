#!/bin/bash
# fused decoder self-attention input projections: parity tests, model tests, C2 bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/qkv
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -k "small_linear or self_attn_in_proj or decoder_layer" tests/test_gpu_ops.py > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_train_parity.py > $O/model.log 2>&1 || exit $?
tail -1 $O/model.log
for s in 1 0 1 0; do
  VS_SMALL_LINEAR_FUSED=$s timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity --steps 20 > $O/bench_$s.log 2>&1 || exit $?
  echo "small_fused=$s $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$s.log)"
done
