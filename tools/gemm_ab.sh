#!/bin/bash
# A/B of vendor GEMM selection for the bench step (each run under its own time limit).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gemm_ab
mkdir -p $O
run() { # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 python3 $R/bench.py --steps 5 --warmup 3 --no-cpu-baseline --kernel-timing 0 > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/$name.log)"
  return $rc
}
run default && \
run rocblas TORCH_BLAS_PREFER_HIPBLASLT=0 && \
run tunableop PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop_results%d.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5
