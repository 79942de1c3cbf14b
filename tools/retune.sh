#!/bin/bash
# Re-tune the vendor-GEMM table (PyTorch TunableOp over hipBLASLt/rocBLAS) for the bench
# configs on the GPU box, then time C2 with the new table and the shipped one.  TunableOp
# inserts the device ordinal into the file name ("%d" here), so the shipped table is
# seeded as tunableop0.csv and only shapes it lacks are tuned.  When it wins, copy
# gpurun_out/tune/tunableop0.csv over vision-instance-seg_amd/visionseg/tuning/tunableop_mi355x.csv.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/tune
mkdir -p $O
cp vision-instance-seg_amd/visionseg/tuning/tunableop_mi355x.csv $O/tunableop0.csv || exit 1
T="PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop%d.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5"
for cfg in "c2|" "c3|--model swin_b" "c4|--arch maskdino --model swin_l" "c5|--model swin_l --size 1536"; do
  name=${cfg%%|*}; args=${cfg#*|}
  env $T timeout -k 10 400 python3 bench.py $args --gemm-tuning tune --no-cpu-baseline --no-parity --graphs 0 \
      --kernel-timing 0 --steps 2 --warmup 1 > $O/tune_$name.log 2>&1 || { echo "tune $name failed"; exit 1; }
  echo "tuned $name: $(grep -c . $O/tunableop0.csv) table lines"
done
VS_GEMM_TABLE=$O/tunableop0.csv timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity > $O/bench_new.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity > $O/bench_old.log 2>&1 || exit 1
echo "new: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_new.log)  old: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_old.log)"
