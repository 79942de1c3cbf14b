#!/bin/bash
# Round evidence in one GPU call (run from the repo root on the box): the C2 profile set
# (tools/profile_round.sh), the other BASELINE configs' per-GPU bench lines, and a PMC
# traffic pair for C5 so its bench line carries its own traffic.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/all
mkdir -p $O
bash tools/profile_round.sh || exit $?
python tools/pmc_traffic.py gpurun_out/round/fetch/b_counter_collection.csv gpurun_out/round/write/b_counter_collection.csv gpurun_out/round/pmc.json > gpurun_out/round/pmc_top.txt || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch5 -o b -- python3 bench.py --model swin_l --size 1536 --no-cpu-baseline --no-parity --graphs 0 --steps 2 --warmup 1 > $O/fetch5.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write5 -o b -- python3 bench.py --model swin_l --size 1536 --no-cpu-baseline --no-parity --graphs 0 --steps 2 --warmup 1 > $O/write5.log 2>&1 || exit $?
python tools/pmc_traffic.py $O/fetch5/b_counter_collection.csv $O/write5/b_counter_collection.csv profiles/pmc_traffic_swin_l_1536.json > $O/pmc5_top.txt || exit $?
timeout -k 10 300 python3 bench.py --model swin_b --no-cpu-baseline --no-parity --steps 5 > $O/c3.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --arch maskdino --model swin_l --no-cpu-baseline --steps 5 > $O/c4.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --model swin_l --size 1536 --no-cpu-baseline --no-parity --steps 5 > $O/c5_bf16.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --model swin_l --size 1536 --attn-fp8 --no-cpu-baseline --no-parity --steps 5 > $O/c5_fp8.log 2>&1 || exit $?
echo done
