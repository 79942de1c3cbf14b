#!/bin/bash
# Round-4 evidence, call 2 of 2: C3 / C4 / C5 bench lines, the C5 PMC pair, the C5 step
# breakdown.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/all
mkdir -p $O
timeout -k 10 300 python3 bench.py --model swin_b --no-cpu-baseline --no-parity --steps 5 > $O/c3.log 2>&1 || exit $?
tail -1 $O/c3.log | cut -c1-200
timeout -k 10 300 python3 bench.py --arch maskdino --model swin_l --no-cpu-baseline --steps 5 > $O/c4.log 2>&1 || exit $?
tail -1 $O/c4.log | cut -c1-200
timeout -k 10 300 python3 bench.py --model swin_l --size 1536 --no-cpu-baseline --no-parity --steps 5 > $O/c5_bf16.log 2>&1 || exit $?
tail -1 $O/c5_bf16.log | cut -c1-200
timeout -k 10 300 python3 bench.py --model swin_l --size 1536 --attn-fp8 --no-cpu-baseline --no-parity --steps 5 > $O/c5_fp8.log 2>&1 || exit $?
tail -1 $O/c5_fp8.log | cut -c1-200
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch5 -o b -- python3 bench.py --model swin_l --size 1536 --no-cpu-baseline --no-parity --graphs 0 --steps 2 --warmup 1 > $O/fetch5.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write5 -o b -- python3 bench.py --model swin_l --size 1536 --no-cpu-baseline --no-parity --graphs 0 --steps 2 --warmup 1 > $O/write5.log 2>&1 || exit $?
python tools/pmc_traffic.py $O/fetch5/b_counter_collection.csv $O/write5/b_counter_collection.csv $O/pmc_swin_l_1536.json > $O/pmc5_top.txt || exit 1
rm -rf $O/fetch5 $O/write5
echo done
