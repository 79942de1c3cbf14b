# HBM traffic per kernel (FETCH_SIZE / WRITE_SIZE, one rocprofv3 pass each) of eager
# steady-state training steps at C2 and C5, summarised on the box (tools/pmc_traffic.py
# keeps only the dispatches after the second optimiser step: no MIOpen Find kernels)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pmc
mkdir -p $O
for cfg in c2 c5; do
  if [ $cfg = c2 ]; then A="--no-cpu-baseline --no-parity"; J=pmc_traffic_swin_t_1024.json; else A="--model swin_l --size 1536 --no-cpu-baseline --no-parity"; J=pmc_traffic_swin_l_1536.json; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/${cfg}_$c -o b -- python3 bench.py $A --graphs 0 --steps 3 --warmup 2 > $O/${cfg}_$c.log 2>&1 || exit $?
  done
  python3 tools/pmc_traffic.py $O/${cfg}_FETCH_SIZE/b_counter_collection.csv $O/${cfg}_WRITE_SIZE/b_counter_collection.csv $O/$J > $O/${cfg}_top.txt || exit 1
  rm -rf $O/${cfg}_FETCH_SIZE $O/${cfg}_WRITE_SIZE
  head -5 $O/${cfg}_top.txt
done
