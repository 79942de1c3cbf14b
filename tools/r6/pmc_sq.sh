#!/bin/bash
# SQ counters (MFMA / VALU / LDS / wait mix) of the hand-written kernels in an eager C2 step
# (bench.py --graphs 0; PMC is collected per dispatch), one rocprofv3 pass per counter
# group (<= 8 SQ counters a pass), summarised per kernel on the box.
#   WHAT=c2 (default) | c5: the C5 step (Swin-L 1536^2, bf16)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
W=${WHAT:-c2}
O=gpurun_out/r6/pmc_$W
mkdir -p $O
A="--no-cpu-baseline --no-parity --graphs 0 --steps 2 --warmup 2"
[ "$W" = c5 ] && A="$A --model swin_l --size 1536"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_LEVEL_WAVES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o b -- python3 bench.py $A > $O/p$i.log 2>&1 || exit $?
done
for k in msda_bwd_col msda_fwd4 token_gemm_kernel token_gemm_stream token_wgrad_kernel win_attn_bwd gn_stats gn_bwd_stats; do
  python3 tools/pmc_kernels.py --match $k $O/p1/b_counter_collection.csv $O/p2/b_counter_collection.csv $O/p3/b_counter_collection.csv
done > $O/summary.txt || exit 1
rm -rf $O/p1 $O/p2 $O/p3
head -c 6000 $O/summary.txt
