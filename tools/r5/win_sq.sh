# SQ counters of the window-attention backward kernels: C5 stage 1 (win_attn_bwd_fb<5>, the
# default, and the round-4 win_attn_bwd_fa<5>) and C2 stage 1 (win_attn_bwd_fa<2>)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5sq
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
run() {  # tag env args
  local tag=$1 envv=$2; shift 2
  local i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    env $envv timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/${tag}_p$i -o w -- python3 tools/r5/win_one.py --iters 3 "$@" > $O/${tag}_p$i.log 2>&1 || return 1
  done
  python3 tools/pmc_kernels.py --match win_attn_bwd $O/${tag}_p1/w_counter_collection.csv $O/${tag}_p2/w_counter_collection.csv $O/${tag}_p3/w_counter_collection.csv > $O/sq_$tag.txt || return 1
  rm -rf $O/${tag}_p1 $O/${tag}_p2 $O/${tag}_p3
}
run c5_fb VS_WIN_BWD_FB=1 || exit 1
run c5_fa VS_WIN_BWD_FB=0 || exit 1
run c2_fa VS_WIN_BWD_FB=1 --bw 5476 --heads 3 --ws 7 --nw 37 || exit 1
for t in c5_fb c5_fa c2_fa; do echo "== $t"; cat $O/sq_$t.txt; done > $O/sq_all.txt
head -5 $O/sq_all.txt
