# SQ counters of the window-attention kernels at C5 / C2 shapes (tools/winbench.py), one
# rocprofv3 pass per counter group (at most 8 SQ counters a pass), summarised on the box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/winpmc
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_LEVEL_WAVES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o w -- python3 tools/winbench.py --configs ${WIN_CFG:-C5,C2} --iters 3 > $O/p$i.log 2>&1 || exit $?
done
python3 tools/pmc_kernels.py --match win_attn $O/p1/w_counter_collection.csv $O/p2/w_counter_collection.csv $O/p3/w_counter_collection.csv > $O/summary.txt || exit 1
rm -rf $O/p1 $O/p2 $O/p3
cat $O/summary.txt | head -120
