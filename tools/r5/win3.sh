# fb backward at C5 stage 1: timing split (fb debug instances) + SQ counters for fa and fb
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5w3
mkdir -p $O
for v in 0 1 2 4 6 3; do
  VS_WIN_BWD_VAR=$v timeout -k 10 120 python3 -u tools/winbench.py --configs C5 --iters 10 > $O/split_$v.log 2>&1 || exit $?
  echo "var $v: $(grep 'stage1' $O/split_$v.log | grep 'bf16' | grep bwd)"
done
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_LEVEL_WAVES GRBM_GUI_ACTIVE"
for fb in 0 1; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    VS_WIN_BWD_FB=$fb timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/fb${fb}_p$i -o w -- python3 tools/r5/win_one.py --iters 3 > $O/fb${fb}_p$i.log 2>&1 || exit $?
  done
  python3 tools/pmc_kernels.py --match win_attn_bwd $O/fb${fb}_p1/w_counter_collection.csv $O/fb${fb}_p2/w_counter_collection.csv $O/fb${fb}_p3/w_counter_collection.csv > $O/sq_fb$fb.txt || exit 1
  rm -rf $O/fb${fb}_p1 $O/fb${fb}_p2 $O/fb${fb}_p3
done
cat $O/sq_fb0.txt $O/sq_fb1.txt
