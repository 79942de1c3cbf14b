#!/bin/bash
# SQ / TCC counters of token_wgrad at the C2 stage-3 fc1 shape (one rocprofv3 pass per group)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5h
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_LEVEL_WAVES GRBM_GUI_ACTIVE"
P4="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  VS_WGRAD_CFG=0 timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o b -- python3 tools/r5/wg_pmc.py > $O/p$i.log 2>&1 || exit $?
done
python3 tools/pmc_kernels.py --match token_wgrad_kernel $O/p1/b_counter_collection.csv $O/p2/b_counter_collection.csv $O/p3/b_counter_collection.csv $O/p4/b_counter_collection.csv > $O/summary.txt 2>&1
cat $O/summary.txt
