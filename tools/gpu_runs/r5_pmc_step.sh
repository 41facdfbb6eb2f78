#!/bin/bash
# Round 5: PMC counters of the one-launch fused step (AC-SA; one counter group per pass)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R

O=gpurun_out/${TAG:-r5pmcstep}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 10 --warmup 2 --min-warmup-s 0 --no-l2"
i=0
for G in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
         "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex "tdq_fused_step" -d $R/$O/pmc$i --output-format csv -- $B > $R/$O/pmc$i.log 2>&1 || { echo "pmc fail $i"; tail -3 $R/$O/pmc$i.log; exit 1; }
done
cd $R && python tools/pmc_summary.py $O > $O/pmc_summary.txt && cat $O/pmc_summary.txt
rm -rf $O/pmc1 $O/pmc2 $O/pmc3
