#!/bin/bash
# Round 4: PMC counters of the high-order kernels in the AC-baseline step (one counter group per pass)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4pmchi
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --problem ac-baseline --steps 10 --warmup 2 --min-warmup-s 0 --no-l2"
i=0
for G in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex "jet_hi" -d $R/$O/pmc$i --output-format csv -- $B > $R/$O/pmc$i.log 2>&1 || { echo "pmc fail $i"; tail -3 $R/$O/pmc$i.log; exit 1; }
done
cd $R && python tools/pmc_summary.py $O > $O/pmc_summary.txt && head -80 $O/pmc_summary.txt
