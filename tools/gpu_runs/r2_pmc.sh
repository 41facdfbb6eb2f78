#!/bin/bash
# PMC passes over the jet kernels of the current build (one counter group per rocprofv3 run).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TDQ_RUN:-r2pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 10 --warmup 2 --no-l2 --precision ${PREC:-bf16}"
i=0
for G in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
         "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex "jet_" -d $O/pmc$i --output-format csv -- $B > $O/pmc$i.log 2>&1 || { echo "pmc fail $i"; tail -3 $O/pmc$i.log; exit 1; }
done
cd $R && python tools/pmc_summary.py $O
