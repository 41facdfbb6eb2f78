#!/bin/bash
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 10 --warmup 2 --no-l2"
i=0
for G in "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES" \
         "SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $G --kernel-include-regex "jet_" -d $R/gpurun_out/pmcc$i --output-format csv -- $B > $R/gpurun_out/pmcc$i.log 2>&1 || { echo "fail $i"; tail -3 $R/gpurun_out/pmcc$i.log; exit 1; }
done
echo done
