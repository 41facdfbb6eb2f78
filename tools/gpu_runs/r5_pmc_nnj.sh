#!/bin/bash
# Round 5: PMC of the layered engine's epilogue GEMM (bf16 W512)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5pmcnnj}
mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "lay_nnj|lay_tn2" --output-format csv -d $R/$O/pmc1 -o run -- python3 $R/bench.py --steps 3 --warmup 2 --min-warmup-s 0 --no-l2 --precision bf16 --layers 2,512,512,512,512,1 > $R/$O/p1.log 2>&1 || { tail -5 $R/$O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE FETCH_SIZE --kernel-include-regex "lay_nnj|lay_tn2" --output-format csv -d $R/$O/pmc2 -o run -- python3 $R/bench.py --steps 3 --warmup 2 --min-warmup-s 0 --no-l2 --precision bf16 --layers 2,512,512,512,512,1 > $R/$O/p2.log 2>&1 || { tail -5 $R/$O/p2.log; exit 1; }
cd $R && python tools/pmc_summary.py $O | tee $O/pmc_summary.txt
rm -rf $O/pmc1 $O/pmc2
