#!/bin/bash
# Round 5: fused step - smoke (fp64 oracle), line-search L-BFGS on GPU, phase stamps, PMC passes,
# discovery diagnosis (reference parametrization)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5s2}
mkdir -p $O
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
grep smoke $O/smoke.log
timeout -k 10 300 python -u -m pytest tests/test_lbfgs_wolfe.py -x -v -s -m gpu --timeout 250 --timeout-method thread > $O/pytest_wolfe.log 2>&1 || { tail -30 $O/pytest_wolfe.log; exit 1; }
grep -E "WOLFE|passed|failed" $O/pytest_wolfe.log
timeout -k 10 200 python -u tools/fused_step_timing.py > $O/timing.txt 2>&1 || { tail -10 $O/timing.txt; exit 1; }
cat $O/timing.txt
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 10 --warmup 2 --min-warmup-s 0 --no-l2"
i=0
for G in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
         "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex "tdq_fused_step|jet_bwd_bf3|jet_fwd_bf3" -d $R/$O/pmc$i --output-format csv -- $B > $R/$O/pmc$i.log 2>&1 || { echo "pmc fail $i"; tail -3 $R/$O/pmc$i.log; exit 1; }
done
cd $R && python tools/pmc_summary.py $O > $O/pmc_summary.txt && cat $O/pmc_summary.txt
timeout -k 10 400 python -u tools/discovery_diag.py --seeds 0 1 2 --iters 10000 --out $O/disc_bf16.json > $O/disc_bf16.log 2>&1 || { tail -20 $O/disc_bf16.log; exit 1; }
cat $O/disc_bf16.log | cut -c1-600
timeout -k 10 300 python -u tools/discovery_diag.py --seeds 0 --iters 10000 --precision fp32 --out $O/disc_fp32.json > $O/disc_fp32.log 2>&1 || { tail -20 $O/disc_fp32.log; exit 1; }
cat $O/disc_fp32.log | cut -c1-600
