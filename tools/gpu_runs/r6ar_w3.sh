#!/bin/bash
# round 6: bf16x3 objective - weight fragments issued before the barrier in front of each GEMM (A/B: -DFZ3_LOAD_AT_GEMM)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6ar
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_kernels.py -m gpu -q -x -s --timeout 300 --timeout-method thread -k bf16x3 > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|Error|FUSED_FP64" $O/pytest.log | head -30; exit 1; }
grep -E "FUSED_FP64|passed" $O/pytest.log | cut -c1-160
timeout -k 10 200 python -u tools/det_check.py bf16x3 > $O/det.log 2>&1 || { tail -5 $O/det.log; exit 1; }
grep distinct $O/det.log | cut -c1-120
for D in "" "-DFZ3_LOAD_AT_GEMM" "" "-DFZ3_LOAD_AT_GEMM"; do
  TDQ_FUSED_STEP_DEFINES="$D" timeout -k 10 200 python -u tools/obj_bench.py --reps 300 > $O/obj.log 2>&1 || { tail -5 $O/obj.log; exit 1; }
  echo "[$D] obj $(grep -o "\"us_per_eval\": [0-9.]*" $O/obj.log | tail -1)"
done
timeout -k 10 200 python -u tools/prof_lbfgs.py --iters 3000 > $O/lbfgs.log 2>&1 || { tail -5 $O/lbfgs.log; exit 1; }
tail -1 $O/lbfgs.log
