#!/bin/bash
# round 6: weight-image L2 warm-up in both fused kernels: tests, objective time, L-BFGS ms/iter
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6x
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_kernels.py -m gpu -q -x -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|Error|FUSED_FP64" $O/pytest.log | head -30; exit 1; }
grep -E "FUSED_FP64|passed" $O/pytest.log | cut -c1-200
timeout -k 10 200 python -u tools/obj_bench.py --reps 300 > $O/obj.log 2>&1 || { tail -5 $O/obj.log; exit 1; }
grep us_per_eval $O/obj.log | tail -2
timeout -k 10 200 python -u tools/prof_lbfgs.py --iters 3000 > $O/lbfgs.log 2>&1 || { tail -5 $O/lbfgs.log; exit 1; }
tail -2 $O/lbfgs.log
