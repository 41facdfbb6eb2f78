#!/bin/bash
# round 6: bf16x3 objective under max-ilp - fp64 tests, determinism, objective / L-BFGS timing
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6bb
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_kernels.py tests/test_fused_step.py tests/test_lbfgs_device.py -m gpu -q -x -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|Error" $O/pytest.log | head -30; exit 1; }
grep -E "FUSED_FP64.*bf16x3|passed" $O/pytest.log | cut -c1-160
timeout -k 10 200 python -u tools/det_check.py bf16x3 > $O/det.log 2>&1 || { tail -5 $O/det.log; exit 1; }
grep distinct $O/det.log | cut -c1-120
timeout -k 10 200 python -u tools/obj_bench.py --reps 300 > $O/obj.log 2>&1 || exit 1
grep -o "\"us_per_eval\": [0-9.]*" $O/obj.log | tail -1
timeout -k 10 200 python -u tools/prof_lbfgs.py --iters 3000 > $O/l.log 2>&1 || exit 1
tail -1 $O/l.log | grep -o "\"ms_per_iter\": [0-9.]*"
