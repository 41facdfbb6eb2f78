#!/bin/bash
# round 6: J partial sums folded into the loss (one phase + barrier fewer) vs HEAD (worktree _ab), same box
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r6ag
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused_kernels.py tests/test_fused_step.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|Error" $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u tools/det_check.py > $O/det.log 2>&1 || { tail -5 $O/det.log; exit 1; }
grep distinct $O/det.log | cut -c1-120
for rep in 1 2; do
  for D in $R $R/_ab; do
    (cd $D && timeout -k 10 200 python -u bench.py --steps 2000 --warmup 200 --no-l2 > $O/b.log 2>&1 && timeout -k 10 200 python -u tools/obj_bench.py --reps 300 > $O/obj.log 2>&1) || { tail -5 $O/b.log $O/obj.log; exit 1; }
    echo "$(basename $D) step $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)  obj $(grep -o "\"us_per_eval\": [0-9.]*" $O/obj.log | tail -1)"
  done
done
