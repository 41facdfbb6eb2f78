#!/bin/bash
# round 6: L-BFGS dots pass with 16 elements per thread round (LB_R 8 -> 16: one load round per
# chunk at the AC-SA size) - device L-BFGS tests, ms/iteration, phase stamps
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6bu
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lbfgs_device.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for F in a b c; do
  timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 > $O/l$F.log 2>&1 || { tail -5 $O/l$F.log; exit 1; }
  echo "$(tail -1 $O/l$F.log | grep -o '"ms_per_iter": [0-9.]*')"
done
timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 --ts > $O/ts.log 2>&1 || { tail -5 $O/ts.log; exit 1; }
tail -2 $O/ts.log | head -1
