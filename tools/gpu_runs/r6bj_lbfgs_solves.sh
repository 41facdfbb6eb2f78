#!/bin/bash
# round 6: L-BFGS logic with operands of the triangular solves preloaded into registers; phase stamps of the
# dots + logic kernel
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6bj
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lbfgs_device.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for F in 1 1; do
  TDQ_LBFGS_FUSED=$F timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 > $O/l$F.log 2>&1 || { tail -5 $O/l$F.log; exit 1; }
  tail -1 $O/l$F.log
done
timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 --ts > $O/ts.log 2>&1 || { tail -5 $O/ts.log; exit 1; }
tail -2 $O/ts.log
