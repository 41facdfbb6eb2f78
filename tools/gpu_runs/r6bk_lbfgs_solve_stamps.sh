#!/bin/bash
# round 6 (diagnostic build): stamps around each of the L-BFGS logic's three solve loops
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6bk
mkdir -p $O
timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 --ts > $O/ts.log 2>&1 || { tail -5 $O/ts.log; exit 1; }
tail -2 $O/ts.log
