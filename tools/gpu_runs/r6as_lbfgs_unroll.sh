#!/bin/bash
# round 6: L-BFGS iterations per captured graph (TDQ_LBFGS_UNROLL) - ms per iteration
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6as
mkdir -p $O
for U in 8 16 32 4 8 16; do
  TDQ_LBFGS_UNROLL=$U timeout -k 10 200 python -u tools/prof_lbfgs.py --iters 3000 > $O/l.log 2>&1 || { tail -5 $O/l.log; exit 1; }
  echo "unroll $U $(tail -1 $O/l.log | grep -o "\"ms_per_iter\": [0-9.]*")"
done
