#!/bin/bash
# round 6: L-BFGS graphs queued ahead of the GPU (TDQ_LBFGS_DEPTH: 0 = the whole poll batch and the
# next) - ms/iteration
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
export TDQ_LBFGS_HOSTPROF=1
O=gpurun_out/r6cb
mkdir -p $O
for D in 0 1 2 4 0 1 2; do
  TDQ_LBFGS_DEPTH=$D timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 > $O/l$D.log 2>&1 || { tail -5 $O/l$D.log; exit 1; }
  echo "depth $D $(tail -1 $O/l$D.log | grep -o '"ms_per_iter": [0-9.]*') $(tail -2 $O/l$D.log | head -1)" | tee -a $O/depth.txt
done
