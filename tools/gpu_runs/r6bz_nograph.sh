#!/bin/bash
# round 6: the L-BFGS iteration launched eagerly (TDQ_NO_GRAPH=1) vs captured graphs - ms/iteration
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6bz
mkdir -p $O
for K in 0 1 0 1; do
  TDQ_NO_GRAPH=$K timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 > $O/l$K.log 2>&1 || { tail -5 $O/l$K.log; exit 1; }
  echo "no_graph $K lbfgs $(tail -1 $O/l$K.log | grep -o '"ms_per_iter": [0-9.]*')" | tee -a $O/nograph.txt
done
